/*
 * sanitize_host.c — the host-side C of the checksum path under ASan + UBSan
 * ("ASan/UBSan on the host C, plus a bounds-checked CPU
 * restatement"). Built and run on the CPU by tests/test_sanitize.py:
 *
 *   gcc -fsanitize=address,undefined -fno-sanitize-recover=all -Iinclude -Ioracle \
 *       tests/c/sanitize_host.c tcp_amd/csrc/scalar_dropin.c oracle/csum_oracle.c -lpthread
 *
 * Every buffer is an exact-size heap allocation, so a read or write one byte
 * past a segment, packet or region end is an ASan error; UBSan catches bad
 * shifts and signed overflow. Checks:
 *   1. the scalar drop-ins (tcpcsum_pseudo / tcpcsum_continue, the library's
 *      replacements for context.c:104-145) equal the oracle on random segments
 *      of every length 0..2100 and random start values, plus Appendix A KATs;
 *   2. the oracle's wire restatement (context.c:169-209) fills, then verifies to
 *      zero, packets laid back to back in an exact-size region (IHL 5..7, IPv4
 *      header checksum included), and the drop-ins verify every filled segment;
 *   3. the oracle's segment builder (context.c:150-213) writes packets that
 *      verify, into an exact-size output region.
 * Exit status 0 = every check passed.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "tcpcsum.h"

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

static int fails = 0;
#define CHECK(cond, ...)                           \
    do {                                           \
        if (!(cond)) {                             \
            fprintf(stderr, "FAIL: " __VA_ARGS__); \
            fputc('\n', stderr);                   \
            ++fails;                               \
        }                                          \
    } while (0)

static uint16_t htons16(unsigned v) { return (uint16_t) (((v & 0xffu) << 8) | ((v >> 8) & 0xffu)); }

static void check_scalar(void) {
    const char z2[2] = {0, 0};
    const char z3[3] = {0, 0, 0x7f};
    CHECK(tcpcsum_continue(0, z2, 2) == 0xffff, "KAT 00 00");
    CHECK(tcpcsum_continue(0, z3, 3) == 0xff80, "KAT 00 00 7f");
    for (int len = 0; len <= 2100; ++len) {
        char *p = (char *) malloc(len ? (size_t) len : 1);
        for (int i = 0; i < len; ++i) p[i] = (char) rnd();
        for (int r = 0; r < 3; ++r) {
            const unsigned long ss = (unsigned long) (rnd() & (r == 0 ? 0xffffu : 0xffffffffu));
            CHECK(tcpcsum_continue(ss, p, len) == oracle_csum_continue(ss, p, len), "continue len %d", len);
        }
        const uint32_t sa = (uint32_t) rnd(), da = (uint32_t) rnd();
        const uint16_t lb = (uint16_t) rnd();
        CHECK(tcpcsum_pseudo(sa, da, lb) == oracle_pseudo(sa, da, lb), "pseudo");
        free(p);
    }
}

/* n packets back to back in an exact-size region; fill, then verify */
static void check_wire(int n) {
    unsigned *ihl = (unsigned *) malloc((size_t) n * sizeof(unsigned));
    uint64_t *off = (uint64_t *) malloc((size_t) n * sizeof(uint64_t));
    size_t total = 0;
    for (int i = 0; i < n; ++i) {
        ihl[i] = 5 + (unsigned) (rnd() % 3);   /* IP options sometimes */
        const size_t tot = ihl[i] * 4u + 24u + (size_t) (rnd() % 1457);
        off[i] = total;
        total += tot;
    }
    uint8_t *region = (uint8_t *) malloc(total);
    for (size_t b = 0; b < total; ++b) region[b] = (uint8_t) rnd();
    for (int i = 0; i < n; ++i) {
        uint8_t *ip = region + off[i];
        const size_t tot = (i + 1 < n ? off[i + 1] : total) - off[i];
        ip[0] = (uint8_t) (0x40 | ihl[i]);
        ip[2] = (uint8_t) (tot >> 8);
        ip[3] = (uint8_t) tot;
        ip[9] = 6;
    }
    uint16_t *out = (uint16_t *) malloc((size_t) n * sizeof(uint16_t));
    uint8_t *st = (uint8_t *) malloc((size_t) n);
    oracle_ipv4_batch(region, off, (uint64_t) n, 65535u, 0 | 2, out, st);
    for (int i = 0; i < n; ++i) CHECK(st[i] == 0, "fill status %d = %d", i, st[i]);
    oracle_ipv4_batch(region, off, (uint64_t) n, 65535u, 1 | 2, out, st);
    for (int i = 0; i < n; ++i) CHECK(st[i] == 0 && out[i] == 0, "verify %d: st %d out %04x", i, st[i], out[i]);
    for (int i = 0; i < n; ++i) {   /* the scalar drop-ins agree on every filled segment */
        const uint8_t *ip = region + off[i];
        const unsigned th = (ip[0] & 15u) * 4u, tot = ((unsigned) ip[2] << 8) | ip[3];
        uint32_t sa, da;
        memcpy(&sa, ip + 12, 4);
        memcpy(&da, ip + 16, 4);
        const unsigned tl = tot - th;
        CHECK(tcpcsum_continue(tcpcsum_pseudo(sa, da, htons16(tl)), (const char *) ip + th, (int) tl) == 0,
              "drop-in verify %d", i);
    }
    free(st);
    free(out);
    free(region);
    free(off);
    free(ihl);
}

static void check_builder(int n) {
    oracle_txseg_t *segs = (oracle_txseg_t *) calloc((size_t) n, sizeof(oracle_txseg_t));
    size_t ptotal = 0, ototal = 0;
    for (int i = 0; i < n; ++i) {
        const unsigned len = (unsigned) (rnd() % 1457);
        segs[i].payload_off = ptotal;
        segs[i].out_off = ototal;
        segs[i].saddr_be = (uint32_t) rnd();
        segs[i].daddr_be = (uint32_t) rnd();
        segs[i].seq = (uint32_t) rnd();
        segs[i].ack = (uint32_t) rnd();
        segs[i].sport = 4000;
        segs[i].dport = 45001;
        segs[i].len = (uint16_t) len;
        segs[i].flags = (uint8_t) (1 | ((rnd() & 1) ? 16 : 0));
        ptotal += len;
        ototal += 44u + ((segs[i].flags & 16) ? len : 0u);
    }
    uint8_t *payload = (uint8_t *) malloc(ptotal ? ptotal : 1);
    for (size_t b = 0; b < ptotal; ++b) payload[b] = (uint8_t) rnd();
    uint8_t *outp = (uint8_t *) malloc(ototal);
    uint16_t *checks = (uint16_t *) malloc((size_t) n * sizeof(uint16_t));
    oracle_tx_build(payload, segs, (uint64_t) n, outp, 1, checks);
    uint64_t *off = (uint64_t *) malloc((size_t) n * sizeof(uint64_t));
    for (int i = 0; i < n; ++i) off[i] = segs[i].out_off;
    uint16_t *out = (uint16_t *) malloc((size_t) n * sizeof(uint16_t));
    uint8_t *st = (uint8_t *) malloc((size_t) n);
    oracle_ipv4_batch(outp, off, (uint64_t) n, 65535u, 1 | 2, out, st);
    for (int i = 0; i < n; ++i) CHECK(st[i] == 0 && out[i] == 0, "built packet %d: st %d out %04x", i, st[i], out[i]);
    free(st);
    free(out);
    free(off);
    free(checks);
    free(outp);
    free(payload);
    free(segs);
}

int main(void) {
    check_scalar();
    check_wire(3000);
    check_builder(3000);
    if (fails) {
        fprintf(stderr, "%d failures\n", fails);
        return 1;
    }
    printf("sanitize_host: ok\n");
    return 0;
}
