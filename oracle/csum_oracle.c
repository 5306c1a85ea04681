/*
 * csum_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the uNetworking/tcp TCP checksum path, used only as
 * the checker in tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg. The product library (tcp_amd/libtcpcsum.so) never links or calls it.
 *
 * Reference functions restated (paths relative to /root/reference):
 *   oracle_pseudo        <- context.c:104-119  getPseudoHeaderSum
 *   oracle_csum_continue <- context.c:121-145  csum_continue
 *   oracle_ipv4_batch    <- context.c:169-209  (IPv4/TCP framing + the call at :208)
 *                           and loop.c:44-47 (tot_len -> iov_len) for the wire layout
 * Generator and digests: SURVEY.md Appendix B.
 *
 * Parity pin: tests/test_oracle.py checks this file against SURVEY.md
 * Appendix A KATs and Appendix B digests (both produced by the reference's own
 * code) and against tests/golden/ fixtures.
 */
#include "oracle.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/ip.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---- context.c:104-119 ------------------------------------------------------
 * The reference packs {u32 saddr, u32 daddr, u8 0, u8 IPPROTO_TCP, u16 len}
 * into a 12-byte struct and sums it as six native-order u16 words. We build
 * the same 12 bytes and read them the same way. */
unsigned long oracle_pseudo(uint32_t saddr_be, uint32_t daddr_be, uint16_t len_be) {
    uint8_t ph[12];
    memcpy(ph + 0, &saddr_be, 4);
    memcpy(ph + 4, &daddr_be, 4);
    ph[8] = 0;
    ph[9] = 6; /* IPPROTO_TCP */
    memcpy(ph + 10, &len_be, 2);
    unsigned long sum = 0;
    for (int i = 0; i < 6; ++i) {
        uint16_t w;
        memcpy(&w, ph + 2 * i, 2);
        sum += w;
    }
    return sum;
}

/* ---- context.c:121-145 ------------------------------------------------------
 * sum (signed 64-bit) = sumStart + native u16 words; an odd trailing byte is
 * added as the low byte of a zeroed u16; then EXACTLY two folds and a
 * complement truncated to 16 bits. */
unsigned short oracle_csum_continue(unsigned long sum_start, const char *p, int nbytes) {
    long sum = (long) sum_start;
    const unsigned char *q = (const unsigned char *) p;
    while (nbytes > 1) {
        uint16_t w;
        memcpy(&w, q, 2);
        sum += w;
        q += 2;
        nbytes -= 2;
    }
    if (nbytes == 1) {
        uint16_t odd = 0;
        memcpy(&odd, q, 1); /* low byte on little-endian, as *(u_char*)&oddbyte */
        sum += odd;
    }
    sum = (sum >> 16) + (sum & 0xffff);
    sum = sum + (sum >> 16);
    return (unsigned short) (short) ~sum;
}

/* ---- SURVEY.md Appendix B generator ---------------------------------------- */
uint64_t oracle_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t stream_word(uint64_t w) {
    return oracle_mix64(0x5EEDC0DEull + (w + 1) * 0x9E3779B97F4A7C15ull);
}

void oracle_gen_stream(uint8_t *dst, uint64_t off, uint64_t nbytes) {
    uint64_t b = off, end = off + nbytes;
    while (b < end && (b & 7)) {
        uint64_t v = stream_word(b >> 3);
        *dst++ = (uint8_t) (v >> (8 * (b & 7)));
        ++b;
    }
    while (b + 8 <= end) {
        uint64_t v = stream_word(b >> 3);
        memcpy(dst, &v, 8);
        dst += 8;
        b += 8;
    }
    while (b < end) {
        uint64_t v = stream_word(b >> 3);
        *dst++ = (uint8_t) (v >> (8 * (b & 7)));
        ++b;
    }
}

uint32_t oracle_saddr(uint64_t i) { return htonl(0x0A000000u | (uint32_t) (i & 0xFFFFFFu)); }
uint32_t oracle_daddr(uint64_t i) { return htonl(0xC0A80000u | (uint32_t) ((i * 7u) & 0xFFFFu)); }

struct synth_job {
    uint64_t s0, s1, seg_base;
    uint32_t L;
    uint16_t *out;
    int err;
};

static void *synth_worker(void *arg) {
    struct synth_job *j = (struct synth_job *) arg;
    uint8_t *buf = (uint8_t *) malloc(j->L ? j->L : 1);
    if (!buf) { j->err = 1; return 0; }
    const uint16_t len_be = htons((uint16_t) j->L);
    for (uint64_t k = j->s0; k < j->s1; ++k) {
        uint64_t i = j->seg_base + k;
        oracle_gen_stream(buf, i * (uint64_t) j->L, j->L);
        j->out[k] = oracle_csum_continue(oracle_pseudo(oracle_saddr(i), oracle_daddr(i), len_be),
                                         (const char *) buf, (int) j->L);
    }
    free(buf);
    return 0;
}

int oracle_synth_batch(uint64_t seg0, uint64_t n, uint32_t L, uint16_t *out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    struct synth_job jobs[64];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].s0 = n * (uint64_t) t / (uint64_t) nthreads;
        jobs[t].s1 = n * (uint64_t) (t + 1) / (uint64_t) nthreads;
        jobs[t].seg_base = seg0;
        jobs[t].L = L;
        jobs[t].out = out;
        jobs[t].err = 0;
        pthread_create(&th[t], 0, synth_worker, &jobs[t]);
    }
    int err = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], 0);
        err |= jobs[t].err;
    }
    return err ? -1 : 0;
}

void oracle_batch_desc(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                       const uint32_t *sum_start, uint64_t n, uint16_t *out) {
    for (uint64_t k = 0; k < n; ++k)
        out[k] = oracle_csum_continue(sum_start[k], (const char *) (base + off[k]), (int) len[k]);
}

/* ---- wire framing: context.c:169-209 (build) / loop.c:44-47 (flush) --------
 * struct iphdr on little-endian: byte0 = version<<4 | ihl, tot_len @2 (BE),
 * protocol @9, saddr @12, daddr @16. TCP header at ihl*4; check at TCP+16.
 * mode bit0: verify; bit1: IPv4 header checksum too (status 2 = bad). */
void oracle_ipv4_batch(uint8_t *base, const uint64_t *off, uint64_t n, uint32_t cap,
                       int mode, uint16_t *out, uint8_t *status) {
    for (uint64_t k = 0; k < n; ++k) {
        uint8_t *ip = base + off[k];
        unsigned ver = ip[0] >> 4, ihl = ip[0] & 15u;
        unsigned tot = ((unsigned) ip[2] << 8) | ip[3];
        unsigned proto = ip[9];
        if (ver != 4 || proto != 6 || ihl < 5 || tot < ihl * 4u + 20u || tot > cap) {
            if (status) status[k] = 1;
            if (out) out[k] = 0;
            continue;
        }
        uint32_t sa, da;
        memcpy(&sa, ip + 12, 4);
        memcpy(&da, ip + 16, 4);
        uint8_t *tcp = ip + ihl * 4u;
        unsigned tcp_len = tot - ihl * 4u;
        unsigned long ps = oracle_pseudo(sa, da, htons((uint16_t) tcp_len));
        int verify = mode & 1, iphdr = mode & 2;
        uint8_t st = 0;
        if (!verify) {
            tcp[16] = 0;
            tcp[17] = 0;
            uint16_t c = oracle_csum_continue(ps, (const char *) tcp, (int) tcp_len);
            memcpy(tcp + 16, &c, 2);
            if (out) out[k] = c;
        } else {
            uint16_t v = oracle_csum_continue(ps, (const char *) tcp, (int) tcp_len);
            if (out) out[k] = v;
            /* CHECKSUM_PARTIAL: check holds the un-complemented folded pseudo sum
             * (new behaviour, no reference result: SURVEY.md §4.5) */
            uint16_t cw;
            memcpy(&cw, tcp + 16, 2);
            if (v != 0 && cw == (uint16_t) ~oracle_csum_continue(ps, "", 0)) st |= 4;
        }
        if (iphdr) { /* context.c:179 (commented out in the reference), over ihl*4 bytes */
            if (!verify) {
                ip[10] = 0;
                ip[11] = 0;
                uint16_t c = oracle_csum_continue(0, (const char *) ip, (int) (ihl * 4u));
                memcpy(ip + 10, &c, 2);
            } else if (oracle_csum_continue(0, (const char *) ip, (int) (ihl * 4u)) != 0) {
                st |= 2;
            }
        }
        if (status) status[k] = st;
    }
}

/* ---- context.c:150-213, us_internal_socket_context_send_packet -------------
 * The same field assignments on the same system structs (struct iphdr, the
 * reference's struct TcpHeader = struct tcphdr + options[4], Packets.h:46-50).
 * Not restated: the 10 % drop (:153-156), getIpPacketBuffer (:167), printf. */
void oracle_tx_build(const uint8_t *payload, const oracle_txseg_t *segs, uint64_t n, uint8_t *out, int iphdr,
                     uint16_t *checks) {
    for (uint64_t k = 0; k < n; ++k) {
        const oracle_txseg_t *d = &segs[k];
        const int data = (d->flags & 16) != 0;
        const size_t length = data ? d->len : 0;
        if (length > 65491) {
            if (checks) checks[k] = 0;
            continue;
        }
        /* The reference casts its (aligned) out-buffer to the system structs; the
         * packets here may sit at any offset, so the same assignments go to an
         * aligned 44-byte image that is then copied into place (UBSan-clean). */
        union {
            struct {
                struct iphdr ip;
                struct tcphdr th;
                uint8_t opts[4];
            } s;
            uint8_t b[44];
        } h;
        _Static_assert(sizeof(struct iphdr) == 20 && sizeof(struct tcphdr) == 20, "wire header sizes");
        struct iphdr *ip = &h.s.ip;
        memset(ip, 0, sizeof(struct iphdr));                           /* :169 */
        ip->ihl = 5;                                                   /* :171 */
        ip->version = 4;
        ip->tot_len = htons((uint16_t) (sizeof(struct iphdr) + 24 + length));
        ip->id = (uint16_t) htonl(54321);                              /* :174, u32 -> u16 as stored */
        ip->ttl = 255;
        ip->protocol = IPPROTO_TCP;
        ip->saddr = d->saddr_be;
        ip->daddr = d->daddr_be;
        struct tcphdr *th = &h.s.th;
        uint8_t *tcp = h.b + sizeof(struct iphdr);
        memset(tcp, 0, 24);                                            /* :182, sizeof(struct TcpHeader) */
        th->ack = (d->flags & 1) != 0;                                 /* :184-187 */
        th->syn = (d->flags & 2) != 0;
        th->fin = (d->flags & 4) != 0;
        th->rst = (d->flags & 8) != 0;
        if (data) th->psh = 1;                                         /* :188-189 */
        th->ack_seq = htonl(d->ack);                                   /* :193-196 */
        th->seq = htonl(d->seq);
        th->source = htons(d->sport);
        th->dest = htons(d->dport);
        tcp[20] = 3; tcp[21] = 3; tcp[22] = 5; tcp[23] = 0;            /* :199-202 */
        th->doff = 6;                                                  /* :205 */
        th->window = htons(8192);
        uint8_t *op = out + d->out_off;
        memcpy(op, h.b, 44);
        if (data) memcpy(op + 44, payload + d->payload_off, length);   /* :190 */
        const uint16_t c = oracle_csum_continue(oracle_pseudo(d->saddr_be, d->daddr_be,
                                                              htons((uint16_t) (24 + length))),
                                                (const char *) op + 20, (int) (24 + length));   /* :208-209 */
        memcpy(op + 20 + 16, &c, 2);
        if (iphdr) {                                                   /* :179 */
            const uint16_t ic = oracle_csum_continue(0, (const char *) op, sizeof(struct iphdr));
            memcpy(op + 10, &ic, 2);
        }
        if (checks) checks[k] = c;
    }
}

void oracle_digest(const uint16_t *out, uint64_t n, uint64_t *fnv, uint64_t *sum, uint16_t *xr) {
    uint64_t h = 0xcbf29ce484222325ull, s = 0;
    uint16_t x = 0;
    for (uint64_t i = 0; i < n; ++i) {
        h = (h ^ (out[i] & 0xFFu)) * 0x100000001b3ull;
        h = (h ^ (out[i] >> 8)) * 0x100000001b3ull;
        s += out[i];
        x ^= out[i];
    }
    if (fnv) *fnv = h;
    if (sum) *sum = s;
    if (xr) *xr = x;
}

/* ---- CPU throughput harness (bench.py cpu_baseline, kind "port") ----------- */
#define CB_PSEUDO(s, d, l) oracle_pseudo((s), (d), (l))
#define CB_CSUM(s, p, n) oracle_csum_continue((s), (p), (n))
#define CB_BENCH_NAME oracle_cpu_bench
#include "cpu_bench.inc.c"
