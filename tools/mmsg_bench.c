/*
 * mmsg_bench.c — per-batch latency of the sendmmsg seam on the reference's own
 * buffer layout: 1024 in/out buffers malloc'd alternately, 32 KiB each
 * (/root/reference/loop.c:180-183), one finished 1500-byte IPv4/TCP packet at
 * the start of each out-buffer (context.c:169-206, check = 0 as at :182), and
 * one sendmmsg of all 1024 messages, one iov_base each (loop.c:44-75).
 *
 *   mmsg_bench gpu <iters>   time sendmmsg; run under LD_PRELOAD=libtcpcsum_preload.so
 *                            with TCPCSUM_PRELOAD_ANY_SOCKET=1 (the socket is an
 *                            unconnected UDP socket, so the real sendmmsg returns
 *                            EDESTADDRREQ at once: the time is the interposer's)
 *   mmsg_bench cpu <iters>   the reference's CPU path for the same batch: one
 *                            csum_continue(getPseudoHeaderSum(...)) per packet
 *                            (tcpcsum_continue / tcpcsum_pseudo == context.c:104-145,
 *                            gcc -O2), stored at TCP+16 as context.c:208 does
 *   mmsg_bench gpu <iters> pinned   the out-buffers carved from one tcpcsum_host_alloc
 *                            pool instead (INTEGRATION.md level 2: loop.c:180-183
 *                            allocating page-locked memory): filled in place
 *   mmsg_bench rx <iters>    the recvmmsg side (loop.c:22-25): 1024 finished packets sent
 *                            as UDP datagrams over loopback, then ONE recvmmsg of all
 *                            1024 into the loop's 32 KiB malloc'd in-buffers is timed —
 *                            under the interposer with TCPCSUM_PRELOAD_RX=drop (verify
 *                            on the GPU; the count returned = segments that verify),
 *                            or without it (plain: the syscall alone)
 *   mmsg_bench rxcpu <iters> the same recvmmsg, then the CPU verify of every segment
 *                            (csum_continue over pseudo header + segment == 0, -O2):
 *                            what verifying on one core would cost the loop
 *
 * Prints one JSON line: first-call and steady-state (min / median) latency
 * per 1024-packet batch, the CPU time the whole process spent per batch
 * (CLOCK_PROCESS_CPUTIME_ID: the calling thread, the library's copy threads
 * and the HIP runtime's own threads — "core-us"), and whether every check
 * equals the CPU's.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "tcpcsum.h"

enum { NPKT = 1024, SLOT = 32768, PAYLOAD = 1456 };

static uint64_t rng = 0x243F6A8885A308D3ull;
static uint32_t next32(void) {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (uint32_t) (rng >> 16);
}

static void build(uint8_t *b, int i) {
    const size_t tot = 20 + 24 + PAYLOAD;
    memset(b, 0, 44);
    b[0] = 0x45;
    b[2] = (uint8_t) (tot >> 8); b[3] = (uint8_t) tot;
    b[4] = 0xd4; b[5] = 0x31;
    b[8] = 255; b[9] = 6;
    uint32_t sa = htonl(0x7F000001u), da = htonl(0x0A000000u | (uint32_t) i);
    memcpy(b + 12, &sa, 4); memcpy(b + 16, &da, 4);
    uint8_t *t = b + 20;
    t[0] = 4000 >> 8; t[1] = 4000 & 255; t[2] = 45001 >> 8; t[3] = 45001 & 255;
    uint32_t seq = htonl(next32()), ack = htonl(next32());
    memcpy(t + 4, &seq, 4); memcpy(t + 8, &ack, 4);
    t[12] = 6 << 4; t[13] = 0x18;
    t[14] = 8192 >> 8;
    t[20] = 3; t[21] = 3; t[22] = 5;
    for (size_t k = 0; k < PAYLOAD; ++k) t[24 + k] = (uint8_t) next32();
}

/* The reference's per-packet check (context.c:208), on the CPU. */
static uint16_t cpu_check(const uint8_t *ip) {
    uint32_t sa, da;
    memcpy(&sa, ip + 12, 4);
    memcpy(&da, ip + 16, 4);
    const int len = 24 + PAYLOAD;
    return tcpcsum_continue(tcpcsum_pseudo(sa, da, htons((uint16_t) len)), (const char *) ip + 20, len);
}

static double now_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static double cpu_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int cmp_d(const void *a, const void *b) {
    const double x = *(const double *) a, y = *(const double *) b;
    return x < y ? -1 : x > y;
}

/* csum_continue over the pseudo header and the whole segment, check included: 0 when
 * the segment verifies (the rx check, context.c:121-145 applied to a received packet) */
static int cpu_verify(const uint8_t *ip, unsigned len) {
    uint32_t sa, da;
    memcpy(&sa, ip + 12, 4);
    memcpy(&da, ip + 16, 4);
    const unsigned tl = len - 20;
    return tcpcsum_continue(tcpcsum_pseudo(sa, da, htons((uint16_t) tl)), (const char *) ip + 20, (int) tl) == 0;
}

static int rx_main(int cpu_verify_mode, int iters) {
    static uint8_t *outb[NPKT], *inb[NPKT];
    static struct iovec tiov[NPKT], riov[NPKT];
    static struct mmsghdr tv[NPKT], rv[NPKT];
    for (int i = 0; i < NPKT; ++i) {
        outb[i] = malloc(SLOT);
        inb[i] = malloc(SLOT);
        memset(inb[i], 0, SLOT);
        build(outb[i], i);
        const uint16_t c = cpu_check(outb[i]);
        memcpy(outb[i] + 36, &c, 2);
        tiov[i].iov_base = outb[i];
        tiov[i].iov_len = 20 + 24 + PAYLOAD;
        tv[i].msg_hdr.msg_iov = &tiov[i];
        tv[i].msg_hdr.msg_iovlen = 1;
        riov[i].iov_base = inb[i];
        riov[i].iov_len = SLOT;
        rv[i].msg_hdr.msg_iov = &riov[i];
        rv[i].msg_hdr.msg_iovlen = 1;
    }
    const int rx = socket(AF_INET, SOCK_DGRAM, 0), tx = socket(AF_INET, SOCK_DGRAM, 0);
    int big = 32 << 20;
    setsockopt(rx, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    setsockopt(tx, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    struct sockaddr_in a = {0};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(0x7F000001u);
    if (bind(rx, (struct sockaddr *) &a, sizeof a) != 0) { perror("bind"); return 2; }
    socklen_t al = sizeof a;
    getsockname(rx, (struct sockaddr *) &a, &al);
    if (connect(tx, (struct sockaddr *) &a, sizeof a) != 0) { perror("connect"); return 2; }
    double *t = malloc(sizeof(double) * (size_t) iters), *c = malloc(sizeof(double) * (size_t) iters);
    int short_batches = 0, bad = 0, kept_last = 0, call_errors = 0;
    for (int k = 0; k < iters; ++k) {
        int sent = 0;
        while (sent < NPKT) {
            const int r = sendmmsg(tx, tv + sent, (unsigned) (NPKT - sent), 0);
            if (r <= 0) { perror("sendmmsg"); return 3; }
            sent += r;
        }
        usleep(2000);   /* every datagram queued before the timed call */
        for (int i = 0; i < NPKT; ++i) riov[i].iov_base = inb[i], riov[i].iov_len = SLOT;
        const double c0 = cpu_us();
        const double t0 = now_us();
        const int r = recvmmsg(rx, rv, NPKT, MSG_DONTWAIT, NULL);
        if (r < 0) ++call_errors;   /* e.g. ENXIO: the interposer had no GPU path */
        int ok = r;
        if (cpu_verify_mode && r > 0) {
            ok = 0;
            for (int i = 0; i < r; ++i) ok += cpu_verify((const uint8_t *) riov[i].iov_base, rv[i].msg_len);
        }
        t[k] = now_us() - t0;
        c[k] = cpu_us() - c0;
        if (r != NPKT) ++short_batches;
        if (ok != NPKT) ++bad;
        kept_last = ok;
        /* drain anything left (a short batch) so the next iteration starts empty */
        while (recvmmsg(rx, rv, NPKT, MSG_DONTWAIT, NULL) > 0) {}
    }
    const double first = t[0];
    qsort(t + 1, (size_t) (iters - 1), sizeof(double), cmp_d);
    qsort(c + 1, (size_t) (iters - 1), sizeof(double), cmp_d);
    double csum = 0;
    for (int k = 1; k < iters; ++k) csum += c[k];
    printf("{\"path\": \"%s\", \"batch\": \"1024 x 1500-B packets received into separate 32 KiB malloc'd buffers "
           "(loop.c:22-25, 180-183), UDP over loopback\", \"first_us\": %.1f, \"min_us\": %.1f, "
           "\"median_us\": %.1f, \"cpu_us_median\": %.1f, \"cpu_us_mean\": %.1f, \"iters\": %d, "
           "\"short_batches\": %d, \"batches_not_all_verified\": %d, \"verified_last\": %d, \"call_errors\": %d}\n",
           cpu_verify_mode ? "recvmmsg + cpu verify per packet (-O2)" : "recvmmsg (interposed when LD_PRELOAD is set)",
           first, t[1], t[1 + (iters - 1) / 2], c[1 + (iters - 1) / 2], csum / (iters - 1), iters, short_batches, bad,
           kept_last, call_errors);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s gpu|cpu|rx|rxcpu iters [pinned]\n", argv[0]); return 2; }
    if (!strcmp(argv[1], "rx") || !strcmp(argv[1], "rxcpu"))
        return rx_main(!strcmp(argv[1], "rxcpu"), atoi(argv[2]) > 1 ? atoi(argv[2]) : 2);
    const int gpu = !strcmp(argv[1], "gpu");
    const int iters = atoi(argv[2]) > 1 ? atoi(argv[2]) : 2;
    const int pinned = argc > 3 && !strcmp(argv[3], "pinned");
    static uint8_t *inb[NPKT], *outb[NPKT];
    uint8_t *pool = pinned ? (uint8_t *) tcpcsum_host_alloc((size_t) NPKT * SLOT) : NULL;
    if (pinned && !pool) { fprintf(stderr, "tcpcsum_host_alloc failed\n"); return 2; }
    for (int i = 0; i < NPKT; ++i) {   /* loop.c:180-183: in and out buffers alternate */
        inb[i] = malloc(SLOT);
        memset(inb[i], 0, SLOT);          /* the rx buffers, touched as recvmmsg would */
        outb[i] = pinned ? pool + (size_t) i * SLOT : malloc(SLOT);
        build(outb[i], i);
    }
    static struct iovec iov[NPKT];
    static struct mmsghdr vec[NPKT];
    for (int i = 0; i < NPKT; ++i) {
        iov[i].iov_base = outb[i];
        iov[i].iov_len = 20 + 24 + PAYLOAD;   /* = tot_len, as loop.c:47,54 */
        vec[i].msg_hdr.msg_iov = &iov[i];
        vec[i].msg_hdr.msg_iovlen = 1;
    }
    const int fd = socket(AF_INET, SOCK_DGRAM, 0);
    double *t = malloc(sizeof(double) * (size_t) iters);
    double *c = malloc(sizeof(double) * (size_t) iters);
    int call_errors = 0;
    for (int k = 0; k < iters; ++k) {
        for (int i = 0; i < NPKT; ++i) memset(outb[i] + 36, 0, 2);   /* check = 0 (context.c:182) */
        const double c0 = cpu_us();
        const double t0 = now_us();
        if (gpu) {
            /* the unconnected socket's own EDESTADDRREQ is expected; ENXIO means no GPU path */
            if (sendmmsg(fd, vec, NPKT, 0) < 0 && errno == ENXIO) ++call_errors;
        } else {
            for (int i = 0; i < NPKT; ++i) {
                const uint16_t c = cpu_check(outb[i]);
                memcpy(outb[i] + 36, &c, 2);
            }
        }
        t[k] = now_us() - t0;
        c[k] = cpu_us() - c0;
    }
    int mismatches = 0;
    for (int i = 0; i < NPKT; ++i) {
        uint16_t got;
        memcpy(&got, outb[i] + 36, 2);
        memset(outb[i] + 36, 0, 2);
        mismatches += got != cpu_check(outb[i]);
    }
    const double first = t[0];
    qsort(t + 1, (size_t) (iters - 1), sizeof(double), cmp_d);
    qsort(c + 1, (size_t) (iters - 1), sizeof(double), cmp_d);
    double csum = 0;
    for (int k = 1; k < iters; ++k) csum += c[k];
    printf("{\"path\": \"%s\", \"batch\": \"1024 x 1500-B packets, separate 32 KiB %s buffers (loop.c:180-183)\", "
           "\"first_us\": %.1f, \"min_us\": %.1f, \"median_us\": %.1f, \"cpu_us_median\": %.1f, "
           "\"cpu_us_mean\": %.1f, \"iters\": %d, \"checks_match_cpu\": %s, \"mismatches\": %d, \"call_errors\": %d}\n",
           gpu ? "sendmmsg under libtcpcsum_preload.so" : "cpu csum_continue per packet (-O2)",
           pinned ? "tcpcsum_host_alloc'd" : "malloc'd", first, t[1], t[1 + (iters - 1) / 2],
           c[1 + (iters - 1) / 2], csum / (iters - 1), iters, mismatches ? "false" : "true", mismatches, call_errors);
    close(fd);
    return 0;
}
