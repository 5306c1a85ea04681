/*
 * mmsg_loop.c — drives the sendmmsg/recvmmsg seam the way the reference's loop
 * does (loop.c:27-94 releaseSend, loop.c:22-25 fetchPackageBatch), over UDP
 * loopback so no root is needed. Run under LD_PRELOAD=libtcpcsum_preload.so.
 *
 *   mmsg_loop <npkts> <out-file> [cpu-checks | corrupt | trunc | forge | plain] [pinned | iov2 | fork]
 *
 * Allocates the loop's buffers as loop.c:180-183 does (1024 in-buffers and 1024
 * out-buffers, 32 KiB each, malloc'd alternately), builds npkts IPv4/TCP
 * packets, packet i in outBuffer[i % 1024] as it is queued, with the reference's framing
 * (context.c:169-206): check = 0, or — with "cpu-checks" — the check the
 * reference's CPU path would store (tcpcsum_continue == csum_continue,
 * context.c:208). "corrupt": CPU checks, then one TCP header byte (the
 * window's low byte) of every 7th packet flipped after the check was taken,
 * so those no longer verify; the receiver then expects only the others (the
 * interposer's TCPCSUM_PRELOAD_RX=drop). "trunc": CPU checks, and every
 * packet received into a 600-byte buffer with MSG_TRUNC, so a longer datagram
 * is cut short while msg_len reports its full length. "forge": CPU checks,
 * except that every 7th packet (i % 7 == 3) carries a forged CHECKSUM_PARTIAL
 * check word (the un-complemented pseudo-header fold, which is what Linux
 * loopback leaves for offload) from a non-loopback source, 192.0.2.1, and
 * every 7th packet at i % 7 == 5 a genuine-looking one with both addresses
 * in 127/8 (daddr 127.x.y.z). "pinned": the out-buffers are carved from one
 * tcpcsum_host_alloc pool (INTEGRATION.md level 2: loop.c:180-183 allocating
 * its pool page-locked), so the interposer fills them in place. "iov2": every
 * message is received into two iovecs (the first 800 bytes of an in-buffer,
 * then the rest): a packet the first holds whole is verified, a longer one is
 * a scatter read the interposer passes through unverified. Under
 * TCPCSUM_PRELOAD_POOL=1 the interposer serves the loop's 2048 mallocs from its
 * page-locked arena and both seams run in place. "fork": after the run, a forked
 * child mallocs and writes a 32 KiB buffer, frees one of the parent's, sends one
 * packet through the seam, and prints "fork child parent_owned=<0|1|-1>
 * child_owned=<..> send=<r> errno=<e>" (owned: whether the interposer's pool holds
 * the block, -1 without the interposer); the parent waits for it (exit 6 if it failed).
 * "threads": before the loop allocates its buffers, a thread of its own and a HIP
 * host callback (the GPU runtime's thread) each malloc one 32 KiB buffer and free it;
 * prints "threads app_owned=<0|1> cb_owned=<0|1> cb_guarded=<0|1>" (the pool should
 * serve the loop's thread, never the runtime's; exit 8 if the callback did not run).
 * Under TCPCSUM_PRELOAD_RX=drop the receiver expects exactly the packets the
 * mode makes unverifiable to go missing (corrupt / forge: i % 7 == 3, with iov2
 * only those of at most 800 bytes; trunc: those longer than 600 bytes). Sends them with sendmmsg in batches
 * of <= 1024 and receives them with recvmmsg. Writes to <out-file>: for every
 * packet u32 length + the bytes as built, then u32 length + the bytes as
 * received (length 0: never received). Exit 0 on success; 3 if sendmmsg
 * failed (errno printed); 4 if recvmmsg failed; 5 if a packet went missing;
 * 6 if the fork child failed.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <pthread.h>
#include <netinet/in.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "tcpcsum.h"

enum { NBUF = 1024, SLOT = 1024 * 32, IOV2_FIRST = 800 };   /* loop.c:180-183 */

/* the interposer's (preload or --wrap build); absent when the loop runs without it */
extern int tcpcsum_preload_pool_owns(const void *p) __attribute__((weak));
extern int tcpcsum_preload_thread_guarded(void) __attribute__((weak));

/* "threads": who gets a block of the loop's size */
struct probe_alloc {
    int ran, owned, guarded;
};

static void *probe_alloc_run(void *arg) {
    struct probe_alloc *pa = (struct probe_alloc *) arg;
    uint8_t *p = malloc(SLOT);
    if (p) memset(p, 1, SLOT);
    pa->owned = p && tcpcsum_preload_pool_owns ? tcpcsum_preload_pool_owns(p) : 0;
    pa->guarded = tcpcsum_preload_thread_guarded ? tcpcsum_preload_thread_guarded() : -1;
    free(p);
    pa->ran = 1;
    return NULL;
}

static void probe_alloc_cb(void *arg) {
    probe_alloc_run(arg);
}

/* the loop's own thread, then a HIP host callback (hipLaunchHostFunc on the null
 * stream, found in the HIP runtime libtcpcsum brought in) */
static int threads_check(void) {
    struct probe_alloc app = {0, 0, 0}, cb = {0, 0, 0};
    pthread_t th;
    if (pthread_create(&th, NULL, probe_alloc_run, &app) || pthread_join(th, NULL)) return 8;
    typedef int (*launch_host_fn)(void *, void (*)(void *), void *);
    typedef int (*sync_fn)(void *);
    launch_host_fn lh = (launch_host_fn) dlsym(RTLD_DEFAULT, "hipLaunchHostFunc");
    sync_fn sy = (sync_fn) dlsym(RTLD_DEFAULT, "hipStreamSynchronize");
    if (!lh || !sy || lh(NULL, probe_alloc_cb, &cb) || sy(NULL) || !cb.ran) return 8;
    printf("threads app_owned=%d cb_owned=%d cb_guarded=%d\n", app.owned, cb.owned, cb.guarded);
    fflush(stdout);
    return 0;
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next32(void) {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (uint32_t) (rng >> 16);
}

/* the un-complemented fold of the pseudo-header sum: a CHECKSUM_PARTIAL check word */
static uint16_t partial_word(uint32_t sa, uint32_t da, uint16_t len_be) {
    return (uint16_t) ~tcpcsum_continue(tcpcsum_pseudo(sa, da, len_be), "", 0);
}

static size_t build(uint8_t *b, int i, int cpu_checks, int corrupt, int forge) {
    size_t payload = (size_t) (next32() % 1457);            /* 0 .. 1456 (1500-B MTU) */
    size_t tot = 20 + 24 + payload;
    memset(b, 0, 44);
    b[0] = 0x45;                                              /* version 4, ihl 5 */
    b[2] = (uint8_t) (tot >> 8); b[3] = (uint8_t) tot;        /* tot_len (BE) */
    b[4] = 0xd4; b[5] = 0x31;                                 /* id */
    b[8] = 255; b[9] = 6;                                     /* ttl, IPPROTO_TCP */
    uint32_t sa = htonl(0x7F000001u), da = htonl(0x0A000000u | (uint32_t) i);
    if (forge && i % 7 == 3) sa = htonl(0xC0000201u);                   /* 192.0.2.1: not loopback */
    if (forge && i % 7 == 5) da = htonl(0x7F000000u | (uint32_t) i);    /* 127.x.y.z */
    memcpy(b + 12, &sa, 4); memcpy(b + 16, &da, 4);
    uint8_t *t = b + 20;
    t[0] = 4000 >> 8; t[1] = 4000 & 255; t[2] = 45001 >> 8; t[3] = 45001 & 255;
    uint32_t seq = htonl(next32()), ack = htonl(next32());
    memcpy(t + 4, &seq, 4); memcpy(t + 8, &ack, 4);
    t[12] = 6 << 4; t[13] = 0x18;                             /* doff 6, PSH|ACK */
    t[14] = 8192 >> 8; t[15] = 0;                             /* window */
    t[20] = 3; t[21] = 3; t[22] = 5; t[23] = 0;               /* window scale option */
    for (size_t k = 0; k < payload; ++k) t[24 + k] = (uint8_t) next32();
    if (cpu_checks) {
        uint16_t c = tcpcsum_continue(tcpcsum_pseudo(sa, da, htons((uint16_t) (24 + payload))),
                                      (const char *) t, (int) (24 + payload));
        memcpy(t + 16, &c, 2);
    }
    if (corrupt && i % 7 == 3) t[15] ^= 0x5a;
    if (forge && (i % 7 == 3 || i % 7 == 5)) {
        const uint16_t c = partial_word(sa, da, htons((uint16_t) (24 + payload)));
        memcpy(t + 16, &c, 2);
    }
    return tot;
}

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s npkts out [cpu-checks|corrupt|trunc|forge|plain] [pinned|iov2|fork]\n", argv[0]); return 2; }
    int n = atoi(argv[1]);
    int corrupt = argc > 3 && !strcmp(argv[3], "corrupt");
    int trunc = argc > 3 && !strcmp(argv[3], "trunc");
    int forge = argc > 3 && !strcmp(argv[3], "forge");
    int pinned = argc > 4 && !strcmp(argv[4], "pinned");
    int iov2 = argc > 4 && !strcmp(argv[4], "iov2");
    int forkm = argc > 4 && !strcmp(argv[4], "fork");
    if (argc > 4 && !strcmp(argv[4], "threads")) {
        const int rc = threads_check();
        if (rc) return rc;
    }
    int cpu_checks = corrupt || trunc || forge || (argc > 3 && !strcmp(argv[3], "cpu-checks"));
    const char *rxm = getenv("TCPCSUM_PRELOAD_RX");
    const int rx_drop = rxm && !strcmp(rxm, "drop");
    const size_t rx_cap = trunc ? 600 : SLOT;
    FILE *f = fopen(argv[2], "wb");
    if (!f || n <= 0) return 2;
    int rx = socket(AF_INET, SOCK_DGRAM, 0), tx = socket(AF_INET, SOCK_DGRAM, 0);
    struct sockaddr_in a = {0};
    a.sin_family = AF_INET; a.sin_addr.s_addr = htonl(0x7F000001u); a.sin_port = 0;
    if (bind(rx, (struct sockaddr *) &a, sizeof a)) { perror("bind"); return 2; }
    socklen_t al = sizeof a;
    getsockname(rx, (struct sockaddr *) &a, &al);
    /* a receive that finds nothing for 3 s returns EAGAIN instead of blocking for ever
     * (recvmmsg's own timeout is checked only after a datagram arrives): under rx drop
     * the rest of the burst was dropped */
    struct timeval rto = {3, 0};
    setsockopt(rx, SOL_SOCKET, SO_RCVTIMEO, &rto, sizeof rto);
    /* the loop's packet buffers, exactly as loop.c:180-183 allocates them: 1024
     * in-buffers and 1024 out-buffers of 32 KiB, malloc'd alternately. "pinned"
     * carves the out-buffers from one tcpcsum_host_alloc block instead. */
    static uint8_t *buffer[NBUF], *outBuffer[NBUF];
    uint8_t *pool = NULL;
    if (pinned) {
        pool = (uint8_t *) tcpcsum_host_alloc((size_t) NBUF * SLOT);
        if (!pool) { fprintf(stderr, "tcpcsum_host_alloc failed\n"); return 2; }
    }
    for (int i = 0; i < NBUF; ++i) {
        buffer[i] = malloc(SLOT);
        outBuffer[i] = pinned ? pool + (size_t) i * SLOT : malloc(SLOT);
        if (!buffer[i] || !outBuffer[i]) return 2;
    }
    /* what was built and what arrived, per packet, at their own sizes */
    uint8_t **orig = calloc((size_t) n, sizeof *orig), **in = calloc((size_t) n, sizeof *in);
    size_t *olen = calloc((size_t) n, sizeof *olen), *ilen = calloc((size_t) n, sizeof *ilen);
    int drops_only = 0;
    enum { B = 64 };   /* stay below the default socket receive buffer per burst */
    struct mmsghdr mv[B];
    struct iovec iv[2 * B];
    for (int s0 = 0; s0 < n; s0 += B) {
        int cnt = n - s0 < B ? n - s0 : B;
        memset(mv, 0, sizeof mv);
        for (int k = 0; k < cnt; ++k) {   /* packet i goes out of outBuffer[i % 1024], as queued */
            const int i = s0 + k;
            uint8_t *ob = outBuffer[i % NBUF];
            olen[i] = build(ob, i, cpu_checks, corrupt, forge);
            orig[i] = malloc(olen[i]);
            memcpy(orig[i], ob, olen[i]);
            iv[k].iov_base = ob; iv[k].iov_len = olen[i];
            mv[k].msg_hdr.msg_iov = &iv[k]; mv[k].msg_hdr.msg_iovlen = 1;
            mv[k].msg_hdr.msg_name = &a; mv[k].msg_hdr.msg_namelen = sizeof a;
        }
        int sent = 0;
        while (sent < cnt) {
            int r = sendmmsg(tx, mv + sent, (unsigned) (cnt - sent), 0);
            if (r < 0) { fprintf(stderr, "sendmmsg: %s\n", strerror(errno)); return 3; }
            sent += r;
        }
        int want = cnt;   /* under rx drop: the packets this mode makes unverifiable never arrive */
        if (rx_drop)
            for (int k = 0; k < cnt; ++k) {
                const int i = s0 + k;
                /* iov2: a packet longer than the first iovec is a scatter read, passed unverified */
                const int whole = !iov2 || olen[i] <= IOV2_FIRST;
                want -= ((corrupt || forge) && i % 7 == 3 && whole) || (trunc && olen[i] > rx_cap);
            }
        int got = 0;
        while (got < want) {
            memset(mv, 0, sizeof mv);
            for (int k = 0; k < cnt - got; ++k) {   /* into the loop's in-buffers (loop.c:186-189) */
                if (iov2) {
                    iv[2 * k].iov_base = buffer[k]; iv[2 * k].iov_len = IOV2_FIRST;
                    iv[2 * k + 1].iov_base = buffer[k] + IOV2_FIRST; iv[2 * k + 1].iov_len = rx_cap - IOV2_FIRST;
                    mv[k].msg_hdr.msg_iov = &iv[2 * k]; mv[k].msg_hdr.msg_iovlen = 2;
                } else {
                    iv[k].iov_base = buffer[k]; iv[k].iov_len = rx_cap;
                    mv[k].msg_hdr.msg_iov = &iv[k]; mv[k].msg_hdr.msg_iovlen = 1;
                }
            }
            struct timespec to = {5, 0};
            int r = recvmmsg(rx, mv, (unsigned) (cnt - got), MSG_WAITFORONE | (trunc ? MSG_TRUNC : 0), &to);
            if (r < 0 && rx_drop && (errno == EAGAIN || errno == EWOULDBLOCK)) break;   /* more dropped than expected */
            if (r < 0) { fprintf(stderr, "recvmmsg: %s\n", strerror(errno)); return 4; }
            if (r == 0 && !rx_drop) return 5;
            for (int k = 0; k < r; ++k) {
                /* which packet: daddr = 10.x.y.z carries its index. Read through the
                 * iovec array by position, as the reference does (getIpPacket,
                 * loop.c:96-100: loop->iovecs[index]), not through mv[k].msg_iov;
                 * a receive with several iovecs per message is reordered by vector
                 * entries, so it is read through the vector */
                const uint8_t *b = iov2 ? (const uint8_t *) mv[k].msg_hdr.msg_iov[0].iov_base
                                        : (const uint8_t *) iv[k].iov_base;
                const size_t held = mv[k].msg_len < rx_cap ? mv[k].msg_len : rx_cap;
                const int idx = held >= 20 ? (b[17] << 16) | (b[18] << 8) | b[19] : -1;   /* 24-bit index */
                if (idx < s0 || idx >= s0 + cnt || ilen[idx]) { fprintf(stderr, "unexpected message\n"); return 5; }
                in[idx] = malloc(held);
                memcpy(in[idx], b, held);
                ilen[idx] = held;
            }
            got += r;
            if (r == 0) {   /* every message of this receive was dropped: wait for the rest */
                struct timespec ts = {0, 1000000};
                nanosleep(&ts, NULL);
                if (++drops_only > 5000) return 5;
            }
        }
    }
    for (int i = 0; i < n; ++i) {
        uint32_t l = (uint32_t) olen[i];
        fwrite(&l, 4, 1, f); fwrite(orig[i], 1, l, f);
        l = (uint32_t) ilen[i];
        fwrite(&l, 4, 1, f);
        if (l) fwrite(in[i], 1, l, f);
    }
    fclose(f);
    if (forkm) {
        fflush(NULL);
        const pid_t pid = fork();
        if (pid < 0) return 6;
        if (pid == 0) {
            const int parent_owned = tcpcsum_preload_pool_owns ? tcpcsum_preload_pool_owns(buffer[0]) : -1;
            uint8_t *p = malloc(SLOT);   /* the loop's size: the child's own memory */
            if (!p) _exit(7);
            memset(p, 0x5a, SLOT);
            const int child_owned = tcpcsum_preload_pool_owns ? tcpcsum_preload_pool_owns(p) : -1;
            free(p);
            free(buffer[0]);             /* a parent's block: freeing it is allowed */
            uint8_t *q = malloc(2048);
            if (!q) _exit(7);
            struct iovec civ = {q, build(q, 1, 0, 0, 0)};
            struct mmsghdr cm;
            memset(&cm, 0, sizeof cm);
            cm.msg_hdr.msg_iov = &civ; cm.msg_hdr.msg_iovlen = 1;
            cm.msg_hdr.msg_name = &a; cm.msg_hdr.msg_namelen = sizeof a;
            errno = 0;
            const int r = sendmmsg(tx, &cm, 1, 0);
            printf("fork child parent_owned=%d child_owned=%d send=%d errno=%d\n", parent_owned, child_owned, r,
                   r < 0 ? errno : 0);
            fflush(stdout);
            _exit(0);
        }
        int st = 0;
        if (waitpid(pid, &st, 0) != pid || !WIFEXITED(st) || WEXITSTATUS(st) != 0) {
            fprintf(stderr, "fork child failed: status 0x%x\n", st);
            return 6;
        }
    }
    for (int i = 0; i < NBUF; ++i) {   /* the buffers go back the way they came */
        free(buffer[i]);
        if (!pinned) free(outBuffer[i]);
    }
    printf("ok %d\n", n);
    return 0;
}
