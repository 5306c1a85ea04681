/*
 * preload_mmsg.c — libtcpcsum_preload.so: zero-edit GPU checksum offload at
 * the reference's syscall seams.
 *
 * The reference flushes finished IPv4/TCP packets in batches of <= 1024 with
 * sendmmsg (/root/reference/loop.c:75, inside releaseSend loop.c:27-94) and
 * reads them with recvmmsg (loop.c:24). Both are dynamic imports, so
 *     LD_PRELOAD=tcp_amd/libtcpcsum_preload.so ./stress
 * puts a whole batch through the GPU without touching context.c / loop.c:
 *
 *   sendmmsg  TCPCSUM_PRELOAD_TX=fill   (default) compute every TCP check on
 *                                       the GPU and store it at TCP+16, then send
 *             TCPCSUM_PRELOAD_TX=verify check that the checks the CPU already
 *                                       wrote (context.c:208) verify to 0 on the
 *                                       GPU: live GPU-vs-reference parity
 *             TCPCSUM_PRELOAD_TX=off
 *   recvmmsg  TCPCSUM_PRELOAD_RX=verify verify every received batch on the GPU
 *                                       (the reference verifies nothing,
 *                                       loop.c:314-399); failures are counted
 *             TCPCSUM_PRELOAD_RX=drop   verify, and return only the segments
 *                                       that pass: the received messages are
 *                                       reordered (the caller's iovecs swap
 *                                       contents, so every buffer stays
 *                                       referenced and loop.c:97's by-index
 *                                       reads see them) with the passing
 *                                       segments first, and the count returned
 *                                       is theirs
 *             TCPCSUM_PRELOAD_RX=off    (default)
 *   TCPCSUM_PRELOAD_IPHDR=1      also fill / verify the IPv4 header checksum
 *   TCPCSUM_PRELOAD_ANY_SOCKET=1 act on every socket, not only SOCK_RAW ones
 *                                (tests run it over UDP loopback, no root)
 *   TCPCSUM_PRELOAD_STATS=1      print counters to stderr at exit
 *   TCPCSUM_PRELOAD_WAIT=spin    wait for the GPU in HIP's spin (default: block,
 *                                TCPCSUM_CTX_BLOCKING_WAIT — the thread sleeps
 *                                while the kernel runs)
 *
 * Buffers the application page-locked (tcpcsum_host_alloc for its out-buffer
 * pool, loop.c:180-183 — INTEGRATION.md level 2 — or its own hipHostRegister)
 * are read and filled in place, with no copy. Any other message's bytes are
 * copied by the library's host threads into pinned staging
 * (tcpcsum_ipv4_batch_ptrs_host), checksummed there, and FILL's 2-byte checks
 * are written back into the caller's buffers. Nothing is ever page-locked
 * behind the application's back (round 3's TCPCSUM_PRELOAD_INPLACE=1, which
 * did that, is gone with ABI v4: DESIGN.md §7). If the GPU path cannot run,
 * the call fails with errno = ENXIO rather than sending (or accepting) packets
 * with unchecked checksums: there is no silent CPU fallback.
 *
 * A segment passes RX verification when its TCP checksum verifies to 0 — or it
 * is CHECKSUM_PARTIAL (its checksum left to offload: Linux loopback does this
 * for locally generated segments) AND both its addresses are
 * in 127.0.0.0/8, which Linux accepts on the loopback interface only (a packet
 * with a 127/8 source arriving on any other interface is a martian and dropped
 * by the kernel) — and (with IPHDR) its IPv4 header checksum verifies. A
 * forged or corrupted segment from anywhere else whose check word happens to
 * equal the un-complemented pseudo-header fold is therefore rejected.
 * Messages that are not IPv4/TCP are passed through untouched (the reference
 * filters them itself, loop.c:319). IPv4/TCP messages the library cannot
 * verify — truncated (tot_len past the bytes received), bad IHL or lengths —
 * are counted as skipped; in drop mode they are dropped, since they would
 * reach the application's TCP handler unverified.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>

#include "rx_compact.h"
#include "tcpcsum.h"

typedef int (*sendmmsg_fn)(int, struct mmsghdr *, unsigned int, int);
typedef int (*recvmmsg_fn)(int, struct mmsghdr *, unsigned int, int, struct timespec *);

enum { MODE_OFF = 0, MODE_FILL = 1, MODE_VERIFY = 2, MODE_DROP = 3 };

struct tcpcsum_preload_stats {
    unsigned long long tx_batches, tx_packets, tx_filled, tx_verified, tx_verify_failed, tx_skipped;
    unsigned long long rx_batches, rx_packets, rx_verified, rx_verify_failed, rx_skipped, rx_partial, rx_dropped;
    unsigned long long errors;
};

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static sendmmsg_fn real_sendmmsg;
static recvmmsg_fn real_recvmmsg;
static int g_tx = MODE_FILL, g_rx = MODE_OFF, g_iphdr, g_any, g_stats;
static tcpcsum_ctx_t *g_ctx;
static int g_ctx_failed;
static uint16_t *g_out;     /* pinned: the kernel writes results straight here */
static uint8_t *g_status;
static struct tcpcsum_preload_stats g_st;

static int env_mode(const char *name, int dflt) {
    const char *v = getenv(name);
    if (!v) return dflt;
    if (!strcmp(v, "fill")) return MODE_FILL;
    if (!strcmp(v, "verify")) return MODE_VERIFY;
    if (!strcmp(v, "drop")) return MODE_DROP;
    if (!strcmp(v, "off") || !strcmp(v, "0")) return MODE_OFF;
    return dflt;
}

static int env_flag(const char *name) {
    const char *v = getenv(name);
    return v && atoi(v);
}

static void print_stats(void) {
    if (!g_stats) return;
    tcpcsum_ctx_stats_t cs;
    memset(&cs, 0, sizeof cs);
    pthread_mutex_lock(&g_mu);
    if (g_ctx) tcpcsum_ctx_get_stats(g_ctx, &cs);
    pthread_mutex_unlock(&g_mu);
    fprintf(stderr,
            "tcpcsum_preload: tx batches=%llu packets=%llu filled=%llu verified=%llu verify_failed=%llu "
            "skipped=%llu | rx batches=%llu packets=%llu verified=%llu verify_failed=%llu skipped=%llu "
            "partial=%llu dropped=%llu | errors=%llu | ctx in_place=%llu staged=%llu copy_threads=%llu "
            "cpu_caller_us=%llu cpu_workers_us=%llu\n",
            g_st.tx_batches, g_st.tx_packets, g_st.tx_filled, g_st.tx_verified, g_st.tx_verify_failed,
            g_st.tx_skipped, g_st.rx_batches, g_st.rx_packets, g_st.rx_verified, g_st.rx_verify_failed,
            g_st.rx_skipped, g_st.rx_partial, g_st.rx_dropped, g_st.errors,
            (unsigned long long) cs.pkts_in_place, (unsigned long long) cs.pkts_staged,
            (unsigned long long) cs.copy_threads, (unsigned long long) (cs.ns_cpu_caller / 1000),
            (unsigned long long) (cs.ns_cpu_workers / 1000));
}

static void init_once(void) {
    real_sendmmsg = (sendmmsg_fn) dlsym(RTLD_NEXT, "sendmmsg");
    real_recvmmsg = (recvmmsg_fn) dlsym(RTLD_NEXT, "recvmmsg");
    g_tx = env_mode("TCPCSUM_PRELOAD_TX", MODE_FILL);
    if (g_tx == MODE_DROP) g_tx = MODE_VERIFY;   /* never drop what the application sends */
    g_rx = env_mode("TCPCSUM_PRELOAD_RX", MODE_OFF);
    g_iphdr = env_flag("TCPCSUM_PRELOAD_IPHDR");
    g_any = env_flag("TCPCSUM_PRELOAD_ANY_SOCKET");
    g_stats = env_flag("TCPCSUM_PRELOAD_STATS");
    if (env_flag("TCPCSUM_PRELOAD_INPLACE"))
        fprintf(stderr, "tcpcsum_preload: TCPCSUM_PRELOAD_INPLACE is gone (ABI v4): buffers from "
                        "tcpcsum_host_alloc are filled in place, all others are copied\n");
    atexit(print_stats);
}

/* Exported for tests / the application: a copy of the counters. */
void tcpcsum_preload_get_stats(struct tcpcsum_preload_stats *out) {
    pthread_mutex_lock(&g_mu);
    if (out) *out = g_st;
    pthread_mutex_unlock(&g_mu);
}

static int wants_fd(int fd) {
    if (g_any) return 1;
    int type = 0;
    socklen_t len = sizeof type;
    if (getsockopt(fd, SOL_SOCKET, SO_TYPE, &type, &len) != 0) return 0;
    return type == SOCK_RAW;
}

/* g_mu held. */
static int ensure_ctx(void) {
    if (g_ctx_failed) return -1;
    if (!g_ctx) {
        int rc = tcpcsum_ctx_create(0, 0, &g_ctx);
        const char *w = getenv("TCPCSUM_PRELOAD_WAIT");
        if (!rc && !(w && !strcmp(w, "spin"))) rc = tcpcsum_ctx_set_flags(g_ctx, TCPCSUM_CTX_BLOCKING_WAIT);
        if (!rc) {
            g_out = (uint16_t *) tcpcsum_host_alloc(1024 * sizeof(uint16_t));
            g_status = (uint8_t *) tcpcsum_host_alloc(1024);
            if (!g_out || !g_status) rc = TCPCSUM_ENOMEM;
        }
        if (rc) {
            fprintf(stderr, "tcpcsum_preload: GPU checksum path unavailable (%s); refusing to send/accept "
                            "packets with unchecked checksums\n", tcpcsum_strerror(rc));
            g_ctx_failed = 1;
            tcpcsum_ctx_destroy(g_ctx);
            g_ctx = NULL;
            return -1;
        }
    }
    return 0;
}

/* Message bytes as received: IPv4 carrying TCP (enough of the header to say so). */
static int is_ipv4_tcp(const uint8_t *p, uint32_t len) {
    return p && len >= 10 && (p[0] >> 4) == 4 && p[9] == 6;
}

/* Both addresses in 127.0.0.0/8: a segment Linux accepted on the loopback
 * interface only (martian source anywhere else). len >= 20 (verified packets). */
static int loopback_pair(const uint8_t *p) {
    return p[12] == 127 && p[16] == 127;
}

/* g_mu held. Whether message k of a finished batch is kept (rx drop), and its
 * accounting. p / len: its bytes as the GPU batch saw them. */
static int account(int k, int fill, int is_tx, const uint8_t *p, uint32_t len) {
    const int skipped = (g_status[k] & TCPCSUM_PKT_SKIPPED) != 0;
    if (skipped) {
        if (is_tx) g_st.tx_skipped++; else g_st.rx_skipped++;
        /* an IPv4/TCP segment that could not be verified (truncated, bad IHL or
         * lengths) is not passed on unverified in drop mode; anything else is
         * not TCP and goes through (the reference filters it, loop.c:319) */
        return !(g_rx == MODE_DROP && !is_tx && is_ipv4_tcp(p, len));
    }
    if (fill) {
        g_st.tx_filled++;
        return 1;
    }
    /* CHECKSUM_PARTIAL segments (checksum left to offload, Linux loopback;
     * SURVEY.md §4.5) are counted apart, not as corrupt — on 127/8 only */
    const int partial = (g_status[k] & TCPCSUM_PKT_CSUM_PARTIAL) != 0 && loopback_pair(p);
    const int bad = (g_out[k] != 0 && !partial) || (g_status[k] & TCPCSUM_PKT_IPHDR_BAD);
    if (is_tx) { g_st.tx_verified++; if (bad) g_st.tx_verify_failed++; }
    else { g_st.rx_verified++; if (bad) g_st.rx_verify_failed++; if (partial) g_st.rx_partial++; }
    return !bad;
}

/* Checksum a batch of <= 1024 messages on the GPU (one iov_base per message:
 * the reference's layout, loop.c:53-54; other messages are SKIPPED). lens:
 * each message's byte count (iov_len for tx, msg_len for rx). fill: store the
 * checks in the caller's buffers. keep (nullable): per message, whether it
 * passed. Returns 0, or -1 with errno set. */
static int gpu_batch(struct mmsghdr *vec, unsigned int vlen, const unsigned int *lens, int fill, int is_tx,
                     unsigned char *keep) {
    void *ptrs[1024];
    uint32_t plen[1024];
    const uint8_t *head[1024];   /* the message's first bytes, to tell IPv4/TCP from the rest */
    uint32_t hlen[1024];
    for (unsigned int i = 0; i < vlen; ++i) {
        const struct msghdr *h = &vec[i].msg_hdr;
        const int one = h->msg_iovlen == 1;
        ptrs[i] = one ? h->msg_iov[0].iov_base : NULL;
        plen[i] = one ? lens[i] : 0;   /* < 20 bytes: SKIPPED, nothing read */
        head[i] = h->msg_iovlen >= 1 && h->msg_iov ? (const uint8_t *) h->msg_iov[0].iov_base : NULL;
        hlen[i] = 0;
        if (head[i]) {
            const size_t cap = h->msg_iov[0].iov_len;
            const unsigned int got = is_tx ? (unsigned int) cap : vec[i].msg_len;
            hlen[i] = (uint32_t) (got < cap ? got : cap);
        }
    }
    pthread_mutex_lock(&g_mu);
    if (ensure_ctx()) {
        g_st.errors++;
        pthread_mutex_unlock(&g_mu);
        errno = ENXIO;
        return -1;
    }
    int mode = (fill ? TCPCSUM_IPV4_FILL : TCPCSUM_IPV4_VERIFY) | (g_iphdr ? TCPCSUM_IPV4_IPHDR : 0);
    int rc = tcpcsum_ipv4_batch_ptrs_host(g_ctx, ptrs, plen, vlen, mode, g_out, g_status);
    if (rc) {
        g_st.errors++;
        pthread_mutex_unlock(&g_mu);
        fprintf(stderr, "tcpcsum_preload: batch failed: %s\n", tcpcsum_strerror(rc));
        errno = ENXIO;
        return -1;
    }
    for (unsigned int i = 0; i < vlen; ++i) {
        const int ok = account((int) i, fill, is_tx, head[i], hlen[i]);
        if (keep) keep[i] = (unsigned char) ok;
    }
    pthread_mutex_unlock(&g_mu);
    return 0;
}

int sendmmsg(int fd, struct mmsghdr *vec, unsigned int vlen, int flags) {
    pthread_once(&g_once, init_once);
    if (g_tx != MODE_OFF && vlen && vec && wants_fd(fd)) {
        unsigned int lens[1024];
        unsigned int done = 0;
        while (done < vlen) {   /* GPU batches of <= 1024 messages */
            unsigned int cnt = vlen - done < 1024 ? vlen - done : 1024;
            for (unsigned int i = 0; i < cnt; ++i) {
                const struct msghdr *h = &vec[done + i].msg_hdr;
                lens[i] = h->msg_iovlen == 1 ? (unsigned int) h->msg_iov[0].iov_len : 0;
            }
            if (gpu_batch(vec + done, cnt, lens, g_tx == MODE_FILL, 1, NULL)) return -1;
            pthread_mutex_lock(&g_mu);
            g_st.tx_batches++;
            g_st.tx_packets += cnt;
            pthread_mutex_unlock(&g_mu);
            done += cnt;
        }
    }
    return real_sendmmsg(fd, vec, vlen, flags);
}

int recvmmsg(int fd, struct mmsghdr *vec, unsigned int vlen, int flags, struct timespec *timeout) {
    pthread_once(&g_once, init_once);
    int r = real_recvmmsg(fd, vec, vlen, flags, timeout);
    if (r > 0 && g_rx != MODE_OFF && wants_fd(fd)) {
        unsigned int lens[1024];
        unsigned char keep[1024];
        unsigned int done = 0, kept = 0;
        const int by_entry = g_rx == MODE_DROP && rx_by_entry(vec, (unsigned int) r);
        while (done < (unsigned int) r) {
            unsigned int cnt = (unsigned int) r - done < 1024 ? (unsigned int) r - done : 1024;
            /* the bytes received, never past the buffer: with MSG_TRUNC in flags a
             * raw or UDP socket reports the datagram's real length in msg_len */
            for (unsigned int i = 0; i < cnt; ++i) {
                const struct msghdr *h = &vec[done + i].msg_hdr;
                const unsigned int cap = h->msg_iovlen == 1 ? (unsigned int) h->msg_iov[0].iov_len : 0;
                lens[i] = vec[done + i].msg_len < cap ? vec[done + i].msg_len : cap;
            }
            if (gpu_batch(vec + done, cnt, lens, 0, 0, keep)) return -1;
            if (g_rx == MODE_DROP) {
                /* stable partition by swaps: passing messages move to the front in
                 * arrival order; failing ones end up behind them, still in the
                 * vector (the caller's buffers all stay referenced) */
                kept = rx_keep_passing(vec, kept, done, cnt, keep, by_entry);
            } else {
                kept += cnt;
            }
            pthread_mutex_lock(&g_mu);
            g_st.rx_batches++;
            g_st.rx_packets += cnt;
            pthread_mutex_unlock(&g_mu);
            done += cnt;
        }
        if (g_rx == MODE_DROP) {
            pthread_mutex_lock(&g_mu);
            g_st.rx_dropped += (unsigned int) r - kept;
            pthread_mutex_unlock(&g_mu);
            r = (int) kept;
        }
    }
    return r;
}
