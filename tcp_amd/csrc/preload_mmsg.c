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
 *             TCPCSUM_PRELOAD_RX=off    (default)
 *   TCPCSUM_PRELOAD_IPHDR=1      also fill / verify the IPv4 header checksum
 *   TCPCSUM_PRELOAD_ANY_SOCKET=1 act on every socket, not only SOCK_RAW ones
 *                                (tests run it over UDP loopback, no root)
 *   TCPCSUM_PRELOAD_STATS=1      print counters to stderr at exit
 *   TCPCSUM_PRELOAD_COPY=1       gather packets into a page-locked staging
 *                                area instead (for applications that free()
 *                                their packet buffers; see below)
 *
 * Default: the kernel works on the caller's own buffers — one iov_base per
 * message, each buffer page-locked on first use and kept registered for the
 * life of the process (tcpcsum_ipv4_batch_ptrs_host) — reading the packets
 * over PCIe and storing the checks in place: no CPU pass over packet bytes.
 * This suits the reference, which allocates its 2 x 1024 packet buffers once
 * and never frees them (loop.c:180-183). With TCPCSUM_PRELOAD_COPY=1 packets
 * are copied into pinned staging and only the 2-byte check fields are
 * written back. If the GPU path cannot run, the call fails with errno = ENXIO
 * rather than sending packets with unchecked checksums: there is no silent
 * CPU fallback.
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

#include "tcpcsum.h"

typedef int (*sendmmsg_fn)(int, struct mmsghdr *, unsigned int, int);
typedef int (*recvmmsg_fn)(int, struct mmsghdr *, unsigned int, int, struct timespec *);

enum { MODE_OFF = 0, MODE_FILL = 1, MODE_VERIFY = 2 };

struct tcpcsum_preload_stats {
    unsigned long long tx_batches, tx_packets, tx_filled, tx_verified, tx_verify_failed, tx_skipped;
    unsigned long long rx_batches, rx_packets, rx_verified, rx_verify_failed, rx_skipped, rx_partial;
    unsigned long long errors;
};

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static sendmmsg_fn real_sendmmsg;
static recvmmsg_fn real_recvmmsg;
static int g_tx = MODE_FILL, g_rx = MODE_OFF, g_iphdr, g_any, g_stats, g_copy;
static tcpcsum_ctx_t *g_ctx;
static int g_ctx_failed;
static uint8_t *g_stage;   /* pinned */
static size_t g_stage_bytes;
static uint64_t *g_off;
static uint16_t *g_out;
static uint8_t *g_status;
static size_t g_cap_pkts;
static struct tcpcsum_preload_stats g_st;

static int env_mode(const char *name, int dflt) {
    const char *v = getenv(name);
    if (!v) return dflt;
    if (!strcmp(v, "fill")) return MODE_FILL;
    if (!strcmp(v, "verify")) return MODE_VERIFY;
    if (!strcmp(v, "off") || !strcmp(v, "0")) return MODE_OFF;
    return dflt;
}

static void print_stats(void) {
    if (!g_stats) return;
    fprintf(stderr,
            "tcpcsum_preload: tx batches=%llu packets=%llu filled=%llu verified=%llu verify_failed=%llu "
            "skipped=%llu | rx batches=%llu packets=%llu verified=%llu verify_failed=%llu skipped=%llu "
            "partial=%llu | errors=%llu\n",
            g_st.tx_batches, g_st.tx_packets, g_st.tx_filled, g_st.tx_verified, g_st.tx_verify_failed,
            g_st.tx_skipped, g_st.rx_batches, g_st.rx_packets, g_st.rx_verified, g_st.rx_verify_failed,
            g_st.rx_skipped, g_st.rx_partial, g_st.errors);
}

static void init_once(void) {
    real_sendmmsg = (sendmmsg_fn) dlsym(RTLD_NEXT, "sendmmsg");
    real_recvmmsg = (recvmmsg_fn) dlsym(RTLD_NEXT, "recvmmsg");
    g_tx = env_mode("TCPCSUM_PRELOAD_TX", MODE_FILL);
    g_rx = env_mode("TCPCSUM_PRELOAD_RX", MODE_OFF);
    g_iphdr = getenv("TCPCSUM_PRELOAD_IPHDR") && atoi(getenv("TCPCSUM_PRELOAD_IPHDR"));
    g_any = getenv("TCPCSUM_PRELOAD_ANY_SOCKET") && atoi(getenv("TCPCSUM_PRELOAD_ANY_SOCKET"));
    g_stats = getenv("TCPCSUM_PRELOAD_STATS") && atoi(getenv("TCPCSUM_PRELOAD_STATS"));
    g_copy = getenv("TCPCSUM_PRELOAD_COPY") && atoi(getenv("TCPCSUM_PRELOAD_COPY"));
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
static int ensure_ctx(size_t bytes, size_t npkts) {
    if (g_ctx_failed) return -1;
    if (!g_ctx) {
        int rc = tcpcsum_ctx_create(0, 0, &g_ctx);
        if (rc) {
            fprintf(stderr, "tcpcsum_preload: GPU checksum path unavailable (%s); refusing to send/accept "
                            "packets with unchecked checksums\n", tcpcsum_strerror(rc));
            g_ctx_failed = 1;
            g_ctx = NULL;
            return -1;
        }
    }
    if (bytes > g_stage_bytes) {
        size_t nb = g_stage_bytes ? g_stage_bytes : (size_t) 1 << 21;
        while (nb < bytes) nb *= 2;
        uint8_t *p = (uint8_t *) tcpcsum_host_alloc(nb);
        if (!p) return -1;
        tcpcsum_host_free(g_stage);
        g_stage = p;
        g_stage_bytes = nb;
    }
    if (npkts > g_cap_pkts) {
        size_t np = g_cap_pkts ? g_cap_pkts : 1024;
        while (np < npkts) np *= 2;
        uint64_t *o = (uint64_t *) tcpcsum_host_alloc(np * sizeof(uint64_t));
        uint16_t *u = (uint16_t *) tcpcsum_host_alloc(np * sizeof(uint16_t));
        uint8_t *s = (uint8_t *) tcpcsum_host_alloc(np);
        if (!o || !u || !s) {
            tcpcsum_host_free(o); tcpcsum_host_free(u); tcpcsum_host_free(s);
            return -1;
        }
        tcpcsum_host_free(g_off); tcpcsum_host_free(g_out); tcpcsum_host_free(g_status);
        g_off = o; g_out = u; g_status = s;
        g_cap_pkts = np;
    }
    return 0;
}

/* g_mu held. Count one message of a finished batch (k: its slot in the
 * batch arrays). */
static void account(int k, int fill, int is_tx) {
    const int skipped = (g_status[k] & TCPCSUM_PKT_SKIPPED) != 0;
    if (skipped) {
        if (is_tx) g_st.tx_skipped++; else g_st.rx_skipped++;
    } else if (fill) {
        g_st.tx_filled++;
    } else {
        /* CHECKSUM_PARTIAL segments (checksum left to offload, e.g. Linux
         * loopback) are counted apart, not as corrupt */
        const int partial = (g_status[k] & TCPCSUM_PKT_CSUM_PARTIAL) != 0;
        const int bad = (g_out[k] != 0 && !partial) || (g_status[k] & TCPCSUM_PKT_IPHDR_BAD);
        if (is_tx) { g_st.tx_verified++; if (bad) g_st.tx_verify_failed++; }
        else { g_st.rx_verified++; if (bad) g_st.rx_verify_failed++; if (partial) g_st.rx_partial++; }
    }
}

/* Default path: the GPU reads the caller's buffers in place (scatter-gather,
 * each buffer page-locked once) and FILL stores the checks there. */
static int gpu_batch_inplace(struct mmsghdr *vec, unsigned int vlen, const unsigned int *lens, int fill, int is_tx) {
    void *ptrs[1024];
    uint32_t plen[1024];
    for (unsigned int i = 0; i < vlen; ++i) {
        const int one = vec[i].msg_hdr.msg_iovlen == 1;
        ptrs[i] = one ? vec[i].msg_hdr.msg_iov[0].iov_base : NULL;
        plen[i] = one ? lens[i] : 0;   /* < 20 bytes: SKIPPED, nothing read */
    }
    pthread_mutex_lock(&g_mu);
    if (ensure_ctx(0, vlen)) {
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
    for (unsigned int i = 0; i < vlen; ++i) account((int) i, fill, is_tx);
    pthread_mutex_unlock(&g_mu);
    return 0;
}

/* Checksum a batch of single-iovec messages on the GPU. fill: write the check
 * fields back into the caller's buffers. Returns 0, or -1 (errno set). lens
 * gives each message's byte count (iov_len for tx, msg_len for rx). */
static int gpu_batch(struct mmsghdr *vec, unsigned int vlen, const unsigned int *lens, int fill, int is_tx) {
    if (!g_copy) return gpu_batch_inplace(vec, vlen, lens, fill, is_tx);
    size_t total = 0;
    unsigned int m = 0;
    for (unsigned int i = 0; i < vlen; ++i) {
        if (vec[i].msg_hdr.msg_iovlen != 1 || lens[i] < 20) continue;
        total += ((size_t) lens[i] + 16 + 15) & ~(size_t) 15;
        ++m;
    }
    if (!m) return 0;
    pthread_mutex_lock(&g_mu);
    if (ensure_ctx(total, vlen)) {
        g_st.errors++;
        pthread_mutex_unlock(&g_mu);
        errno = ENXIO;
        return -1;
    }
    /* gather: each packet at a 16-B aligned offset, 16 zero bytes of slack after it */
    size_t pos = 0;
    unsigned int k = 0;
    for (unsigned int i = 0; i < vlen; ++i) {
        if (vec[i].msg_hdr.msg_iovlen != 1 || lens[i] < 20) continue;
        memcpy(g_stage + pos, vec[i].msg_hdr.msg_iov[0].iov_base, lens[i]);
        memset(g_stage + pos + lens[i], 0, 16);
        g_off[k++] = pos;
        pos += ((size_t) lens[i] + 16 + 15) & ~(size_t) 15;
    }
    int mode = (fill ? TCPCSUM_IPV4_FILL : TCPCSUM_IPV4_VERIFY) | (g_iphdr ? TCPCSUM_IPV4_IPHDR : 0);
    /* cap: a packet may not claim more bytes than were handed to the socket */
    int rc = tcpcsum_ipv4_batch_host(g_ctx, g_stage, pos, g_off, m, 65535u, mode, g_out, g_status);
    if (rc) {
        g_st.errors++;
        pthread_mutex_unlock(&g_mu);
        fprintf(stderr, "tcpcsum_preload: batch failed: %s\n", tcpcsum_strerror(rc));
        errno = ENXIO;
        return -1;
    }
    k = 0;
    for (unsigned int i = 0; i < vlen; ++i) {
        if (vec[i].msg_hdr.msg_iovlen != 1 || lens[i] < 20) {
            if (is_tx) g_st.tx_skipped++; else g_st.rx_skipped++;
            continue;
        }
        const uint8_t *sp = g_stage + g_off[k];
        uint8_t *dp = (uint8_t *) vec[i].msg_hdr.msg_iov[0].iov_base;
        const unsigned int tot = ((unsigned) sp[2] << 8) | sp[3];
        if (tot > lens[i]) g_status[k] |= TCPCSUM_PKT_SKIPPED;   /* claims more than was handed over */
        if (fill && !(g_status[k] & TCPCSUM_PKT_SKIPPED)) {
            const unsigned int tcp = (sp[0] & 15u) * 4u;
            memcpy(dp + tcp + 16, sp + tcp + 16, 2);
            if (g_iphdr) memcpy(dp + 10, sp + 10, 2);
        }
        account((int) k, fill, is_tx);
        ++k;
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
            if (gpu_batch(vec + done, cnt, lens, g_tx == MODE_FILL, 1)) return -1;
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
    if (r > 0 && g_rx == MODE_VERIFY && wants_fd(fd)) {
        unsigned int lens[1024];
        unsigned int done = 0;
        while (done < (unsigned int) r) {
            unsigned int cnt = (unsigned int) r - done < 1024 ? (unsigned int) r - done : 1024;
            for (unsigned int i = 0; i < cnt; ++i) lens[i] = vec[done + i].msg_len;
            if (gpu_batch(vec + done, cnt, lens, 0, 0)) return -1;
            pthread_mutex_lock(&g_mu);
            g_st.rx_batches++;
            g_st.rx_packets += cnt;
            pthread_mutex_unlock(&g_mu);
            done += cnt;
        }
    }
    return r;
}
