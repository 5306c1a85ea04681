/*
 * cpu_bench.inc.c — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * Textually included into a translation unit that already defines the two
 * checksum helpers, so that — exactly as in the reference, where the static
 * helpers are inlined into us_internal_socket_context_send_packet
 * (context.c:208-209) — the per-segment call can be inlined.
 *
 * The including TU (oracle/csum_oracle.c) defines:
 *   CB_PSEUDO(saddr, daddr, len_be)  -> unsigned long   (context.c:104 semantics)
 *   CB_CSUM(sum_start, ptr, nbytes)  -> unsigned short  (context.c:121 semantics)
 *   CB_BENCH_NAME                    exported symbol name of the harness
 *
 * Inputs are the SURVEY.md Appendix B synthetic stream (host-resident).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <stdint.h>
#include <arpa/inet.h>

static uint64_t cb_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void cb_fill(uint8_t *dst, uint64_t nbytes) {
    /* stream offset 0, nbytes multiple of 8 handled bytewise at the tail */
    uint64_t w = 0;
    for (; (w + 1) * 8 <= nbytes; ++w) {
        uint64_t v = cb_mix(0x5EEDC0DEull + (w + 1) * 0x9E3779B97F4A7C15ull);
        memcpy(dst + w * 8, &v, 8);
    }
    if (w * 8 < nbytes) {
        uint64_t v = cb_mix(0x5EEDC0DEull + (w + 1) * 0x9E3779B97F4A7C15ull);
        memcpy(dst + w * 8, &v, nbytes - w * 8);
    }
}

struct cb_job {
    const uint8_t *buf;
    uint32_t seg_len;
    uint64_t s0, s1;
    uint16_t *out;
};

static void *cb_worker(void *arg) {
    struct cb_job *j = (struct cb_job *) arg;
    const uint16_t len_be = htons((uint16_t) j->seg_len);
    for (uint64_t i = j->s0; i < j->s1; ++i) {
        uint32_t sa = htonl(0x0A000000u | (uint32_t) (i & 0xFFFFFFu));
        uint32_t da = htonl(0xC0A80000u | (uint32_t) ((i * 7u) & 0xFFFFu));
        j->out[i] = CB_CSUM(CB_PSEUDO(sa, da, len_be),
                            (char *) (j->buf + i * (uint64_t) j->seg_len), (int) j->seg_len);
    }
    return 0;
}

static double cb_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

double CB_BENCH_NAME(int nthreads, uint32_t seg_len, uint64_t nseg, double min_seconds,
                     uint64_t *digest_out, int *passes_out) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    uint64_t bytes = nseg * (uint64_t) seg_len;
    uint8_t *buf = (uint8_t *) aligned_alloc(64, (bytes + 63) & ~63ull);
    uint16_t *out = (uint16_t *) calloc(nseg ? nseg : 1, sizeof(uint16_t));
    if (!buf || !out) { free(buf); free(out); return -1.0; }
    cb_fill(buf, bytes);
    /* first-touch the output */
    memset(out, 0, nseg * sizeof(uint16_t));

    pthread_t th[256];
    struct cb_job jobs[256];
    double best = 1e300, total = 0.0;
    int passes = 0;
    while (passes < 3 || total < min_seconds) {
        double t0 = cb_now();
        for (int t = 0; t < nthreads; ++t) {
            jobs[t].buf = buf; jobs[t].seg_len = seg_len; jobs[t].out = out;
            jobs[t].s0 = nseg * (uint64_t) t / (uint64_t) nthreads;
            jobs[t].s1 = nseg * (uint64_t) (t + 1) / (uint64_t) nthreads;
            if (nthreads == 1) cb_worker(&jobs[t]);
            else pthread_create(&th[t], 0, cb_worker, &jobs[t]);
        }
        if (nthreads > 1)
            for (int t = 0; t < nthreads; ++t) pthread_join(th[t], 0);
        double dt = cb_now() - t0;
        total += dt;
        if (dt < best) best = dt;
        ++passes;
        if (passes > 100000) break;
    }
    if (digest_out) {
        uint64_t h = 0xcbf29ce484222325ull;
        for (uint64_t i = 0; i < nseg; ++i) {
            h = (h ^ (out[i] & 0xFF)) * 0x100000001b3ull;
            h = (h ^ (out[i] >> 8)) * 0x100000001b3ull;
        }
        *digest_out = h;
    }
    if (passes_out) *passes_out = passes;
    free(buf);
    free(out);
    return (double) bytes / best / (double) (1ull << 30);
}
