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

/* bytes [b0, b1) of the stream, written at dst + b0 */
static void cb_fill_range(uint8_t *dst, uint64_t b0, uint64_t b1) {
    uint64_t b = b0;
    for (; b < b1 && (b & 7); ++b)
        dst[b] = (uint8_t) (cb_mix(0x5EEDC0DEull + (b / 8 + 1) * 0x9E3779B97F4A7C15ull) >> (8 * (b & 7)));
    for (; b + 8 <= b1; b += 8) {
        uint64_t v = cb_mix(0x5EEDC0DEull + (b / 8 + 1) * 0x9E3779B97F4A7C15ull);
        memcpy(dst + b, &v, 8);
    }
    for (; b < b1; ++b)
        dst[b] = (uint8_t) (cb_mix(0x5EEDC0DEull + (b / 8 + 1) * 0x9E3779B97F4A7C15ull) >> (8 * (b & 7)));
}

struct cb_job {
    const uint8_t *buf;
    uint32_t seg_len;
    uint64_t s0, s1;
    uint16_t *out;
};

static void cb_work(const struct cb_job *j) {
    const uint16_t len_be = htons((uint16_t) j->seg_len);
    for (uint64_t i = j->s0; i < j->s1; ++i) {
        uint32_t sa = htonl(0x0A000000u | (uint32_t) (i & 0xFFFFFFu));
        uint32_t da = htonl(0xC0A80000u | (uint32_t) ((i * 7u) & 0xFFFFu));
        j->out[i] = CB_CSUM(CB_PSEUDO(sa, da, len_be),
                            (char *) (j->buf + i * (uint64_t) j->seg_len), (int) j->seg_len);
    }
}

/* A persistent pool: every pass is [barrier, work, barrier], so thread
 * creation is outside the timed passes (it would dominate at hundreds of
 * threads). Thread 0 is the caller. */
struct cb_pool {
    pthread_barrier_t start, done;
    volatile int stop;
    volatile int fill;   /* this round writes the thread's shard of the input instead */
};

struct cb_arg {
    struct cb_pool *pool;
    struct cb_job job;
};

/* One round of thread a: its shard of the checksums, or (fill round) its shard
 * of the input bytes — so every page is first touched by the thread that
 * later reads it (NUMA-local on a multi-socket host). */
static void cb_round(const struct cb_arg *a) {
    if (a->pool->fill)
        cb_fill_range((uint8_t *) a->job.buf, a->job.s0 * a->job.seg_len, a->job.s1 * a->job.seg_len);
    else
        cb_work(&a->job);
}

static void *cb_worker(void *arg) {
    struct cb_arg *a = (struct cb_arg *) arg;
    for (;;) {
        pthread_barrier_wait(&a->pool->start);
        if (a->pool->stop) break;
        cb_round(a);
        pthread_barrier_wait(&a->pool->done);
    }
    return 0;
}

static double cb_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

#define CB_MAX_THREADS 1024
#define CB_MAX_PASSES 4096

static int cb_cmp_double(const void *a, const void *b) {
    const double x = *(const double *) a, y = *(const double *) b;
    return x < y ? -1 : x > y;
}

/* Passes over the batch: at least 5 and min_seconds of them (at most
 * CB_MAX_PASSES). A pass is timed from just BEFORE thread 0 releases the
 * start barrier to just after the last thread reaches the done barrier, so a
 * worker that starts early (thread 0 preempted after the release) or late (a
 * cgroup quota throttling it) is inside the pass, never outside it. Returns
 * the best pass in GiB/s; *median_out = the median pass in GiB/s. */
double CB_BENCH_NAME(int nthreads, uint32_t seg_len, uint64_t nseg, double min_seconds,
                     uint64_t *digest_out, int *passes_out, double *total_out, double *median_out) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > CB_MAX_THREADS) nthreads = CB_MAX_THREADS;
    uint64_t bytes = nseg * (uint64_t) seg_len;
    uint8_t *buf = (uint8_t *) aligned_alloc(64, (bytes + 63) & ~63ull);
    uint16_t *out = (uint16_t *) calloc(nseg ? nseg : 1, sizeof(uint16_t));
    pthread_t *th = (pthread_t *) calloc((size_t) nthreads, sizeof(pthread_t));
    struct cb_arg *args = (struct cb_arg *) calloc((size_t) nthreads, sizeof(struct cb_arg));
    double *times = (double *) calloc(CB_MAX_PASSES, sizeof(double));
    if (!buf || !out || !th || !args || !times) {
        free(buf); free(out); free(th); free(args); free(times);
        return -1.0;
    }
    memset(out, 0, nseg * sizeof(uint16_t));   /* first-touch the output */

    struct cb_pool pool;
    pool.stop = 0;
    pool.fill = 1;
    pthread_barrier_init(&pool.start, 0, (unsigned) nthreads);
    pthread_barrier_init(&pool.done, 0, (unsigned) nthreads);
    for (int t = 0; t < nthreads; ++t) {
        args[t].pool = &pool;
        args[t].job.buf = buf; args[t].job.seg_len = seg_len; args[t].job.out = out;
        args[t].job.s0 = nseg * (uint64_t) t / (uint64_t) nthreads;
        args[t].job.s1 = nseg * (uint64_t) (t + 1) / (uint64_t) nthreads;
        if (t) pthread_create(&th[t], 0, cb_worker, &args[t]);
    }
    /* untimed: the fill round, then one warm pass */
    for (int r = 0; r < 2; ++r) {
        pthread_barrier_wait(&pool.start);
        cb_round(&args[0]);
        pthread_barrier_wait(&pool.done);
        pool.fill = 0;
    }
    double total = 0.0;
    int passes = 0;
    while ((passes < 5 || total < min_seconds) && passes < CB_MAX_PASSES) {
        double t0 = cb_now();
        pthread_barrier_wait(&pool.start);
        cb_round(&args[0]);
        pthread_barrier_wait(&pool.done);
        double dt = cb_now() - t0;
        times[passes++] = dt;
        total += dt;
    }
    pool.stop = 1;
    pthread_barrier_wait(&pool.start);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], 0);
    pthread_barrier_destroy(&pool.start);
    pthread_barrier_destroy(&pool.done);
    if (digest_out) {
        uint64_t h = 0xcbf29ce484222325ull;
        for (uint64_t i = 0; i < nseg; ++i) {
            h = (h ^ (out[i] & 0xFF)) * 0x100000001b3ull;
            h = (h ^ (out[i] >> 8)) * 0x100000001b3ull;
        }
        *digest_out = h;
    }
    qsort(times, (size_t) passes, sizeof(double), cb_cmp_double);
    const double best = times[0];
    const double med = passes & 1 ? times[passes / 2] : 0.5 * (times[passes / 2 - 1] + times[passes / 2]);
    if (passes_out) *passes_out = passes;
    if (total_out) *total_out = total;
    if (median_out) *median_out = (double) bytes / med / (double) (1ull << 30);
    free(buf);
    free(out);
    free(th);
    free(args);
    free(times);
    return (double) bytes / best / (double) (1ull << 30);
}
