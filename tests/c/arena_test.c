/*
 * arena_test.c — the interposer's packet-buffer arena (tcp_amd/csrc/preload_arena.h,
 * TCPCSUM_PRELOAD_POOL=1) under ASan/UBSan, with ordinary heap memory standing in
 * for the page-locked block and glibc's malloc as the allocator underneath.
 *
 *   * off until published: nothing owned, every request falls through;
 *   * the loop's 2 x 1024 malloc(32 KiB) (loop.c:180-183) are served in address
 *     order, the 2049th falls through, and so do other sizes and guarded calls;
 *   * free / realloc route arena pointers back to the arena (shrink in place,
 *     grow moves underneath with the contents, size 0 frees);
 *   * churn from 8 threads: no block is handed out twice (each holder's tag
 *     survives until it frees), counters balance;
 *   * an interior or double free aborts, as glibc's free() does;
 *   * closed (a forked child): nothing more is served, blocks already out are still
 *     owned and released.
 */
#define _GNU_SOURCE
#include <assert.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "../../tcp_amd/csrc/preload_arena.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); exit(1); } } while (0)

enum { BLK = 32768, NBLK = ARENA_MAX_BLOCKS, THREADS = 8, ITERS = 20000, HOLD = 1024 };   /* ~4000 held at a time: more than the 2048 blocks */

static arena_t A = ARENA_INIT;
static const arena_libc_t L = {malloc, free, realloc};

static void tag(void *p, size_t n, unsigned long v) {
    memcpy(p, &v, sizeof v);
    memcpy((char *) p + n - sizeof v, &v, sizeof v);
}
static int tagged(const void *p, size_t n, unsigned long v) {
    unsigned long a, b;
    memcpy(&a, p, sizeof a);
    memcpy(&b, (const char *) p + n - sizeof b, sizeof b);
    return a == v && b == v;
}

struct held { void *p; size_t n; unsigned long v; };

static void *churn(void *arg) {
    const unsigned long id = (unsigned long) (size_t) arg;
    unsigned int seed = (unsigned int) (id * 2654435761u + 1u);
    struct held h[HOLD];
    memset(h, 0, sizeof h);
    unsigned long serial = id << 40;
    for (int it = 0; it < ITERS; ++it) {
        struct held *s = &h[rand_r(&seed) % HOLD];
        const int op = rand_r(&seed) % 8;
        if (s->p) {
            CHECK(tagged(s->p, s->n, s->v));    /* nobody else was handed these bytes */
            if (op < 2) {                        /* realloc: shrink, same size or grow */
                const size_t n2 = op == 0 ? (size_t) BLK / 2 : (size_t) BLK + 100;
                void *q = arena_route_realloc(&A, s->p, n2, &L);
                CHECK(q);
                CHECK(tagged(q, sizeof(unsigned long), s->v));   /* contents move along */
                if (op == 0 && arena_owns(&A, s->p)) CHECK(q == s->p);
                s->p = q;
                s->n = n2 < s->n ? n2 : s->n;
                s->v = ++serial;
                tag(s->p, s->n, s->v);
            } else {
                arena_route_free(&A, s->p, &L);
                s->p = NULL;
            }
        } else {
            const size_t n = op < 6 ? (size_t) BLK : (size_t) (64 + rand_r(&seed) % 4000);   /* the loop's size, mostly */
            s->p = arena_route_malloc(&A, n, op == 5, &L);
            CHECK(s->p);
            if (op == 5) CHECK(!arena_owns(&A, s->p));   /* guarded: the runtime's, never the arena's */
            s->n = n;
            s->v = ++serial;
            tag(s->p, n, s->v);
        }
    }
    for (int i = 0; i < HOLD; ++i)
        if (h[i].p) {
            CHECK(tagged(h[i].p, h[i].n, h[i].v));
            arena_route_free(&A, h[i].p, &L);
        }
    return NULL;
}

static int dies_by_abort(void (*fn)(void *), void *arg) {
    fflush(NULL);
    const pid_t pid = fork();
    if (pid == 0) {
        fn(arg);
        _exit(0);
    }
    int st = 0;
    waitpid(pid, &st, 0);
    return WIFSIGNALED(st) && WTERMSIG(st) == SIGABRT;
}
static void free_interior(void *p) {
    void *volatile q = (char *) p + 16;   /* an interior pointer: what a corrupt caller would pass */
    arena_route_free(&A, q, &L);
}
static void free_twice(void *p) { arena_route_free(&A, p, &L); arena_route_free(&A, p, &L); }

int main(void) {
    /* off: nothing owned, everything underneath */
    void *x = arena_route_malloc(&A, BLK, 0, &L);
    CHECK(x && !arena_owns(&A, x) && arena_block(&A) == 0);
    arena_route_free(&A, x, &L);
    CHECK(!arena_owns(&A, NULL));
    void *z = arena_route_malloc(&A, 0, 0, &L);   /* malloc(0) never matches an off arena */
    CHECK(!arena_owns(&A, z));
    free(z);

    uint8_t *mem = aligned_alloc(4096, (size_t) BLK * NBLK);
    CHECK(mem);
    CHECK(arena_publish(&A, NULL, BLK, NBLK) == -1);
    CHECK(arena_publish(&A, mem, BLK, NBLK + 1) == -1);
    CHECK(arena_publish(&A, mem, BLK, NBLK) == 0);
    CHECK(arena_publish(&A, mem, BLK, NBLK) == -1);   /* once */
    CHECK(arena_block(&A) == BLK);

    /* the loop's allocation pattern: buffer[i], outBuffer[i] alternately */
    static void *buf[NBLK], *extra;
    for (unsigned i = 0; i < NBLK; ++i) {
        buf[i] = arena_route_malloc(&A, BLK, 0, &L);
        CHECK(buf[i] == mem + (size_t) i * BLK);        /* address order */
    }
    extra = arena_route_malloc(&A, BLK, 0, &L);        /* the 2049th: libc */
    void *cz = arena_route_calloc(&A, 8, BLK / 8, 0, calloc);   /* full: calloc falls through too */
    CHECK(cz && !arena_owns(&A, cz));
    free(cz);
    CHECK(extra && !arena_owns(&A, extra));
    void *small = arena_route_malloc(&A, 100, 0, &L);
    CHECK(small && !arena_owns(&A, small));
    uint64_t served, released, full;
    arena_counters(&A, &served, &released, &full);
    CHECK(served == NBLK && released == 0 && full == 2);   /* the 2049th malloc and the calloc */
    arena_route_free(&A, extra, &L);
    arena_route_free(&A, small, &L);

    /* realloc of a block: shrink keeps it, grow moves it (contents along), 0 frees */
    memset(buf[7], 0xab, BLK);
    CHECK(arena_route_realloc(&A, buf[7], 100, &L) == buf[7]);
    void *g = arena_route_realloc(&A, buf[7], 2 * BLK, &L);
    CHECK(g && !arena_owns(&A, g));
    for (size_t k = 0; k < BLK; ++k) CHECK(((uint8_t *) g)[k] == 0xab);
    free(g);
    CHECK(arena_route_malloc(&A, BLK, 0, &L) == buf[7]);   /* the freed block is reused first */
    CHECK(arena_route_realloc(&A, buf[9], 0, &L) == NULL);
    CHECK(arena_route_malloc(&A, BLK, 0, &L) == buf[9]);
    /* calloc of exactly a block: the block, zeroed (it held 0xab); other sizes underneath */
    memset(buf[11], 0xab, BLK);
    arena_route_free(&A, buf[11], &L);
    uint8_t *c = arena_route_calloc(&A, BLK / 16, 16, 0, calloc);
    CHECK(c == buf[11]);
    for (size_t k = 0; k < BLK; ++k) CHECK(c[k] == 0);
    void *c2 = arena_route_calloc(&A, 3, BLK, 0, calloc);
    CHECK(c2 && !arena_owns(&A, c2));
    free(c2);
    void *r = arena_route_realloc(&A, NULL, BLK, &L);     /* realloc(NULL, n) is malloc underneath */
    CHECK(r && !arena_owns(&A, r));
    free(r);

    for (unsigned i = 0; i < NBLK; ++i) arena_route_free(&A, buf[i], &L);

    /* corruption aborts instead of handing a block out twice */
    void *v = arena_route_malloc(&A, BLK, 0, &L);
    CHECK(arena_owns(&A, v));
    CHECK(dies_by_abort(free_interior, v));
    CHECK(dies_by_abort(free_twice, v));
    arena_route_free(&A, v, &L);

    /* churn: more holders than blocks, so the arena runs full and falls through too */
    pthread_t th[THREADS];
    for (unsigned long t = 0; t < THREADS; ++t) CHECK(pthread_create(&th[t], NULL, churn, (void *) (size_t) t) == 0);
    for (int t = 0; t < THREADS; ++t) pthread_join(th[t], NULL);
    arena_counters(&A, &served, &released, &full);
    CHECK(served == released && full > 1);   /* churn ran the arena full: the rest fell through */

    /* closed: blocks out before stay the arena's, nothing new is served */
    void *k = arena_route_malloc(&A, BLK, 0, &L);
    CHECK(arena_owns(&A, k));
    arena_close(&A);
    void *after = arena_route_malloc(&A, BLK, 0, &L);
    void *afterc = arena_route_calloc(&A, 1, BLK, 0, calloc);
    CHECK(after && !arena_owns(&A, after) && afterc && !arena_owns(&A, afterc));
    free(after);
    free(afterc);
    CHECK(arena_route_realloc(&A, k, 64, &L) == k);       /* still a block: shrink keeps it */
    arena_route_free(&A, k, &L);
    void *again = arena_route_malloc(&A, BLK, 0, &L);     /* the freed block is not served again */
    CHECK(again && again != k && !arena_owns(&A, again));
    free(again);
    uint64_t s2, r2, f2;
    arena_counters(&A, &s2, &r2, &f2);
    CHECK(s2 == served + 1 && r2 == released + 1);
    printf("arena_test: served=%llu full=%llu OK\n", (unsigned long long) served, (unsigned long long) full);
    free(mem);
    return 0;
}
