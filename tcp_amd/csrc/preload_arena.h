/*
 * preload_arena.h — the interposer's opt-in packet-buffer arena
 * (TCPCSUM_PRELOAD_POOL=1, tcp_amd/csrc/preload_mmsg.c).
 *
 * The reference allocates its packet buffers as 2 x 1024 separate
 * malloc(1024 * 32) calls (/root/reference/loop.c:180-183: buffer[i] for
 * recvmmsg, outBuffer[i] for sendmmsg). With the arena on, the interposer
 * answers exactly those requests — malloc of the arena's block size — from one
 * page-locked allocation the library made itself (tcpcsum_host_alloc), so the
 * loop's buffers are read and filled in place by the GPU with loop.c unedited.
 * Nothing foreign is page-locked (ABI v4): the arena's memory is the library's.
 *
 * This header is the bookkeeping only — no HIP, no libc malloc — so
 * tests/c/arena_test.c runs it under ASan/UBSan with ordinary memory standing
 * in for the page-locked block. Thread-safe; every function may be called from
 * any thread at any time, before arena_publish() too (the arena is then off:
 * nothing is owned, nothing is served).
 *
 *   arena_publish  hand the arena its memory (once; readers see all of it or none)
 *   arena_close    serve no more blocks (a forked child: the page-locked memory is
 *                  the parent's); blocks already out are still owned and released
 *   arena_alloc    a free block when size == block, else NULL (caller falls through
 *                  to libc); NULL too when every block is taken
 *   arena_owns     whether p lies inside the arena (free / realloc / usable-size
 *                  must route it here, never to libc)
 *   arena_release  return a block; p must be a block's start and in use — anything
 *                  else is heap corruption in the caller and aborts, as glibc's
 *                  free() does for an invalid or double-freed pointer
 *   arena_route_*  what the interposer's malloc / calloc / free / realloc do: arena blocks
 *                  here, everything else to the allocator underneath (libc's)
 */
#pragma once

#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ARENA_MAX_BLOCKS 2048u   /* 2 x 1024: loop.c's in- and out-buffers */

typedef struct {
    uint8_t *base;            /* published last (release); NULL: off */
    uint8_t *end;
    size_t block;
    uint32_t nblocks;
    uint32_t nfree;           /* entries of free_idx in use */
    uint32_t next_fresh;      /* blocks never handed out start here (ascending order) */
    uint16_t free_idx[ARENA_MAX_BLOCKS];
    uint8_t in_use[ARENA_MAX_BLOCKS];
    uint64_t served, released, full;   /* counters (under mu) */
    int closed;               /* arena_close: nothing more is served */
    pthread_mutex_t mu;
} arena_t;

#define ARENA_INIT {NULL, NULL, 0, 0, 0, 0, {0}, {0}, 0, 0, 0, 0, PTHREAD_MUTEX_INITIALIZER}

static inline uint8_t *arena_base(const arena_t *a) {
    return __atomic_load_n(&a->base, __ATOMIC_ACQUIRE);
}

/* mem: block * nblocks bytes, block-aligned blocks. Returns 0, or -1 when the
 * arguments are unusable (the arena stays off). Call once. */
static inline int arena_publish(arena_t *a, void *mem, size_t block, uint32_t nblocks) {
    if (!mem || !block || !nblocks || nblocks > ARENA_MAX_BLOCKS || arena_base(a)) return -1;
    pthread_mutex_lock(&a->mu);
    a->block = block;
    a->nblocks = nblocks;
    a->nfree = 0;
    a->next_fresh = 0;
    a->end = (uint8_t *) mem + block * nblocks;
    memset(a->in_use, 0, sizeof a->in_use);
    __atomic_store_n(&a->base, (uint8_t *) mem, __ATOMIC_RELEASE);
    pthread_mutex_unlock(&a->mu);
    return 0;
}

static inline void arena_close(arena_t *a) {
    __atomic_store_n(&a->closed, 1, __ATOMIC_RELEASE);
}

static inline int arena_owns(const arena_t *a, const void *p) {
    const uint8_t *b = arena_base(a);
    return b && (const uint8_t *) p >= b && (const uint8_t *) p < a->end;
}

/* The arena's block size (0 while off): what a served allocation may hold. */
static inline size_t arena_block(const arena_t *a) {
    return arena_base(a) ? a->block : 0;
}

static inline void *arena_alloc(arena_t *a, size_t size) {
    uint8_t *b = arena_base(a);
    if (!b || size != a->block || __atomic_load_n(&a->closed, __ATOMIC_ACQUIRE)) return NULL;
    pthread_mutex_lock(&a->mu);
    uint32_t idx;
    if (a->nfree) {
        idx = a->free_idx[--a->nfree];   /* LIFO: the block freed last is still warm */
    } else if (a->next_fresh < a->nblocks) {
        idx = a->next_fresh++;           /* fresh blocks in address order */
    } else {
        a->full++;
        pthread_mutex_unlock(&a->mu);
        return NULL;
    }
    a->in_use[idx] = 1;
    a->served++;
    pthread_mutex_unlock(&a->mu);
    return b + (size_t) idx * a->block;
}

static inline void arena_release(arena_t *a, void *p) {
    uint8_t *b = arena_base(a);
    const size_t off = (size_t) ((uint8_t *) p - b);
    if (!arena_owns(a, p) || off % a->block) abort();   /* free(): invalid pointer */
    const uint32_t idx = (uint32_t) (off / a->block);
    pthread_mutex_lock(&a->mu);
    if (!a->in_use[idx]) abort();                        /* free(): double free */
    a->in_use[idx] = 0;
    a->free_idx[a->nfree++] = (uint16_t) idx;
    a->released++;
    pthread_mutex_unlock(&a->mu);
}

/* Counters: blocks handed out, returned, and requests of the block size that
 * found the arena full (those went to libc: their packets are staged). */
static inline void arena_counters(arena_t *a, uint64_t *served, uint64_t *released, uint64_t *full) {
    pthread_mutex_lock(&a->mu);
    *served = a->served;
    *released = a->released;
    *full = a->full;
    pthread_mutex_unlock(&a->mu);
}

/* The allocator underneath (the interposer passes glibc's __libc_* entry points). */
typedef struct {
    void *(*malloc)(size_t);
    void (*free)(void *);
    void *(*realloc)(void *, size_t);
} arena_libc_t;

/* malloc: a block for a request of exactly the block size, unless guard (the
 * library's own thread: the runtime's allocations are not the loop's) or the
 * arena is full; everything else underneath. */
static inline void *arena_route_malloc(arena_t *a, size_t n, int guard, const arena_libc_t *l) {
    if (!guard && n && n == arena_block(a)) {
        void *p = arena_alloc(a, n);
        if (p) return p;
    }
    return l->malloc(n);
}

/* calloc: a zeroed block when nmemb * size is exactly the block size (a compiler may
 * turn the loop's malloc + memset into calloc), else underneath. */
static inline void *arena_route_calloc(arena_t *a, size_t nmemb, size_t size, int guard,
                                       void *(*under)(size_t, size_t)) {
    size_t n;
    if (!guard && !__builtin_mul_overflow(nmemb, size, &n) && n && n == arena_block(a)) {
        void *p = arena_alloc(a, n);
        if (p) return memset(p, 0, n);
    }
    return under(nmemb, size);
}

static inline void arena_route_free(arena_t *a, void *p, const arena_libc_t *l) {
    if (arena_owns(a, p)) arena_release(a, p);
    else l->free(p);
}

/* realloc of an arena block: kept when the new size fits the block, else moved
 * underneath (the block returned); size 0 frees it, as glibc's realloc does. */
static inline void *arena_route_realloc(arena_t *a, void *p, size_t n, const arena_libc_t *l) {
    if (!arena_owns(a, p)) return l->realloc(p, n);
    if (n == 0) {
        arena_release(a, p);
        return NULL;
    }
    const size_t blk = arena_block(a);
    if (n <= blk) return p;
    void *q = l->malloc(n);
    if (!q) return NULL;   /* p stays valid, as realloc promises */
    memcpy(q, p, blk);
    arena_release(a, p);
    return q;
}
