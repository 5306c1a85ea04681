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
 *   TCPCSUM_PRELOAD_DEVICE=<k>   the GPU this process's batches run on (default 0):
 *                                one loop process per GPU on a multi-GPU node
 *   TCPCSUM_PRELOAD_POOL=<prog>  zero copy with loop.c unedited: malloc(32 KiB) —
 *                                the loop's 2 x 1024 packet buffers, loop.c:180-183 —
 *                                is served from one page-locked block the library
 *                                allocates itself (tcpcsum_host_alloc, 64 MiB) before
 *                                main runs, so both seams read and fill the loop's
 *                                buffers in place (preload_arena.h). Every other
 *                                allocation, and any past the first 2048 of that
 *                                size, goes to libc (calloc of exactly 32 KiB is
 *                                served too, zeroed: a compiler may turn malloc +
 *                                memset into it); free / realloc / reallocarray /
 *                                malloc_usable_size route arena pointers back here.
 *                                <prog> is the loop's executable name ("stress"), or
 *                                1 for whatever process loads the interposer. The pool
 *                                initialises HIP in a constructor, and a process that
 *                                has done so must not exec: name the program, or put
 *                                LD_PRELOAD on the loop binary itself, never on a
 *                                wrapper (timeout, a shell). The process that takes the
 *                                pool removes the variable from its environment before
 *                                HIP starts, so its children do not inherit it.
 *   fork: a child of a process whose interposer started HIP (the pool, or a GPU batch)
 *   has no GPU path — HIP does not survive fork — so its seams fail with ENXIO; its
 *   mallocs go to libc (the arena is closed in the child), and it must not touch the
 *   parent's arena buffers (page-locked memory need not be inherited), though freeing
 *   them is allowed (bookkeeping only).
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
 * equal the un-complemented pseudo-header fold is therefore rejected. That
 * argument holds for AF_INET sockets on hosts without route_localnet (which
 * lets 127/8 in on other interfaces; kube-proxy sets it) only: for any other
 * socket family (AF_PACKET sees frames before the martian filter) or when any
 * interface has net.ipv4.conf.*.route_localnet=1 (read once, at the first
 * call), there is no exception and a CHECKSUM_PARTIAL segment counts as failed.
 * Messages that are not IPv4/TCP are passed through untouched (the reference
 * filters them itself, loop.c:319). IPv4/TCP messages the library cannot
 * verify — truncated (tot_len past the bytes received), bad IHL or lengths —
 * are counted as skipped; in drop mode they are dropped, since they would
 * reach the application's TCP handler unverified. A message with several
 * iovecs (the reference uses one, loop.c:187-188) is checked from its first
 * iovec when that holds the whole packet; otherwise it is skipped and, in drop
 * mode, passed through unverified (a scatter read the library cannot see whole).
 */
/*
 * Built twice (Makefile): as the LD_PRELOAD library above, and with
 * -DTCPCSUM_WRAP as tcp_amd/libtcpcsum_wrap.a for the link-time seam SURVEY.md
 * §8(b)(ii) names — link the loop with
 *     -Wl,--wrap=sendmmsg,--wrap=recvmmsg  (+ ,--wrap=malloc,--wrap=calloc,--wrap=free,--wrap=realloc
 *                                           for TCPCSUM_PRELOAD_POOL: all four, or none)
 *     tcp_amd/libtcpcsum_wrap.a -ltcpcsum -ldl -lpthread
 * and the same entry points become __wrap_sendmmsg / __wrap_recvmmsg (the real
 * calls __real_*). The archive holds two members: the seams
 * (TCPCSUM_WRAP_PART=1) and the arena's allocation wraps with the pool's
 * constructor (TCPCSUM_WRAP_PART=2), which the linker pulls in only when
 * --wrap=malloc makes the loop reference __wrap_malloc — so the two mmsg wraps
 * alone link too (tests/c/mmsg_loop_wrap_nopool). The arena then serves only the
 * wrapped objects' own mallocs — the loop's, never the HIP runtime's. The
 * environment variables are the same.
 *
 * Allocations the arena never serves (the LD_PRELOAD build, where every malloc
 * of the process passes through it): those of a thread inside a library call
 * (t_guard: the constructor's HIP start-up, a GPU batch), of a thread the
 * library started (tcpcsum_on_library_thread: its copy threads), and of a
 * thread created by the GPU runtime or by a guarded thread (pthread_create is
 * interposed while the pool is on: HIP's worker and host-callback threads are
 * marked for life). And a process whose interposer started HIP refuses to exec
 * (execve and its family fail with EPERM: on this hardware an exec after the GPU
 * was opened takes the machine down); its forked children may exec.
 */
#define _GNU_SOURCE
#include <dirent.h>
#include <dlfcn.h>
#include <alloca.h>
#include <errno.h>
#include <execinfo.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include "preload_arena.h"
#include "rx_compact.h"
#include "tcpcsum.h"

/* The preload build is one object with everything; the wrap build two archive members
 * (above) that share the arena, the guard flag and the HIP owner's pid by name. */
#ifndef TCPCSUM_WRAP
#define PART_SEAMS 1
#define PART_ALLOC 1
#define SHARED static
#elif TCPCSUM_WRAP_PART == 1
#define PART_SEAMS 1
#define PART_ALLOC 0
#define SHARED
#elif TCPCSUM_WRAP_PART == 2
#define PART_SEAMS 0
#define PART_ALLOC 1
#define SHARED extern
#else
#error "TCPCSUM_WRAP builds need TCPCSUM_WRAP_PART=1 (seams) or 2 (allocation wraps)"
#endif
#ifdef TCPCSUM_WRAP
#define g_arena tcpcsum_wrap_arena
#define t_guard tcpcsum_wrap_guard
#define g_hip_pid tcpcsum_wrap_hip_pid
#endif

typedef int (*sendmmsg_fn)(int, struct mmsghdr *, unsigned int, int);
typedef int (*recvmmsg_fn)(int, struct mmsghdr *, unsigned int, int, struct timespec *);
typedef size_t (*usable_fn)(void *);

enum { MODE_OFF = 0, MODE_FILL = 1, MODE_VERIFY = 2, MODE_DROP = 3 };

struct tcpcsum_preload_stats {
    unsigned long long tx_batches, tx_packets, tx_filled, tx_verified, tx_verify_failed, tx_skipped;
    unsigned long long rx_batches, rx_packets, rx_verified, rx_verify_failed, rx_skipped, rx_partial, rx_dropped;
    unsigned long long errors;
};

#if PART_SEAMS
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static sendmmsg_fn real_sendmmsg;
static recvmmsg_fn real_recvmmsg;
static int g_tx = MODE_FILL, g_rx = MODE_OFF, g_iphdr, g_any, g_stats, g_device, g_localnet;
static tcpcsum_ctx_t *g_ctx;
static int g_ctx_failed;
static int g_forked;        /* a forked child of a process that had started HIP */
static uint16_t *g_out;     /* pinned: the kernel writes results straight here */
static uint8_t *g_status;
static struct tcpcsum_preload_stats g_st;
#endif

/* ------------------------------------------------------------------ the arena
 * TCPCSUM_PRELOAD_POOL: malloc(kPoolBlock) served from page-locked memory the
 * library owns (preload_arena.h). t_guard: this thread is inside the library
 * (the constructor's HIP start-up, a GPU batch) — its allocations of the block
 * size are the runtime's, not the loop's, and go to libc. */
enum { kPoolBlock = 1024 * 32 };   /* loop.c:181-182 */
#if PART_SEAMS
SHARED arena_t g_arena = ARENA_INIT;
SHARED __thread int t_guard __attribute__((tls_model("initial-exec")));
SHARED pid_t g_hip_pid;     /* the process whose interposer started HIP (it must not exec) */
#else
SHARED arena_t g_arena;
SHARED __thread int t_guard __attribute__((tls_model("initial-exec")));
SHARED pid_t g_hip_pid;
#endif
#if PART_ALLOC
static int g_pool_on;       /* the pool was wanted in this process: mark runtime threads */
#endif

extern void *__libc_malloc(size_t);
extern void __libc_free(void *);
extern void *__libc_realloc(void *, size_t);
extern void *__libc_calloc(size_t, size_t);

#ifdef TCPCSUM_WRAP
/* link-time seam: the wrapped objects' calls land here, the rest of the process
 * (HIP included) keeps libc's allocator untouched */
#define SEAM(fn) __wrap_##fn
#define UNDER(fn) __real_##fn
void *__real_malloc(size_t);
void __real_free(void *);
void *__real_realloc(void *, size_t);
void *__real_calloc(size_t, size_t);
int __real_sendmmsg(int, struct mmsghdr *, unsigned int, int);
int __real_recvmmsg(int, struct mmsghdr *, unsigned int, int, struct timespec *);
#else
#define SEAM(fn) fn
#define UNDER(fn) __libc_##fn
#endif

#if PART_ALLOC
static const arena_libc_t k_libc = {UNDER(malloc), UNDER(free), UNDER(realloc)};

#ifndef TCPCSUM_WRAP
/* Whether code address ra lies in the GPU runtime or in libtcpcsum itself. */
static int runtime_caller(const void *ra) {
    static const char *const libs[] = {"libamdhip64", "libhsa-runtime64", "libhsakmt", "libtcpcsum.",
                                       "librocprofiler", "libroctracer", "libamd_comgr"};
    Dl_info di;
    if (!ra || !dladdr(ra, &di) || !di.dli_fname) return 0;
    const char *b = strrchr(di.dli_fname, '/');
    b = b ? b + 1 : di.dli_fname;
    for (size_t i = 0; i < sizeof libs / sizeof libs[0]; ++i)
        if (!strncmp(b, libs[i], strlen(libs[i]))) return 1;
    return 0;
}

/* Whether any of the caller's frames (up to 16; through operator new and the like)
 * lies in the runtime: an allocation the GPU runtime makes on an application thread,
 * inside a HIP call the application made itself. */
static int runtime_on_stack(void) {
    void *fr[16];
    const int n = backtrace(fr, 16);
    for (int i = 2; i < n; ++i)
        if (runtime_caller(fr[i])) return 1;
    return 0;
}
#endif

/* Whether a request of the block size comes from the library's or the runtime's side
 * (never served): asked only for that size, once the arena is on. The preload sees
 * every allocation of the process, the runtime's made on the application's threads
 * too; the wrap build only the wrapped objects' own. */
static int guarded(void) {
#ifndef TCPCSUM_WRAP
    return t_guard || tcpcsum_on_library_thread() || runtime_on_stack();
#else
    return t_guard || tcpcsum_on_library_thread();
#endif
}

void *SEAM(malloc)(size_t n) {
    return arena_route_malloc(&g_arena, n, n == arena_block(&g_arena) && guarded(), &k_libc);
}

void *SEAM(calloc)(size_t nmemb, size_t size) {
    size_t n;
    const int big = !__builtin_mul_overflow(nmemb, size, &n) && n == arena_block(&g_arena);
    return arena_route_calloc(&g_arena, nmemb, size, big && guarded(), UNDER(calloc));
}

void SEAM(free)(void *p) {
    arena_route_free(&g_arena, p, &k_libc);
}

void *SEAM(realloc)(void *p, size_t n) {
    return arena_route_realloc(&g_arena, p, n, &k_libc);
}

#ifndef TCPCSUM_WRAP
/* glibc's reallocarray calls its own realloc internally, which must never see an
 * arena pointer */
void *reallocarray(void *p, size_t nmemb, size_t size) {
    size_t n;
    if (__builtin_mul_overflow(nmemb, size, &n)) {
        errno = ENOMEM;
        return NULL;
    }
    return realloc(p, n);
}

size_t malloc_usable_size(void *p) {
    if (arena_owns(&g_arena, p)) return arena_block(&g_arena);
    static usable_fn real_usable;
    usable_fn f = __atomic_load_n(&real_usable, __ATOMIC_ACQUIRE);
    if (!f) {
        f = (usable_fn) dlsym(RTLD_NEXT, "malloc_usable_size");
        __atomic_store_n(&real_usable, f, __ATOMIC_RELEASE);
    }
    return f ? f(p) : 0;
}
#endif

/* TCPCSUM_PRELOAD_POOL names the process the pool is for: "1" any process that
 * loads the interposer, else the basename of its executable ("stress") — so a
 * wrapper the preload also reaches (timeout, a shell) neither consumes the
 * variable nor starts HIP. */
static int pool_wanted(const char *v) {
    if (!v || !*v || !strcmp(v, "0")) return 0;
    if (!strcmp(v, "1")) return 1;
    char exe[4096];
    const ssize_t n = readlink("/proc/self/exe", exe, sizeof exe - 1);
    if (n <= 0) return 0;
    exe[n] = 0;
    const char *base = strrchr(exe, '/');
    return !strcmp(base ? base + 1 : exe, v);
}

/* Before main: the pool's page-locked block, so HIP never starts inside a malloc
 * call. Dependencies' constructors (the HIP runtime's) have run by now. */
__attribute__((constructor)) static void pool_ctor(void) {
    if (!pool_wanted(getenv("TCPCSUM_PRELOAD_POOL"))) return;
    unsetenv("TCPCSUM_PRELOAD_POOL");   /* children (an exec'd shell, say) never start HIP for it */
    /* the GPU the batches will run on (TCPCSUM_PRELOAD_DEVICE, read again by the seams):
     * the block is allocated for it, on its NUMA node */
    const char *dv = getenv("TCPCSUM_PRELOAD_DEVICE");
    const int dev = dv && *dv ? atoi(dv) : 0;
    g_pool_on = 1;
#ifndef TCPCSUM_WRAP
    void *fr[2];
    (void) backtrace(fr, 2);   /* the unwinder is loaded now, never first inside a malloc */
#endif
    __atomic_store_n(&g_hip_pid, getpid(), __ATOMIC_RELEASE);   /* from here on HIP may be up: no exec */
    t_guard = 1;
    void *mem = tcpcsum_host_alloc_on(dev, (size_t) kPoolBlock * ARENA_MAX_BLOCKS);
    t_guard = 0;
    if (!mem || arena_publish(&g_arena, mem, kPoolBlock, ARENA_MAX_BLOCKS)) {
        fprintf(stderr, "tcpcsum_preload: TCPCSUM_PRELOAD_POOL: no page-locked pool on device %d (%s); the loop's "
                        "buffers stay malloc'd and are copied into staging\n", dev,
                mem ? "publish failed" : tcpcsum_strerror(TCPCSUM_ENOMEM));
    }
}
#endif /* PART_ALLOC */

#if PART_SEAMS

/* fork: the handlers hold the interposer's locks across it, so the child never
 * inherits one taken mid-update; the child then gives up the GPU path and the arena
 * if the parent had started HIP for them. */
static void fork_prepare(void) {
    pthread_mutex_lock(&g_mu);
    pthread_mutex_lock(&g_arena.mu);
}

static void fork_parent(void) {
    pthread_mutex_unlock(&g_arena.mu);
    pthread_mutex_unlock(&g_mu);
}

static void fork_child(void) {
    pthread_mutex_unlock(&g_arena.mu);
    if (g_ctx || arena_base(&g_arena)) {
        arena_close(&g_arena);
        g_ctx = NULL;   /* the parent's: not usable, not destroyable here */
        g_out = NULL;
        g_status = NULL;
        g_ctx_failed = 1;
        g_forked = 1;
        g_stats = 0;    /* the counters are the parent's */
    }
    pthread_mutex_unlock(&g_mu);
}

__attribute__((constructor)) static void fork_ctor(void) {
    pthread_atfork(fork_prepare, fork_parent, fork_child);
}

#ifndef TCPCSUM_WRAP
/* ------------------------------------------------------------------ exec guard
 * A process whose interposer started HIP (the pool's constructor, or the first GPU
 * batch) must not replace itself with another program: on this hardware that takes
 * the machine down. LD_PRELOAD exported in a shell reaches wrappers (timeout, env,
 * a shell) that exec; with TCPCSUM_PRELOAD_POOL=1 they would start HIP and then exec.
 * Every exec entry point of this process fails with EPERM instead; a forked child
 * (another pid) may exec as usual. */
static int exec_refused(const char *what) {
    if (__atomic_load_n(&g_hip_pid, __ATOMIC_ACQUIRE) != getpid()) return 0;
    fprintf(stderr, "tcpcsum_preload: %s refused: this process started HIP for the GPU checksum path and must not "
                    "exec (fork first; put LD_PRELOAD on the loop binary, not on a wrapper)\n", what);
    errno = EPERM;
    return 1;
}

static void *next_sym(void **slot, const char *name) {
    void *f = __atomic_load_n(slot, __ATOMIC_ACQUIRE);
    if (!f) {
        f = dlsym(RTLD_NEXT, name);
        __atomic_store_n(slot, f, __ATOMIC_RELEASE);
    }
    return f;
}
#define NEXT(type, name) ((type) next_sym(&next_##name, #name))
static void *next_execve, *next_execv, *next_execvp, *next_execvpe, *next_fexecve, *next_execveat;
typedef int (*execve_fn)(const char *, char *const[], char *const[]);
typedef int (*execv_fn)(const char *, char *const[]);
typedef int (*fexecve_fn)(int, char *const[], char *const[]);
typedef int (*execveat_fn)(int, const char *, char *const[], char *const[], int);

int execve(const char *path, char *const argv[], char *const envp[]) {
    return exec_refused("execve") ? -1 : NEXT(execve_fn, execve)(path, argv, envp);
}
int execv(const char *path, char *const argv[]) {
    return exec_refused("execv") ? -1 : NEXT(execv_fn, execv)(path, argv);
}
int execvp(const char *file, char *const argv[]) {
    return exec_refused("execvp") ? -1 : NEXT(execv_fn, execvp)(file, argv);
}
int execvpe(const char *file, char *const argv[], char *const envp[]) {
    return exec_refused("execvpe") ? -1 : NEXT(execve_fn, execvpe)(file, argv, envp);
}
int fexecve(int fd, char *const argv[], char *const envp[]) {
    return exec_refused("fexecve") ? -1 : NEXT(fexecve_fn, fexecve)(fd, argv, envp);
}
int execveat(int dirfd, const char *path, char *const argv[], char *const envp[], int flags) {
    return exec_refused("execveat") ? -1 : NEXT(execveat_fn, execveat)(dirfd, path, argv, envp, flags);
}

/* execl / execlp / execle: glibc's call execve internally (not through this
 * library), so they are answered here: the list becomes a vector. */
#define EXECL_ARGV(arg, ap, argv, envp_out)                                  \
    size_t n_ = 1;                                                           \
    {                                                                        \
        va_list c_;                                                          \
        va_copy(c_, ap);                                                     \
        while (va_arg(c_, const char *)) ++n_;                               \
        va_end(c_);                                                          \
    }                                                                        \
    char **argv = alloca((n_ + 1) * sizeof(char *));                         \
    argv[0] = (char *) (arg);                                                \
    for (size_t i_ = 1; i_ <= n_; ++i_) argv[i_] = va_arg(ap, char *);       \
    envp_out

int execl(const char *path, const char *arg, ...) {
    if (exec_refused("execl")) return -1;
    va_list ap;
    va_start(ap, arg);
    EXECL_ARGV(arg, ap, argv, ;);
    va_end(ap);
    return NEXT(execv_fn, execv)(path, argv);
}
int execlp(const char *file, const char *arg, ...) {
    if (exec_refused("execlp")) return -1;
    va_list ap;
    va_start(ap, arg);
    EXECL_ARGV(arg, ap, argv, ;);
    va_end(ap);
    return NEXT(execv_fn, execvp)(file, argv);
}
int execle(const char *path, const char *arg, ...) {
    if (exec_refused("execle")) return -1;
    va_list ap;
    va_start(ap, arg);
    EXECL_ARGV(arg, ap, argv, char *const *envp = va_arg(ap, char *const *););
    va_end(ap);
    return NEXT(execve_fn, execve)(path, argv, envp);
}

/* ------------------------------------------------------------------ runtime threads
 * While the pool is on, a thread created by a guarded thread (inside a library call:
 * the copy threads, HIP's threads started with it) or by the GPU runtime itself (HIP's
 * host-callback and worker threads, whenever they start) is guarded for life: its
 * allocations of the block size are the runtime's, not the loop's. */
typedef int (*pthread_create_fn)(pthread_t *, const pthread_attr_t *, void *(*)(void *), void *);
static void *next_pthread_create;
struct guarded_start {
    void *(*fn)(void *);
    void *arg;
};

static void *guarded_thread(void *p) {
    struct guarded_start st = *(struct guarded_start *) p;
    __libc_free(p);
    t_guard = 1;
    return st.fn(st.arg);
}

int pthread_create(pthread_t *th, const pthread_attr_t *attr, void *(*fn)(void *), void *arg) {
    pthread_create_fn real = NEXT(pthread_create_fn, pthread_create);
    if (__atomic_load_n(&g_pool_on, __ATOMIC_ACQUIRE) &&
        (t_guard || runtime_caller(__builtin_extract_return_addr(__builtin_return_address(0))))) {
        struct guarded_start *st = (struct guarded_start *) __libc_malloc(sizeof *st);
        if (st) {
            st->fn = fn;
            st->arg = arg;
            const int rc = real(th, attr, guarded_thread, st);
            if (rc) __libc_free(st);
            return rc;
        }
    }
    return real(th, attr, fn, arg);
}

/* Exported for tests: whether the calling thread's block-size allocations are kept
 * from the arena. */
int tcpcsum_preload_thread_guarded(void) {
    return t_guard || tcpcsum_on_library_thread();
}
#endif /* !TCPCSUM_WRAP */

/* ------------------------------------------------------------------ seams */
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

/* Whether any interface has net.ipv4.conf.<if>.route_localnet = 1 ("all" included):
 * 127/8 may then arrive on interfaces other than lo. */
static int any_route_localnet(void) {
    DIR *d = opendir("/proc/sys/net/ipv4/conf");
    if (!d) return 0;
    int any = 0;
    for (struct dirent *e; !any && (e = readdir(d));) {
        if (e->d_name[0] == '.' || !strcmp(e->d_name, "lo")) continue;
        char path[320];
        snprintf(path, sizeof path, "/proc/sys/net/ipv4/conf/%s/route_localnet", e->d_name);
        FILE *f = fopen(path, "r");
        if (!f) continue;
        int v = 0;
        if (fscanf(f, "%d", &v) == 1 && v) any = 1;
        fclose(f);
    }
    closedir(d);
    return any;
}

static void print_stats(void) {
    if (!g_stats) return;
    tcpcsum_ctx_stats_t cs;
    memset(&cs, 0, sizeof cs);
    uint64_t served = 0, released = 0, full = 0;
    arena_counters(&g_arena, &served, &released, &full);
    pthread_mutex_lock(&g_mu);
    if (g_ctx) tcpcsum_ctx_get_stats(g_ctx, &cs);
    pthread_mutex_unlock(&g_mu);
    fprintf(stderr,
            "tcpcsum_preload: tx batches=%llu packets=%llu filled=%llu verified=%llu verify_failed=%llu "
            "skipped=%llu | rx batches=%llu packets=%llu verified=%llu verify_failed=%llu skipped=%llu "
            "partial=%llu dropped=%llu | errors=%llu | ctx in_place=%llu staged=%llu copy_threads=%llu "
            "cpu_caller_us=%llu cpu_workers_us=%llu | pool on=%d served=%llu released=%llu full=%llu "
            "device=%d localnet=%d\n",
            g_st.tx_batches, g_st.tx_packets, g_st.tx_filled, g_st.tx_verified, g_st.tx_verify_failed,
            g_st.tx_skipped, g_st.rx_batches, g_st.rx_packets, g_st.rx_verified, g_st.rx_verify_failed,
            g_st.rx_skipped, g_st.rx_partial, g_st.rx_dropped, g_st.errors,
            (unsigned long long) cs.pkts_in_place, (unsigned long long) cs.pkts_staged,
            (unsigned long long) cs.copy_threads, (unsigned long long) (cs.ns_cpu_caller / 1000),
            (unsigned long long) (cs.ns_cpu_workers / 1000), arena_base(&g_arena) != NULL,
            (unsigned long long) served, (unsigned long long) released, (unsigned long long) full, g_device,
            g_localnet);
}

static void init_once(void) {
#ifdef TCPCSUM_WRAP
    real_sendmmsg = __real_sendmmsg;
    real_recvmmsg = __real_recvmmsg;
#else
    real_sendmmsg = (sendmmsg_fn) dlsym(RTLD_NEXT, "sendmmsg");
    real_recvmmsg = (recvmmsg_fn) dlsym(RTLD_NEXT, "recvmmsg");
#endif
    g_tx = env_mode("TCPCSUM_PRELOAD_TX", MODE_FILL);
    if (g_tx == MODE_DROP) g_tx = MODE_VERIFY;   /* never drop what the application sends */
    g_rx = env_mode("TCPCSUM_PRELOAD_RX", MODE_OFF);
    g_iphdr = env_flag("TCPCSUM_PRELOAD_IPHDR");
    g_any = env_flag("TCPCSUM_PRELOAD_ANY_SOCKET");
    g_stats = env_flag("TCPCSUM_PRELOAD_STATS");
    const char *dv = getenv("TCPCSUM_PRELOAD_DEVICE");
    g_device = dv && *dv ? atoi(dv) : 0;
    g_localnet = g_rx != MODE_OFF && any_route_localnet();
    if (g_localnet)
        fprintf(stderr, "tcpcsum_preload: route_localnet is set on this host: CHECKSUM_PARTIAL segments get no "
                        "loopback exception\n");
    if (env_flag("TCPCSUM_PRELOAD_INPLACE"))
        fprintf(stderr, "tcpcsum_preload: TCPCSUM_PRELOAD_INPLACE is gone (ABI v4): buffers from "
                        "tcpcsum_host_alloc (or TCPCSUM_PRELOAD_POOL=1) are filled in place, all others are copied\n");
    atexit(print_stats);
}

/* Exported for tests: whether p is one of the pool's blocks. */
int tcpcsum_preload_pool_owns(const void *p) {
    return arena_owns(&g_arena, p);
}

/* Exported for tests / the application: a copy of the counters. */
void tcpcsum_preload_get_stats(struct tcpcsum_preload_stats *out) {
    pthread_mutex_lock(&g_mu);
    if (out) *out = g_st;
    pthread_mutex_unlock(&g_mu);
}

static int sock_opt(int fd, int opt) {
    int v = -1;
    socklen_t len = sizeof v;
    return getsockopt(fd, SOL_SOCKET, opt, &v, &len) == 0 ? v : -1;
}

static int wants_fd(int fd) {
    return g_any || sock_opt(fd, SO_TYPE) == SOCK_RAW;
}

/* g_mu held. */
static int ensure_ctx(void) {
    if (g_forked == 1) {
        fprintf(stderr, "tcpcsum_preload: forked child of a process that started HIP: no GPU path here; refusing to "
                        "send/accept packets with unchecked checksums\n");
        g_forked = 2;   /* said once */
    }
    if (g_ctx_failed) return -1;
    if (!g_ctx) {
        __atomic_store_n(&g_hip_pid, getpid(), __ATOMIC_RELEASE);   /* HIP starts here: no exec from now on */
        int rc = tcpcsum_ctx_create(g_device, 0, &g_ctx);
        const char *w = getenv("TCPCSUM_PRELOAD_WAIT");
        if (!rc && !(w && !strcmp(w, "spin"))) rc = tcpcsum_ctx_set_flags(g_ctx, TCPCSUM_CTX_BLOCKING_WAIT);
        if (!rc) {
            g_out = (uint16_t *) tcpcsum_host_alloc(1024 * sizeof(uint16_t));
            g_status = (uint8_t *) tcpcsum_host_alloc(1024);
            if (!g_out || !g_status) rc = TCPCSUM_ENOMEM;
        }
        if (rc) {
            fprintf(stderr, "tcpcsum_preload: GPU checksum path unavailable on device %d (%s); refusing to "
                            "send/accept packets with unchecked checksums\n", g_device, tcpcsum_strerror(rc));
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
 * accounting. p / len: its bytes as the GPU batch saw them; multi: it had several
 * iovecs; partial_ok: the socket may claim the loopback CHECKSUM_PARTIAL exception. */
static int account(int k, int fill, int is_tx, const uint8_t *p, uint32_t len, int multi, int partial_ok) {
    const int skipped = (g_status[k] & TCPCSUM_PKT_SKIPPED) != 0;
    if (skipped) {
        if (is_tx) g_st.tx_skipped++; else g_st.rx_skipped++;
        /* an IPv4/TCP segment that could not be verified (truncated, bad IHL or
         * lengths) is not passed on unverified in drop mode; a scatter read
         * (several iovecs, the first not holding the packet) and anything that is
         * not TCP go through (the reference filters the latter, loop.c:319) */
        return !(g_rx == MODE_DROP && !is_tx && !multi && is_ipv4_tcp(p, len));
    }
    if (fill) {
        g_st.tx_filled++;
        return 1;
    }
    /* CHECKSUM_PARTIAL segments (checksum left to offload, Linux loopback;
     * SURVEY.md §4.5) are counted apart, not as corrupt — on 127/8 only */
    const int partial = partial_ok && (g_status[k] & TCPCSUM_PKT_CSUM_PARTIAL) != 0 && loopback_pair(p);
    const int bad = (g_out[k] != 0 && !partial) || (g_status[k] & TCPCSUM_PKT_IPHDR_BAD);
    if (is_tx) { g_st.tx_verified++; if (bad) g_st.tx_verify_failed++; }
    else { g_st.rx_verified++; if (bad) g_st.rx_verify_failed++; if (partial) g_st.rx_partial++; }
    return !bad;
}

/* Checksum a batch of <= 1024 messages on the GPU, each from its first iovec
 * (one iov_base per message: the reference's layout, loop.c:53-54). lens: the
 * bytes of that iovec worth reading (iov_len for tx, msg_len bounded by iov_len
 * for rx); a packet longer than that is SKIPPED. fill: store the checks in the
 * caller's buffers. keep (nullable): per message, whether it passed. partial_ok:
 * see account(). Returns 0, or -1 with errno set. */
static int gpu_batch(struct mmsghdr *vec, unsigned int vlen, const unsigned int *lens, int fill, int is_tx,
                     unsigned char *keep, int partial_ok) {
    void *ptrs[1024];
    uint32_t plen[1024];
    for (unsigned int i = 0; i < vlen; ++i) {
        const struct msghdr *h = &vec[i].msg_hdr;
        ptrs[i] = h->msg_iovlen >= 1 && h->msg_iov ? h->msg_iov[0].iov_base : NULL;
        plen[i] = ptrs[i] ? lens[i] : 0;   /* < 20 bytes: SKIPPED, nothing read */
    }
    pthread_mutex_lock(&g_mu);
    t_guard = 1;
    if (ensure_ctx()) {
        t_guard = 0;
        g_st.errors++;
        pthread_mutex_unlock(&g_mu);
        errno = ENXIO;
        return -1;
    }
    int mode = (fill ? TCPCSUM_IPV4_FILL : TCPCSUM_IPV4_VERIFY) | (g_iphdr ? TCPCSUM_IPV4_IPHDR : 0);
    int rc = tcpcsum_ipv4_batch_ptrs_host(g_ctx, ptrs, plen, vlen, mode, g_out, g_status);
    t_guard = 0;
    if (rc) {
        g_st.errors++;
        pthread_mutex_unlock(&g_mu);
        fprintf(stderr, "tcpcsum_preload: batch failed: %s\n", tcpcsum_strerror(rc));
        errno = ENXIO;
        return -1;
    }
    for (unsigned int i = 0; i < vlen; ++i) {
        const int ok = account((int) i, fill, is_tx, (const uint8_t *) ptrs[i], plen[i], vec[i].msg_hdr.msg_iovlen > 1,
                               partial_ok);
        if (keep) keep[i] = (unsigned char) ok;
    }
    pthread_mutex_unlock(&g_mu);
    return 0;
}

/* The readable bytes of message m's first iovec: iov_len (tx), or what was received
 * into it (rx: msg_len — with MSG_TRUNC a raw or UDP socket reports the datagram's
 * real length there, which may exceed the buffer). */
static unsigned int first_iov_bytes(const struct mmsghdr *m, int is_tx) {
    const struct msghdr *h = &m->msg_hdr;
    if (h->msg_iovlen < 1 || !h->msg_iov) return 0;
    const size_t cap = h->msg_iov[0].iov_len;
    const size_t got = is_tx ? cap : m->msg_len;
    const size_t n = got < cap ? got : cap;
    return n > 0xFFFFFFFFu ? 0xFFFFFFFFu : (unsigned int) n;
}

int SEAM(sendmmsg)(int fd, struct mmsghdr *vec, unsigned int vlen, int flags) {
    pthread_once(&g_once, init_once);
    if (g_tx != MODE_OFF && vlen && vec && wants_fd(fd)) {
        unsigned int lens[1024];
        unsigned int done = 0;
        while (done < vlen) {   /* GPU batches of <= 1024 messages */
            unsigned int cnt = vlen - done < 1024 ? vlen - done : 1024;
            for (unsigned int i = 0; i < cnt; ++i) lens[i] = first_iov_bytes(&vec[done + i], 1);
            if (gpu_batch(vec + done, cnt, lens, g_tx == MODE_FILL, 1, NULL, 0)) return -1;
            pthread_mutex_lock(&g_mu);
            g_st.tx_batches++;
            g_st.tx_packets += cnt;
            pthread_mutex_unlock(&g_mu);
            done += cnt;
        }
    }
    return real_sendmmsg(fd, vec, vlen, flags);
}

int SEAM(recvmmsg)(int fd, struct mmsghdr *vec, unsigned int vlen, int flags, struct timespec *timeout) {
    pthread_once(&g_once, init_once);
    int r = real_recvmmsg(fd, vec, vlen, flags, timeout);
    if (r > 0 && g_rx != MODE_OFF && wants_fd(fd)) {
        unsigned int lens[1024];
        unsigned char keep[1024];
        unsigned int done = 0, kept = 0;
        const int by_entry = g_rx == MODE_DROP && rx_by_entry(vec, (unsigned int) r);
        /* the loopback CHECKSUM_PARTIAL exception: AF_INET sockets, no route_localnet */
        const int partial_ok = !g_localnet && sock_opt(fd, SO_DOMAIN) == AF_INET;
        while (done < (unsigned int) r) {
            unsigned int cnt = (unsigned int) r - done < 1024 ? (unsigned int) r - done : 1024;
            for (unsigned int i = 0; i < cnt; ++i) lens[i] = first_iov_bytes(&vec[done + i], 0);
            if (gpu_batch(vec + done, cnt, lens, 0, 0, keep, partial_ok)) return -1;
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
#endif /* PART_SEAMS */
