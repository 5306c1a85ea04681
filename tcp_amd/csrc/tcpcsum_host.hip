// tcpcsum_host.hip — the host-memory half of the C ABI (tcpcsum_ctx_*, *_host).
//
// The path as the reference runs it starts and ends in host memory: finished
// packets sit in the loop's out-buffers (loop.c:107-116, 1024 separately
// malloc'd 32 KiB buffers, loop.c:180-183) until releaseSend flushes them
// (loop.c:27-94). A context turns such batches into kernel launches.
//
// Which host memory a kernel touches, and how:
//   * memory its owner page-locked — tcpcsum_host_alloc / hipHostMalloc, or a
//     hipHostRegister of the application's own — is read in place by the
//     kernel over PCIe (zero-copy), and FILL stores the checks there; a bulk
//     uniform batch (32 MiB or more) is DMA'd to HBM from those pages instead;
//   * pageable memory is never page-locked and never handed to a HIP copy.
//     CPU threads copy its bytes into the context's own pinned staging —
//     uniform batches chunk by chunk (then DMA'd to HBM), wire batches packet
//     by packet (only the packets, not the slack between them, read by the
//     kernel over PCIe); FILL results go back as 2-byte CPU stores at TCP+16
//     (and IP+10), exactly where context.c:208 puts them.
//
// Every copy and launch of a context goes to its one stream: host-to-HBM copies
// alternating over two streams fell to 43.5 GiB/s in some process states, one
// stream holds 51-53 (tools/dma_state_probe.hip).
//
// The library page-locks only memory it allocates itself (round 4). Rounds 2
// and 3 page-locked pageable heap memory — per call (round 2), then on request
// (tcpcsum_ctx_register_host, TCPCSUM_CTX_AUTO_REGISTER, round 3) — and a
// later pageable HIP copy faulted (hipErrorIllegalAddress) each time, over
// addresses those registrations had covered. GPU mappings of host memory are
// per page; HIP pins the pages of pageable copy buffers in place behind the
// scenes and keeps those pins cached (hipPointerGetAttributes does not show
// them, and a hipHostRegister over them succeeds: tools/pin_cache_probe.cpp);
// a malloc'd buffer shares its first and last page with heap neighbours. So a
// library hipHostRegister / hipHostUnregister of heap pages can change the
// mapping under a pin HIP still uses, and the other way round — and neither
// side can see the other. Nothing here changes any foreign page's state
// (host_registry.h is a lookup only), so it cannot happen through the library;
// a caller that wants zero copy allocates its packet buffers with
// tcpcsum_host_alloc (the pool at loop.c:180-183, INTEGRATION.md level 2).
//
// All checksum arithmetic runs in the gfx950 kernels of tcpcsum_kernels.hip;
// this file reads header fields (IHL, tot_len) only to size the copies.

#include <emmintrin.h>
#include <hip/hip_runtime.h>
#include <sched.h>
#include <linux/mempolicy.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <time.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <chrono>
#include <thread>
#include <vector>

#include "copy_pool.h"
#include "host_registry.h"
#include "tcpcsum.h"
#include "tcpcsum_internal.h"

namespace tcpcsum {

// PinnedLookup backend over HIP: where memory its owner page-locked is mapped
// for the device (on MI355X hosts at its host address: tools/hostreg_probe.py).
// Queries only — nothing here locks or unlocks a page.
struct HipHostBackend {
    bool pinned_extent(uintptr_t p, uintptr_t* lo, uintptr_t* hi, intptr_t* delta) {
        hipPointerAttribute_t a;
        bool ok = hipPointerGetAttributes(&a, (const void*)p) == hipSuccess && a.type == hipMemoryTypeHost &&
                  a.devicePointer;
        uintptr_t rs = 0;
        size_t rsz = 0;
        ok = ok && hipPointerGetAttribute(&rs, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) == hipSuccess &&
             hipPointerGetAttribute(&rsz, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) == hipSuccess;
        (void)hipGetLastError();   // pageable memory: not an error for us
        if (!ok) return false;
        *lo = rs;
        *hi = rs + rsz;
        *delta = (intptr_t)a.devicePointer - (intptr_t)p;
        return true;
    }
};

inline int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

// The switch of a measured-and-rejected or A/B-only variant of the host pipeline:
// read from the environment in measurement builds only (-DTCPCSUM_MEASUREMENT_BUILD=1);
// a product library takes the measured default, and the variable's name is not even
// in its binary. tcpcsum_build_info() lists the runtime knobs a build reads.
#if TCPCSUM_MEASUREMENT_BUILD
#define TCPCSUM_MEAS_KNOB(name, dflt) tcpcsum::env_int(name, dflt)
#else
#define TCPCSUM_MEAS_KNOB(name, dflt) (dflt)
#endif

// NUMA node of the (touched) host page at p, or -1.
inline int page_node(const void* p) {
    int node = -1;
    if (!p || syscall(SYS_get_mempolicy, &node, nullptr, 0, p, MPOL_F_NODE | MPOL_F_ADDR) != 0) return -1;
    return node;
}

// hipHostMalloc on NUMA node `node` (-1: HIP's choice): the calling thread's memory
// policy is set to prefer that node for the allocation (hipHostMallocNumaUser: the
// pages follow the thread's policy) and restored after. On a box whose GPU sits on
// node 1, the default placement put the staging elsewhere: the pageable end-to-end
// path ran at 32 GiB/s there against 50 on node-0 boxes (profiles/r04_bench_first.json).
inline hipError_t host_malloc_on(void** p, size_t bytes, int node) {
    if (node < 0 || node >= 1024) return hipHostMalloc(p, bytes, hipHostMallocDefault);
    int mode = 0;
    unsigned long old_mask[16] = {0};
    const bool saved = syscall(SYS_get_mempolicy, &mode, old_mask, 1024ul, nullptr, 0ul) == 0;
    unsigned long mask[16] = {0};
    mask[node / 64] = 1ul << (node % 64);
    const bool set = saved && syscall(SYS_set_mempolicy, MPOL_PREFERRED, mask, 1024ul) == 0;
    hipError_t e = hipHostMalloc(p, bytes, set ? hipHostMallocNumaUser : hipHostMallocDefault);
    if (set) syscall(SYS_set_mempolicy, mode, (mode == MPOL_DEFAULT) ? nullptr : old_mask, 1024ul);
    return e;
}

// Page-locked host memory owned by a context, with its device view.
struct Pinned {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t bytes = 0;
    int node = -1;   // NUMA node to allocate on (the GPU's), -1: HIP's choice
    Pinned() = default;
    Pinned(const Pinned&) = delete;
    Pinned& operator=(const Pinned&) = delete;
    ~Pinned() { release(); }
    // grow to at least `need` bytes; the caller knows no kernel is using it. Doubling
    // (small per-batch arrays grow a few times), but never past `need` rounded up to
    // 2 MiB: a 128 MiB staging slot is 128 MiB, not the next power of two
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        size_t nb = bytes ? bytes : 4096;
        while (nb < need) nb *= 2;
        const size_t k2m = (size_t)2 << 20;
        nb = std::min(nb, (need + k2m - 1) / k2m * k2m);
        release();
        void* p = nullptr;
        hipError_t e = host_malloc_on(&p, nb, node);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return e;
        }
        void* dp = nullptr;
        e = hipHostGetDevicePointer(&dp, p, 0);
        if (e != hipSuccess || !dp) {
            (void)hipGetLastError();
            (void)hipHostFree(p);
            return e != hipSuccess ? e : hipErrorInvalidValue;
        }
        h = (uint8_t*)p;
        d = (uint8_t*)dp;
        bytes = nb;
        return hipSuccess;
    }
    void release() {
        if (h) (void)hipHostFree(h);
        h = d = nullptr;
        bytes = 0;
    }
};

}  // namespace tcpcsum

using tcpcsum::check_launch;
using tcpcsum::get_tuning;
using tcpcsum::hip_fail;
using tcpcsum::require_device;

// Staging chunk per pipeline slot for pageable uniform batches, and the DMA chunk
// for page-locked ones (scratch_bytes, when given, sets both).
constexpr size_t kDefaultChunk = 128u << 20;
constexpr size_t kDefaultDmaChunk = 256u << 20;
// page-locked uniform batches under two of these are read in place over PCIe
constexpr size_t kDefaultInPlaceChunk = 16u << 20;

struct tcpcsum_ctx {
    int device = 0;
    size_t chunk = 0;       // pageable uniform batches: bytes per staged chunk
    size_t dma_chunk = 0;   // page-locked uniform batches: bytes per DMA to HBM
    size_t in_place_chunk = 0;   // ... read in place when under two of these
    uint32_t flags = 0;
    // every copy and launch of a context goes to this one stream, in order: two
    // streams alternating 16 MiB host-to-HBM copies ran at 43.5 GiB/s instead of
    // 53.3 in some process states (after a 16 GiB device allocation, and on some
    // boxes from the start), one stream never below 51.2 (tools/dma_state_probe.hip)
    hipStream_t st = nullptr;
    // pageable uniform batches: nslots pinned staging chunks in flight
    // (2; measurement builds: TCPCSUM_HOST_SLOTS, 2..4); slot_ev[s] is recorded after the last device
    // work that reads staging slot s, before the copy threads refill it
    int nslots = 2;
    hipEvent_t slot_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    bool slot_busy[4] = {false, false, false, false};
    tcpcsum::Pinned slot[4];   // one staged chunk each
    // HBM for the chunk being checksummed (the stream orders each copy behind
    // the previous chunk's kernel, so one buffer serves every chunk)
    uint8_t* d_buf = nullptr;
    size_t d_buf_bytes = 0;
    tcpcsum::Pinned gath;      // wire batches: packets copied out of pageable memory
    tcpcsum::Pinned ss, res;   // per-segment start values / results, when the caller's are pageable
    // per-packet arrays the wire kernels read (addresses, bounds) and write
    // (results, status), kept in pinned memory so a pageable caller array costs
    // a CPU memcpy rather than a HIP copy
    tcpcsum::Pinned p_off, p_len, p_out, p_stat;
    // gathered packets of the current batch: index, source, staging offset, bytes
    std::vector<uint64_t> g_idx, g_off;
    std::vector<uint8_t*> g_src;
    std::vector<uint32_t> g_len;
    tcpcsum::Tuning tune;
    tcpcsum::HipHostBackend backend;
    tcpcsum::PinnedLookup<tcpcsum::HipHostBackend> pinned{backend};
    std::unique_ptr<tcpcsum::CopyPool> pool;
    int gpu_node = -1;   // the GPU's NUMA node, where the staging is allocated (-1: unknown / off)
    // threads a staged wire batch copies on, the caller included (1): a releaseSend batch
    // is ~1.5 MB, where extra threads cost more CPU than they save time
    int wire_threads = 1;
    // threads a bulk copy (uniform staging chunks, per-segment arrays) runs on, the caller
    // included (4, at most the pool's): the DMA to HBM bounds the pageable pipeline, and 4
    // threads copy 1.5 GB in ~14.5 ms beside its ~28 ms at the rate 8 reach, with 0.060
    // instead of 0.087 core-s (profiles/r04_host_bulk_threads_ab.jsonl)
    int bulk_threads = 4;
    int stage_threads = 1;   // the current staged batch's: wire_threads, or all for a large batch
    // TCPCSUM_CTX_BLOCKING_WAIT: wait for the device by polling this event between
    // short sleeps instead of HIP's spin in hipStreamSynchronize
    hipEvent_t done_ev = nullptr;
    // the sleeping wait's prediction: observed / expected device time (x1024) of this
    // context's batches, [0] releaseSend-sized (expected < 1 ms), [1] bulk; start at
    // 3/4, round 4's fixed first nap
    uint32_t wait_ratio[2] = {768u, 768u};
    // The product's choices below; measurement builds can flip each (the TCPCSUM_HOST_*
    // name in brackets) for A/B runs:
    uint64_t poll_ns = 5000;     // first sleep between polls after the expected time (POLL_US)
    bool nt_copy = true;   // streaming stores for the uniform chunks (NT=0: plain memcpy)
    bool stage_one_pass = true;   // wire staging laid out by bounds, one pass (STAGE_PASSES=2: by lengths)
    bool uniform_dma = true;   // staged uniform chunks go to HBM by DMA (DMA=0: kernel reads them over PCIe)
    bool pinned_dma = true;    // large page-locked uniform batches go to HBM by DMA (PINNED_DMA=0: in place)
    bool slot_sleep = true;    // BLOCKING_WAIT also sleeps in staging-slot waits (SLOT_SLEEP=0: spin)
    // wire staging with streaming stores, each packet from a 64-B line of its own, one
    // fence per copy job (WIRE_NT=0: plain memcpy from 16-B starts). The seam's 1024 x
    // 1500-B batch: 102-112 instead of 119-171 us, 65-75 instead of 72-102 core-us
    // (profiles/r04_wire_nt_ab.jsonl)
    bool wire_nt = true;
    tcpcsum_ctx_stats_t stats{};
    std::mutex mu;
};

namespace {

// A host call that returns early on an error may have queued copies and kernels
// that still read or write the caller's memory: drain the stream before the
// caller gets control back (and may free that memory). Disarmed once the call
// has waited for its work.
struct DrainOnError {
    hipStream_t st;
    bool done = false;
    explicit DrainOnError(hipStream_t s) : st(s) {}
    ~DrainOnError() {
        if (!done && st) (void)hipStreamSynchronize(st);
    }
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) hipSetDevice(prev);
    }
};

// Device-visible address of page-locked (hipHostMalloc / hipHostRegister'ed)
// host memory [p, p + bytes), or nullptr when any of it is pageable. Kernels
// read and write such memory directly over PCIe. The whole range must lie in
// ONE page-locked allocation or registration: a range locked only in part
// (its first page locked by a neighbouring registration, say) is staged.
void* pinned_dev_ptr(const void* p, size_t bytes = 1) {
    if (!p) return nullptr;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory: not an error for us
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
    uintptr_t rs = 0;
    size_t rsz = 0;
    if (hipPointerGetAttribute(&rs, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) != hipSuccess ||
        hipPointerGetAttribute(&rsz, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    const uintptr_t b = (uintptr_t)p;
    if (rs > b || b + (bytes ? bytes : 1) > rs + rsz) return nullptr;
    return a.devicePointer;
}

// memcpy on the context's copy threads (pieces of 256 KiB); nt: streaming stores;
// threads: how many take part, the caller included (-1: bulk_threads, 0: all).
void par_copy(tcpcsum_ctx* c, void* dst, const void* src, size_t n, bool nt = false, int threads = -1) {
    if (threads < 0) threads = c->bulk_threads;
    constexpr size_t kGrain = 256u << 10;
    uint8_t* d = (uint8_t*)dst;
    const uint8_t* s = (const uint8_t*)src;
    const uint64_t t0 = tcpcsum::now_ns();
    if (nt)
        c->pool->run(n, kGrain, [&](size_t lo, size_t hi) { tcpcsum::copy_nt(d + lo, s + lo, hi - lo); },
                     threads);
    else
        c->pool->run(n, kGrain, [&](size_t lo, size_t hi) { memcpy(d + lo, s + lo, hi - lo); }, threads);
    c->stats.ns_copy += tcpcsum::now_ns() - t0;
}

// Sleep until ev has completed: a first nap of nap_ns, then a poll every
// c->poll_ns — at that fixed step until the clock passes fixed_until_ns, then
// doubling up to max_step_ns (1 us timer slack on this thread while it sleeps,
// restored after).
hipError_t sleep_on_event(tcpcsum_ctx* c, hipEvent_t ev, uint64_t nap_ns, uint64_t max_step_ns,
                          uint64_t fixed_until_ns = 0, int* sleeps = nullptr) {
    const int slack = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
    bool slack_set = false;
    uint64_t step = std::min<uint64_t>(c->poll_ns, max_step_ns);
    hipError_t e;
    int n = 0;   // sleeps taken before the event was seen complete
    for (;; ++n) {
        e = hipEventQuery(ev);
        if (e != hipErrorNotReady) break;
        (void)hipGetLastError();   // not ready is not an error for us
        if (!slack_set && slack > 0) {
            prctl(PR_SET_TIMERSLACK, 1000, 0, 0, 0);
            slack_set = true;
        }
        uint64_t ns = nap_ns;
        if (!ns) {
            ns = step;
            if (tcpcsum::now_ns() >= fixed_until_ns) step = std::min<uint64_t>(step * 2, max_step_ns);
        }
        nap_ns = 0;
        timespec ts{(time_t)(ns / 1000000000u), (long)(ns % 1000000000u)};
        nanosleep(&ts, nullptr);
    }
    if (slack_set) prctl(PR_SET_TIMERSLACK, (unsigned long)slack, 0, 0, 0);
    if (sleeps) *sleeps = n;
    return e;
}

// Wait for everything queued on st, timed into stats.ns_wait: hipStreamSynchronize
// (HIP spins: the waiting thread burns a core for the kernel's whole length), or
// with TCPCSUM_CTX_BLOCKING_WAIT a poll of the stream's completion event between
// sleeps. A hipEventBlockingSync event did not help: the runtime waits on its
// signal actively for about a batch kernel's length, and the thread used as much
// CPU as with hipStreamSynchronize (48.7 vs 48.5 us per 1024-packet in-place
// batch, profiles/r04_e2e_first.jsonl).
//
// The sleeping wait predicts when the work ends: expect_ns (the caller's estimate
// from its bytes) times a ratio this context learns per size class. It naps until
// the prediction, then polls every poll_ns for as long again (at most 200 us), then
// backs off. When the work was already done at the end of the nap, the nap may have been
// too long: the ratio shrinks by 1/32. When it took polls, the ratio moves an
// eighth of the way to what the wait took (at most one poll interval late). A wake
// that comes late (a busy host) therefore never lengthens the next nap. Round 4
// napped 3/4 of the estimate and then polled at 5, 10, 20, 40 us, so a releaseSend
// batch done at 64 us was seen at 104 us (profiles/r05_host_fill_ab.jsonl, r05_wait_ab.jsonl).
hipError_t wait_stream(tcpcsum_ctx* c, hipStream_t st, uint64_t expect_ns) {
    const uint64_t t0 = tcpcsum::now_ns();
    hipError_t e;
    if (c->flags & TCPCSUM_CTX_BLOCKING_WAIT) {
        e = hipEventRecord(c->done_ev, st);
        if (e == hipSuccess) {
            uint32_t& ratio = c->wait_ratio[expect_ns < 1000000u ? 0 : 1];   // predicted / expected, x1024
            const uint64_t pred = std::min<uint64_t>(expect_ns * ratio / 1024u, 200000000u);
            int sleeps = 0;
            // fixed-step polls for at most min(pred, 200 us) past the prediction, then back
            // off: a bulk batch (pred up to 200 ms) that overruns is not polled every 5 us
            e = sleep_on_event(c, c->done_ev, pred, 100000u, t0 + pred + std::min<uint64_t>(pred, 200000u), &sleeps);
            const uint64_t took = tcpcsum::now_ns() - t0;
            if (e == hipSuccess && expect_ns) {
                if (sleeps <= 1)   // done by the end of the nap: try a shorter one
                    ratio -= ratio / 32u;
                else
                    ratio = (uint32_t)((ratio * 7u + std::min<uint64_t>(took * 1024u / expect_ns, 8192u)) / 8u);
                ratio = std::max<uint32_t>(ratio, 128u);
            }
        }
    } else {
        e = hipStreamSynchronize(st);
    }
    c->stats.ns_wait += tcpcsum::now_ns() - t0;
    return e;
}

// Wait for a staging slot's event (the DMA that last read the slot), timed into
// stats.ns_wait: spinning in hipEventSynchronize, or with
// TCPCSUM_CTX_BLOCKING_WAIT polling between sleeps of at most 20 us (no first
// nap: how much of that DMA is left when the copy threads get here varies).
hipError_t wait_slot(tcpcsum_ctx* c, hipEvent_t ev) {
    const uint64_t t0 = tcpcsum::now_ns();
    const hipError_t e = ((c->flags & TCPCSUM_CTX_BLOCKING_WAIT) && c->slot_sleep) ? sleep_on_event(c, ev, 0, 20000u)
                                                                                   : hipEventSynchronize(ev);
    c->stats.ns_wait += tcpcsum::now_ns() - t0;
    return e;
}

// What a host batch's device work should take: its bytes over PCIe (~50 GB/s,
// 50 bytes per ns) plus a launch's latency — the sleeping wait's first nap.
inline uint64_t expect_ns(uint64_t bytes) { return bytes / 50u + 8000u; }

// CPU time of the calling thread inside one host call, into stats.ns_cpu_caller.
struct CallerCpu {
    tcpcsum_ctx* c;
    uint64_t t0;
    static uint64_t now() {
        timespec ts;
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
        return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
    }
    explicit CallerCpu(tcpcsum_ctx* ctx) : c(ctx), t0(now()) {}
    ~CallerCpu() { c->stats.ns_cpu_caller += now() - t0; }
};

int ensure_pkt_arrays(tcpcsum_ctx* c, uint64_t n) {
    hipError_t e = c->p_off.ensure(n * sizeof(uint64_t));
    if (e == hipSuccess) e = c->p_len.ensure(n * sizeof(uint32_t));
    if (e == hipSuccess) e = c->p_out.ensure(n * sizeof(uint16_t));
    if (e == hipSuccess) e = c->p_stat.ensure(n);
    if (e != hipSuccess) {
        tcpcsum::note_hip_error((int)e);
        return TCPCSUM_ENOMEM;
    }
    return TCPCSUM_OK;
}

// Bytes of a wire packet worth copying: its tot_len (at least the 20-byte IP
// header), never more than `bound` readable bytes. A packet whose tot_len
// exceeds the bound keeps tot_len > copied bytes and is SKIPPED by the
// kernel exactly as when it is read in place.
inline uint32_t copy_len(const uint8_t* ip, uint64_t bound) {
    const uint32_t tot = ((uint32_t)ip[2] << 8) | ip[3];
    const uint64_t want = tot < 20u ? 20u : tot;
    return (uint32_t)std::min<uint64_t>(want, bound);
}

// Stage the packets listed in g_* (g_len holds each one's readable bound)
// into c->gath, all on the copy threads; the calling thread never reads a
// packet. Each copy thread reads a packet's tot_len (copy_len: the bytes worth
// copying, within its bound) and copies it. Where the bounds add up to at most
// kStageByBound, a packet's place in the staging is laid out by its bound and
// that is one pass; past it (huge bounds: 64 KiB caps over big batches) the
// lengths are read first and the copies packed by them, two passes. Sets
// k_off / k_len of every staged packet.
constexpr size_t kStageByBound = 64u << 20;
constexpr size_t kSmallStage = 8u << 20;
int stage_packets(tcpcsum_ctx* c, uint64_t* k_off, uint32_t* k_len, size_t* staged_bytes) {
    const size_t m = c->g_idx.size();
    *staged_bytes = 0;
    if (!m) return TCPCSUM_OK;
    const uint64_t t0 = tcpcsum::now_ns();
    const size_t am = c->wire_nt ? 63u : 15u;   // each packet's staging start: 64-B line or 16 B
    size_t span = 0;
    for (size_t k = 0; k < m; ++k) {
        c->g_off[k] = span;
        span += ((size_t)c->g_len[k] + am) & ~am;
    }
    const bool by_bound = span <= kStageByBound && c->stage_one_pass;
    // small (releaseSend-sized) batches copy on wire_threads; large ones on every copy thread
    c->stage_threads = span <= kSmallStage ? c->wire_threads : 0;
    if (!by_bound) {
        c->pool->run(m, 64, [&](size_t lo, size_t hi) {
            for (size_t k = lo; k < hi; ++k) c->g_len[k] = copy_len(c->g_src[k], c->g_len[k]);
        }, c->stage_threads);
        span = 0;
        for (size_t k = 0; k < m; ++k) {
            c->g_off[k] = span;
            span += ((size_t)c->g_len[k] + am) & ~am;
        }
    }
    hipError_t e = c->gath.ensure(span ? span : 16);
    if (e != hipSuccess) {
        tcpcsum::note_hip_error((int)e);
        return TCPCSUM_ENOMEM;
    }
    uint8_t* gh = c->gath.h;
    uint8_t* gd = c->gath.d;
    std::atomic<size_t> copied{0};
    c->pool->run(m, 16, [&](size_t lo, size_t hi) {
        size_t b = 0;
        for (size_t k = lo; k < hi; ++k) {
            if (by_bound) c->g_len[k] = copy_len(c->g_src[k], c->g_len[k]);
            // streaming stores from 64-B starts, fenced once per job: with an sfence per
            // packet and 16-B starts (copy_nt) they had made a 1024 x 1500-B staged batch
            // 4.6 x slower on one thread (618 vs 135 us, profiles/r04_e2e_first.jsonl)
            if (c->wire_nt)
                tcpcsum::copy_stream(gh + c->g_off[k], c->g_src[k], c->g_len[k]);
            else
                memcpy(gh + c->g_off[k], c->g_src[k], c->g_len[k]);
            k_off[c->g_idx[k]] = (uint64_t)(uintptr_t)(gd + c->g_off[k]);
            k_len[c->g_idx[k]] = c->g_len[k];
            b += c->g_len[k];
        }
        if (c->wire_nt) _mm_sfence();   // this thread's streaming stores, before the launch
        copied.fetch_add(b, std::memory_order_relaxed);
    }, c->stage_threads);
    c->stats.ns_copy += tcpcsum::now_ns() - t0;
    c->stats.pkts_staged += m;
    c->stats.bytes_staged += copied.load();
    *staged_bytes = copied.load();
    return TCPCSUM_OK;
}

// Stage the packets in g_* and launch the wire kernel over all n packets on
// st (k_off / k_len of the packets read in place already set; in_cap /
// in_foot their largest length and sum). One launch after the copies: queueing
// the kernel first, in blocks each released by a pinned flag the copy threads
// set (hipStreamWaitValue64), was measured and lost — 1 / 2 / 4 / 8 blocks
// against copy-then-launch on 1024 x 1500-B batches: no gain / no gain /
// +15-30 us / +60-90 us, the host cost of each queued launch landing before
// the copies (profiles/r03_hostpath_sweep_wire_split.jsonl).
int stage_and_launch(tcpcsum_ctx* c, uint64_t n, uint32_t in_cap, uint64_t in_foot, int mode, uint16_t* kout,
                     uint8_t* kst, hipStream_t st, const tcpcsum::Tuning& tu) {
    size_t staged = 0;
    int rc = stage_packets(c, (uint64_t*)c->p_off.h, (uint32_t*)c->p_len.h, &staged);
    if (rc) return rc;
    uint32_t cap = in_cap;
    for (size_t k = 0; k < c->g_idx.size(); ++k) cap = std::max(cap, c->g_len[k]);
    tcpcsum::launch_ipv4(nullptr, (const uint64_t*)c->p_off.d, (const uint32_t*)c->p_len.d, n, cap, ~0ull,
                         in_foot + staged, mode, kout, kst, nullptr, st, tu);
    return check_launch();
}

// FILL on staged packets: the kernel stored each check in the staging copy;
// put it (and the IPv4 header checksum, with IPHDR) into the caller's packet,
// on the copy threads.
void write_back_checks(tcpcsum_ctx* c, const uint8_t* status, bool iphdr) {
    const size_t m = c->g_idx.size();
    const uint64_t t0 = tcpcsum::now_ns();
    c->pool->run(m, 64, [&](size_t lo, size_t hi) {
        for (size_t k = lo; k < hi; ++k) {
            if (status[c->g_idx[k]] != TCPCSUM_PKT_OK) continue;
            const uint8_t* sp = c->gath.h + c->g_off[k];
            uint8_t* dp = c->g_src[k];
            const unsigned tcp = (sp[0] & 15u) * 4u;
            memcpy(dp + tcp + 16, sp + tcp + 16, 2);   // context.c:208: native u16 at TCP+16
            if (iphdr) memcpy(dp + 10, sp + 10, 2);
        }
    }, c->stage_threads);
    c->stats.ns_copy += tcpcsum::now_ns() - t0;
}

// Launch shape and FILL store of a host wire batch (tcpcsum_ipv4_batch_host /
// _ptrs_host) unless the context's tuning says otherwise:
//   * 16-lane groups, 512 B per round, for latency-bound batches read over PCIe:
//     more waves with reads in flight beat the HBM-tuned MTU shape — 1024 x
//     1500-B FILL batch 49 vs 59 us (profiles/r02_e2e_ptrs_sweep.jsonl);
//   * the plain 2-byte check store, exactly the bytes context.c:208 writes. The
//     whole-line write-back that pays in HBM (whole lines instead of partial ones)
//     buys nothing over PCIe: 1024 x 1500-B in-place FILL 67.4-70.1 vs 68.2-68.4 us
//     (profiles/r05_host_fill_ab.jsonl, r05_wait_ab.jsonl).
tcpcsum::Tuning host_wire_tuning(const tcpcsum_ctx* c, uint64_t n) {
    tcpcsum::Tuning tu = c->tune;
    if (tu.shape < 0 && n < 65536u) tu.shape = 3;
    if (!(tu.flags & (TCPCSUM_TUNE_FILL_DWORD | TCPCSUM_TUNE_FILL_U16 | TCPCSUM_TUNE_FILL_HALF)))
        tu.flags |= TCPCSUM_TUNE_FILL_U16;
    return tu;
}

}  // namespace

extern "C" {

int tcpcsum_ctx_create(int device, size_t scratch_bytes, tcpcsum_ctx_t** out) {
    if (!out) return TCPCSUM_EINVAL;
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || device < 0 || device >= count) {
        tcpcsum::note_hip_error((int)e);
        return TCPCSUM_ENODEV;
    }
    DeviceGuard g(device);
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    tcpcsum_ctx* c = new (std::nothrow) tcpcsum_ctx();
    if (!c) return TCPCSUM_ENOMEM;
    c->device = device;
    c->chunk = scratch_bytes ? scratch_bytes : kDefaultChunk;
    // copy threads spin TCPCSUM_HOST_SPIN_US (default 50) after a job before they sleep
    const uint64_t spin_ns = (uint64_t)std::max(0, tcpcsum::env_int("TCPCSUM_HOST_SPIN_US", 50)) * 1000u;
    // copy threads on the GPU's NUMA node, where hipHostMalloc put the staging
    // (TCPCSUM_HOST_NUMA=0: wherever the scheduler puts them)
    cpu_set_t node_cpus;
    char bus[64] = {0};
    int gpu_node = -1;
    const bool numa = tcpcsum::env_int("TCPCSUM_HOST_NUMA", 1) != 0 &&
                      hipDeviceGetPCIBusId(bus, sizeof bus, device) == hipSuccess &&
                      tcpcsum::numa_node_cpus(bus, &node_cpus, &gpu_node);
    (void)hipGetLastError();
    // pinned staging on the GPU's node too (the copy threads write it, the DMA reads it)
    c->gpu_node = numa ? gpu_node : -1;
    for (tcpcsum::Pinned* pp : {&c->slot[0], &c->slot[1], &c->slot[2], &c->slot[3], &c->gath, &c->ss, &c->res, &c->p_off, &c->p_len, &c->p_out,
                                &c->p_stat})
        pp->node = c->gpu_node;
    // never more workers than the node has CPUs this process may use (the caller is one of
    // the copiers too, wherever it runs)
    int copiers = tcpcsum::default_copy_threads();
    if (numa) copiers = std::min(copiers, CPU_COUNT(&node_cpus) + 1);
    c->pool.reset(new (std::nothrow) tcpcsum::CopyPool(copiers - 1, spin_ns, numa ? &node_cpus : nullptr));
    if (!c->pool) {
        delete c;
        return TCPCSUM_ENOMEM;
    }
    c->wire_threads = std::max(1, std::min(c->pool->threads(), TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_WIRE_THREADS", 1)));
    c->stats.copy_threads = (uint64_t)c->wire_threads;
    c->bulk_threads = std::max(0, std::min(c->pool->threads(), TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_BULK_THREADS", 4)));
    c->stats.bulk_threads = (uint64_t)(c->bulk_threads ? c->bulk_threads : c->pool->threads());
    c->nt_copy = TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_NT", 1) != 0;
    c->poll_ns = (uint64_t)std::max(1, TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_POLL_US", 5)) * 1000u;
    c->stage_one_pass = TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_STAGE_PASSES", 1) == 1;
    c->uniform_dma = TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_DMA", 1) != 0;
    c->pinned_dma = TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_PINNED_DMA", 1) != 0;
    c->slot_sleep = TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_SLOT_SLEEP", 1) != 0;
    c->wire_nt = TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_WIRE_NT", 1) != 0;
    c->nslots = std::max(2, std::min(4, TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_SLOTS", 2)));
    c->dma_chunk = scratch_bytes ? scratch_bytes : kDefaultDmaChunk;
    c->in_place_chunk = scratch_bytes ? scratch_bytes : kDefaultInPlaceChunk;
    if (!scratch_bytes) {
        c->chunk = (size_t)std::max(1, TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_CHUNK_MB", (int)(kDefaultChunk >> 20))) << 20;
        c->dma_chunk =
            (size_t)std::max(1, TCPCSUM_MEAS_KNOB("TCPCSUM_HOST_DMA_CHUNK_MB", (int)(kDefaultDmaChunk >> 20))) << 20;
    }
    e = hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking);
    if (e != hipSuccess) {
        tcpcsum_ctx_destroy(c);
        return hip_fail(e);
    }
    for (int i = 0; i < 4; ++i) {
        e = hipEventCreateWithFlags(&c->slot_ev[i], hipEventDisableTiming);
        if (e != hipSuccess) {
            tcpcsum_ctx_destroy(c);
            return hip_fail(e);
        }
    }
    e = hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        tcpcsum_ctx_destroy(c);
        return hip_fail(e);
    }
    *out = c;
    return TCPCSUM_OK;
}

void tcpcsum_ctx_destroy(tcpcsum_ctx_t* c) {
    if (!c) return;
    DeviceGuard g(c->device);
    if (c->st) hipStreamSynchronize(c->st);
    c->pool.reset();   // the copy threads are joined here, before any HIP object goes
    if (c->done_ev) hipEventDestroy(c->done_ev);
    for (int i = 0; i < 4; ++i)
        if (c->slot_ev[i]) hipEventDestroy(c->slot_ev[i]);
    if (c->d_buf) hipFree(c->d_buf);
    if (c->st) hipStreamDestroy(c->st);
    delete c;   // pinned buffers go with it
}

int tcpcsum_ctx_set_tuning(tcpcsum_ctx_t* c, const tcpcsum_tuning_t* tune) {
    if (!c) return TCPCSUM_EINVAL;
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->tune = tu;
    return TCPCSUM_OK;
}

int tcpcsum_ctx_set_flags(tcpcsum_ctx_t* c, uint32_t flags) {
    if (!c || (flags & ~(uint32_t)TCPCSUM_CTX_BLOCKING_WAIT)) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->flags = flags;
    return TCPCSUM_OK;
}

int tcpcsum_ctx_get_stats(tcpcsum_ctx_t* c, tcpcsum_ctx_stats_t* out) {
    if (!c || !out) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->stats.ns_cpu_workers = c->pool->worker_cpu_ns();
    c->stats.gpu_numa_node = c->gpu_node < 0 ? UINT64_MAX : (uint64_t)c->gpu_node;
    const void* st = c->slot[0].h ? (const void*)c->slot[0].h : c->gath.h ? (const void*)c->gath.h : (const void*)c->p_off.h;
    const int sn = tcpcsum::page_node(st);
    c->stats.staging_numa_node = sn < 0 ? UINT64_MAX : (uint64_t)sn;
    *out = c->stats;
    return TCPCSUM_OK;
}

void* tcpcsum_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (!bytes) return nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        tcpcsum::note_hip_error((int)e);
        return nullptr;
    }
    return p;
}

void tcpcsum_host_free(void* p) {
    if (p) hipHostFree(p);
}

void* tcpcsum_host_alloc_on(int device, size_t bytes) {
    int cur = -1;
    if (!bytes || hipGetDevice(&cur) != hipSuccess) return nullptr;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        tcpcsum::note_hip_error((int)e);
        return nullptr;
    }
    void* p = tcpcsum_host_alloc(bytes);
    (void)hipSetDevice(cur);
    return p;
}

int tcpcsum_on_library_thread(void) { return tcpcsum::t_library_thread; }

// Page-locked input: batches under two 16 MiB pieces are read in place by one
// launch over PCIe; larger ones go to HBM by DMA straight from the caller's
// pages in dma_chunk pieces (256 MiB), each copy followed by its kernel on the
// context's one stream — in-stream order is the only synchronisation
// (TCPCSUM_HOST_PINNED_DMA=0: always in place). Pageable input: the copy threads
// fill pinned staging slot k % nslots with chunk k (16, 32, 64, then 128 MiB) while the stream
// copies chunk k-1 to HBM and checksums it; a slot is refilled once the DMA that
// read it has finished. Start values and results use the caller's arrays when
// those are page-locked, else pinned staging (copied in / out by the CPU).
int tcpcsum_batch_uniform_host(tcpcsum_ctx_t* c, const void* h_base, uint64_t stride, uint32_t len,
                               const uint32_t* h_sum_start, uint32_t sum_start, uint16_t* h_out, uint64_t n) {
    if (!c) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!h_base || !h_out || len > (uint32_t)INT_MAX) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    CallerCpu cpu(c);
    DeviceGuard g(c->device);
    DrainOnError drain(c->st);
    const tcpcsum::Tuning tu = c->tune;
    c->stats.batches++;
    hipError_t e;
    int rc;
    const uint32_t* kss = nullptr;
    if (h_sum_start) {
        kss = (const uint32_t*)pinned_dev_ptr(h_sum_start, n * sizeof(uint32_t));
        if (!kss) {
            e = c->ss.ensure(n * sizeof(uint32_t));
            if (e != hipSuccess) return hip_fail(e);
            par_copy(c, c->ss.h, h_sum_start, n * sizeof(uint32_t), c->nt_copy);
            kss = (const uint32_t*)c->ss.d;
        }
    }
    uint16_t* kout = (uint16_t*)pinned_dev_ptr(h_out, n * sizeof(uint16_t));
    const bool out_staged = kout == nullptr;
    if (out_staged) {
        e = c->res.ensure(n * sizeof(uint16_t));
        if (e != hipSuccess) return hip_fail(e);
        kout = (uint16_t*)c->res.d;
    }
    const size_t span = (size_t)((n - 1) * stride + len);
    // segments per piece of at most `bytes` (at least one segment)
    auto per_piece = [&](size_t bytes) -> uint64_t {
        uint64_t per = 1;
        if (stride == 0) per = n;
        else if (bytes > len) per = (bytes - len) / stride + 1;
        return per > n ? n : per;
    };
    auto piece_bytes = [&](uint64_t cnt) { return (size_t)((cnt - 1) * stride + len); };
    auto ensure_hbm = [&](size_t bytes) -> hipError_t {
        bytes += 16;   // the piece keeps its start's alignment mod 16
        if (bytes <= c->d_buf_bytes) return hipSuccess;
        if (c->d_buf) {
            (void)hipStreamSynchronize(c->st);
            (void)hipFree(c->d_buf);
        }
        c->d_buf = nullptr;
        c->d_buf_bytes = 0;
        const hipError_t he = hipMalloc(&c->d_buf, bytes);
        if (he == hipSuccess) c->d_buf_bytes = bytes;
        return he;
    };
    // a staging slot holds a piece plus its start's misalignment (16 B) within `chunk`
    const uint64_t per = per_piece(c->chunk > 32 ? c->chunk - 16 : c->chunk);
    const uint8_t* zb = (const uint8_t*)pinned_dev_ptr(h_base, span);
    if (zb && (!c->pinned_dma || per_piece(c->in_place_chunk) * 2 > n)) {
        tcpcsum::launch_uniform(zb, stride, len, kss, sum_start, kout, n, c->st, tu);
        rc = check_launch();
        if (rc) return rc;
        e = wait_stream(c, c->st, expect_ns(span));
        if (e != hipSuccess) return hip_fail(e);
        drain.done = true;
    } else if (zb) {   // page-locked, large: DMA from the caller's pages, every piece queued at once
        const uint64_t dper = per_piece(c->dma_chunk);
        e = ensure_hbm(piece_bytes(dper));
        if (e != hipSuccess) return hip_fail(e);
        for (uint64_t s0 = 0; s0 < n; s0 += dper) {
            const uint64_t cnt = (n - s0) < dper ? (n - s0) : dper;
            const uint8_t* src = (const uint8_t*)h_base + s0 * stride;
            const size_t mis = (uintptr_t)src & 15u;   // the in-place shape's alignment
            e = hipMemcpyAsync(c->d_buf + mis, src, piece_bytes(cnt), hipMemcpyHostToDevice, c->st);
            if (e != hipSuccess) return hip_fail(e);
            tcpcsum::launch_uniform(c->d_buf + mis, stride, len, kss ? kss + s0 : nullptr, sum_start, kout + s0, cnt,
                                    c->st, tu);
            rc = check_launch();
            if (rc) return rc;
        }
        e = wait_stream(c, c->st, expect_ns(span));
        if (e != hipSuccess) return hip_fail(e);
        drain.done = true;
    } else {
        const int ns = c->nslots;
        const size_t slot_bytes = piece_bytes(per) + 16;
        for (int i = 0; i < ns; ++i) {
            e = c->slot[i].ensure(slot_bytes);
            if (e != hipSuccess) return hip_fail(e);
        }
        if (c->uniform_dma) {
            e = ensure_hbm(piece_bytes(per));
            if (e != hipSuccess) return hip_fail(e);
        }
        uint64_t k = 0;
        // chunks ramp up from chunk / 8, doubling: the first copy, which nothing
        // overlaps, is short, and the later DMAs are long (per-copy overhead)
        size_t want = std::max<size_t>(c->chunk / 8, 1);
        // bulk_threads copy while the DMA is the bound; once a full chunk's DMA has
        // finished before the threads come back for its slot, the copy is the bound
        // (a slow host, or few threads): every copy thread from then on
        int copy_threads = c->bulk_threads;
        bool slot_full[4] = {false, false, false, false};
        for (uint64_t s0 = 0, pk = 0; s0 < n; s0 += pk, ++k) {
            const int s = (int)(k % (uint64_t)ns);
            pk = std::min<uint64_t>(per_piece(want), per);
            want = std::min(want * 2, c->chunk);
            const uint64_t cnt = (n - s0) < pk ? (n - s0) : pk;
            const size_t bytes = piece_bytes(cnt);
            const uint8_t* src = (const uint8_t*)h_base + s0 * stride;
            if (c->slot_busy[s]) {   // the DMA (or kernel) that last read this slot: chunk k - nslots
                c->slot_busy[s] = false;
                if (copy_threads != 0 && slot_full[s] && pk == per) {
                    if (hipEventQuery(c->slot_ev[s]) == hipSuccess) copy_threads = 0;
                    else (void)hipGetLastError();   // not ready: the DMA is still the bound
                }
                e = wait_slot(c, c->slot_ev[s]);
                if (e != hipSuccess) return hip_fail(e);
            }
            slot_full[s] = pk == per;
            // keep the start's alignment mod 16, so the kernel shape matches what the
            // same batch gets in place
            const size_t mis = (uintptr_t)src & 15u;
            par_copy(c, c->slot[s].h + mis, src, bytes, c->nt_copy, copy_threads);
            c->stats.bytes_staged += bytes;
            const uint8_t* kin = c->slot[s].d + mis;
            if (c->uniform_dma) {   // pinned -> HBM by the DMA engines, then the kernel reads HBM
                e = hipMemcpyAsync(c->d_buf + mis, c->slot[s].h + mis, bytes, hipMemcpyHostToDevice, c->st);
                if (e != hipSuccess) return hip_fail(e);
                e = hipEventRecord(c->slot_ev[s], c->st);
                if (e != hipSuccess) return hip_fail(e);
                kin = c->d_buf + mis;
            }
            tcpcsum::launch_uniform(kin, stride, len, kss ? kss + s0 : nullptr, sum_start, kout + s0, cnt, c->st, tu);
            rc = check_launch();
            if (rc) return rc;
            if (!c->uniform_dma) {
                e = hipEventRecord(c->slot_ev[s], c->st);
                if (e != hipSuccess) return hip_fail(e);
            }
            c->slot_busy[s] = true;
        }
        // what is left is about the last chunk's DMA and kernel
        for (int i = 0; i < 4; ++i) c->slot_busy[i] = false;
        e = wait_stream(c, c->st, expect_ns(std::min<uint64_t>(span, slot_bytes)));
        if (e != hipSuccess) return hip_fail(e);
        drain.done = true;
    }
    if (out_staged) par_copy(c, h_out, c->res.h, n * sizeof(uint16_t));
    return TCPCSUM_OK;
}

// Wire batch in one host region. A region that one page-locked allocation
// covers is read (FILL: written) in place over PCIe. A pageable region: the
// packets — not the slack between them — are copied into pinned staging, the
// kernel runs over the copies, and FILL's checks are stored back into the
// caller's packets. Per-packet arrays go through pinned staging when the
// caller's are pageable.
int tcpcsum_ipv4_batch_host(tcpcsum_ctx_t* c, void* h_pkts, size_t region_bytes, const uint64_t* h_pkt_off,
                            uint64_t n, uint32_t cap, int mode, uint16_t* h_out, uint8_t* h_status) {
    if (!c) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!h_pkts || !h_pkt_off || !region_bytes || (mode & ~3)) return TCPCSUM_EINVAL;
    if (cap > 65535u) cap = 65535u;
    // every packet header must lie inside the region; packets whose tot_len
    // runs past its end are SKIPPED by the kernel (limit = region_bytes)
    for (uint64_t i = 0; i < n; ++i)
        if (h_pkt_off[i] > region_bytes || region_bytes - h_pkt_off[i] < 20u) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    CallerCpu cpu(c);
    DeviceGuard g(c->device);
    hipStream_t st = c->st;
    DrainOnError drain(st);
    c->stats.batches++;
    int rc = ensure_pkt_arrays(c, n);
    if (rc) return rc;
    uint16_t* zout = h_out ? (uint16_t*)pinned_dev_ptr(h_out, n * sizeof(uint16_t)) : nullptr;
    uint8_t* zst = h_status ? (uint8_t*)pinned_dev_ptr(h_status, n) : nullptr;
    uint16_t* kout = zout ? zout : (uint16_t*)c->p_out.d;
    uint8_t* kst = zst ? zst : c->p_stat.d;
    const bool fill = (mode & TCPCSUM_IPV4_VERIFY) == 0;
    const tcpcsum::Tuning tu = host_wire_tuning(c, n);
    hipError_t e;
    uint8_t* zp = (uint8_t*)pinned_dev_ptr(h_pkts, region_bytes);
    c->g_idx.clear();
    if (zp) {
        const uint64_t* koff = (const uint64_t*)pinned_dev_ptr(h_pkt_off, n * sizeof(uint64_t));
        if (!koff) {
            memcpy(c->p_off.h, h_pkt_off, n * sizeof(uint64_t));
            koff = (const uint64_t*)c->p_off.d;
        }
        c->stats.pkts_in_place += n;
        tcpcsum::launch_ipv4(zp, koff, nullptr, n, cap, (uint64_t)region_bytes, (uint64_t)region_bytes, mode, kout,
                             kst, nullptr, st, tu);
    } else {
        // the region's packets, copied into staging and addressed one by one
        // (the scatter-gather kernel, bounded per packet by the bytes copied)
        uint8_t* base = (uint8_t*)h_pkts;
        c->g_off.resize(n);
        c->g_src.resize(n);
        c->g_len.resize(n);
        c->g_idx.resize(n);
        for (uint64_t i = 0; i < n; ++i) {   // bounds only: the copy threads read the headers
            c->g_idx[i] = i;
            c->g_src[i] = base + h_pkt_off[i];
            c->g_len[i] = (uint32_t)std::min<uint64_t>(cap, region_bytes - h_pkt_off[i]);
        }
        rc = stage_and_launch(c, n, 20u, 0u, mode, kout, kst, st, tu);
        if (rc) return rc;
    }
    rc = check_launch();
    if (rc) return rc;
    e = wait_stream(c, st, expect_ns(std::min<uint64_t>((uint64_t)n * std::min<uint64_t>(cap, 1500u), region_bytes)));
    if (e != hipSuccess) return hip_fail(e);
    drain.done = true;
    if (fill && !c->g_idx.empty())
        write_back_checks(c, zst ? h_status : c->p_stat.h, (mode & TCPCSUM_IPV4_IPHDR) != 0);
    if (h_out && !zout) memcpy(h_out, c->p_out.h, n * sizeof(uint16_t));
    if (h_status && !zst) memcpy(h_status, c->p_stat.h, n);
    return TCPCSUM_OK;
}

// Wire batch over the caller's own per-packet buffers (the loop's layout).
// Each packet is read in place when one page-locked allocation covers it
// (memory its owner page-locked: tcpcsum_host_alloc, hipHostRegister), else
// copied into pinned staging and its check stored back.
int tcpcsum_ipv4_batch_ptrs_host(tcpcsum_ctx_t* c, void* const* h_pkts, const uint32_t* h_lens, uint64_t n, int mode,
                                 uint16_t* h_out, uint8_t* h_status) {
    if (!c) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!h_pkts || !h_lens || (mode & ~3)) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    CallerCpu cpu(c);
    DeviceGuard g(c->device);
    hipStream_t st = c->st;
    DrainOnError drain(st);
    c->stats.batches++;
    int rc = ensure_pkt_arrays(c, n);
    if (rc) return rc;
    // page-locked memory is looked up afresh each batch (its owner may have freed it)
    c->pinned.begin_batch();
    uint64_t* k_off = (uint64_t*)c->p_off.h;
    uint32_t* k_len = (uint32_t*)c->p_len.h;
    c->g_idx.clear();
    c->g_off.clear();
    c->g_src.clear();
    c->g_len.clear();
    uint64_t foot = 0;
    const uint64_t staged_before = c->stats.bytes_staged;
    uint32_t cap = 20;
    uint64_t in_place = 0;
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t len = h_lens[i] > 65535u ? 65535u : h_lens[i];   // tot_len is a u16
        uint8_t* p = (uint8_t*)h_pkts[i];
        k_off[i] = 0;
        if (len < 20u || !p) {   // too short for an IP header: SKIPPED, nothing is read
            k_len[i] = 0;
            continue;
        }
        uintptr_t dev = 0;
        if (c->pinned.resolve((uintptr_t)p, len, &dev) == 0) {
            k_off[i] = dev;
            k_len[i] = len;
            foot += len;
            cap = len > cap ? len : cap;
            ++in_place;
        } else {   // staged: its bound now; its header, size and copy on the copy threads
            c->g_idx.push_back(i);
            c->g_src.push_back(p);
            c->g_len.push_back(len);
            c->g_off.push_back(0);
        }
    }
    c->stats.pkts_in_place += in_place;
    uint16_t* zout = h_out ? (uint16_t*)pinned_dev_ptr(h_out, n * sizeof(uint16_t)) : nullptr;
    uint8_t* zst = h_status ? (uint8_t*)pinned_dev_ptr(h_status, n) : nullptr;
    const tcpcsum::Tuning tu = host_wire_tuning(c, n);
    rc = stage_and_launch(c, n, cap, foot, mode, zout ? zout : (uint16_t*)c->p_out.d, zst ? zst : c->p_stat.d, st, tu);
    if (rc) return rc;
    hipError_t e = wait_stream(c, st, expect_ns(foot + c->stats.bytes_staged - staged_before));
    if (e != hipSuccess) return hip_fail(e);
    drain.done = true;
    if ((mode & TCPCSUM_IPV4_VERIFY) == 0 && !c->g_idx.empty())
        write_back_checks(c, zst ? h_status : c->p_stat.h, (mode & TCPCSUM_IPV4_IPHDR) != 0);
    if (h_out && !zout) memcpy(h_out, c->p_out.h, n * sizeof(uint16_t));
    if (h_status && !zst) memcpy(h_status, c->p_stat.h, n);
    return TCPCSUM_OK;
}

}  // extern "C"
