// tcpcsum_api.hip — the C ABI declared in include/tcpcsum.h.
//
// Argument checking, device checks, error mapping, the host-memory pipeline
// (tcpcsum_ctx_*) and the synthetic-workload entry points. All checksum
// arithmetic on the batch paths runs in the gfx950 kernels of
// tcpcsum_kernels.hip; this file never computes a checksum itself.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <mutex>
#include <new>
#include <vector>

#include "host_registry.h"
#include "tcpcsum.h"
#include "tcpcsum_internal.h"

namespace tcpcsum {

// HostRegistry backend over HIP: hipHostRegister'ed pages are mapped for the
// device (on MI355X hosts at their host address: tools/hostreg_probe.py).
struct HipHostBackend {
    int last_error = 0;
    int lock(uintptr_t lo, size_t bytes, intptr_t* delta) {
        hipError_t e = hipHostRegister((void*)lo, bytes, hipHostRegisterMapped);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            last_error = (int)e;
            return TCPCSUM_EHIP;
        }
        void* d = nullptr;
        e = hipHostGetDevicePointer(&d, (void*)lo, 0);
        if (e != hipSuccess || !d) {
            (void)hipGetLastError();
            (void)hipHostUnregister((void*)lo);
            last_error = (int)(e != hipSuccess ? e : hipErrorInvalidValue);
            return TCPCSUM_EHIP;
        }
        *delta = (intptr_t)d - (intptr_t)lo;
        return 0;
    }
    void unlock(uintptr_t lo) {
        if (hipHostUnregister((void*)lo) != hipSuccess) (void)hipGetLastError();   // nothing to undo
    }
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

}  // namespace tcpcsum

static_assert(sizeof(tcpcsum_desc_t) == 16, "descriptor is read as one 16-B load");
static_assert(sizeof(tcpcsum_txseg_t) == 48, "tx descriptor is read as three 16-B loads");

namespace {

// Diagnostics only (the hipError_t behind the last TCPCSUM_EHIP) and the
// per-device arch cache below; nothing that changes what a launch does.
std::atomic<int> g_last_hip_error{0};

constexpr int kMaxDevices = 64;
std::atomic<int> g_dev_ok[kMaxDevices];   // 0 unknown, 1 gfx950, -1 unusable

int hip_fail(hipError_t e) {
    g_last_hip_error.store((int)e);
    return TCPCSUM_EHIP;
}

// The launch shapes of one call: *t, or the built-in defaults for NULL.
int get_tuning(const tcpcsum_tuning_t* t, tcpcsum::Tuning* out) {
    tcpcsum::Tuning r;
    if (t) {
        const int u = t->unroll;
        if (t->max_blocks < 0 || !(u == 0 || u == 1 || u == 2 || u == 4 || u == 8) || t->shape < -1 ||
            t->shape > 13 || (t->flags & ~511) || (t->flags & 3) == 3 || (t->flags & 12) == 12)
            return TCPCSUM_EINVAL;
        r.max_blocks = t->max_blocks;
        r.unroll = t->unroll;
        r.shape = t->shape;
        r.flags = t->flags;
    }
    *out = r;
    return TCPCSUM_OK;
}

// The current device must be a gfx950 (the only code object in this library).
int require_device(char* arch, size_t arch_len) {
    int dev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess || dev < 0) {
        g_last_hip_error.store((int)e);
        return TCPCSUM_ENODEV;
    }
    if (dev < kMaxDevices && !arch) {
        const int v = g_dev_ok[dev].load(std::memory_order_relaxed);
        if (v == 1) return TCPCSUM_OK;
        if (v == -1) return TCPCSUM_ENODEV;
    }
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) {
        g_last_hip_error.store((int)e);
        return TCPCSUM_ENODEV;
    }
    if (arch && arch_len) {
        strncpy(arch, prop.gcnArchName, arch_len - 1);
        arch[arch_len - 1] = 0;
    }
    const bool ok = strncmp(prop.gcnArchName, "gfx950", 6) == 0;
    if (dev < kMaxDevices) g_dev_ok[dev].store(ok ? 1 : -1);
    return ok ? TCPCSUM_OK : TCPCSUM_ENODEV;
}

int check_launch() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? TCPCSUM_OK : hip_fail(e);
}

}  // namespace

extern "C" {

int tcpcsum_abi_version(void) { return TCPCSUM_ABI_VERSION; }

const char* tcpcsum_strerror(int code) {
    switch (code) {
        case TCPCSUM_OK: return "ok";
        case TCPCSUM_EINVAL: return "invalid argument";
        case TCPCSUM_ENODEV: return "no usable gfx950 device";
        case TCPCSUM_EHIP: return "HIP runtime error";
        case TCPCSUM_ENOMEM: return "out of memory";
        default: return "unknown error";
    }
}

int tcpcsum_last_hip_error(void) { return g_last_hip_error.load(); }

int tcpcsum_device_check(char* arch, size_t arch_len) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) {
        g_last_hip_error.store((int)e);
        if (arch && arch_len) arch[0] = 0;
        return TCPCSUM_ENODEV;
    }
    return require_device(arch, arch_len);
}

int tcpcsum_tuning_check(const tcpcsum_tuning_t* tune) {
    tcpcsum::Tuning t;
    return get_tuning(tune, &t);
}

int tcpcsum_plan_uniform(uint64_t base, uint64_t stride, uint32_t len, uint64_t n, const tcpcsum_tuning_t* tune,
                         int* mode, int* shape, int* unroll, int* max_blocks) {
    if (!mode || !shape || !unroll || !max_blocks || len > (uint32_t)INT_MAX) return TCPCSUM_EINVAL;
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    const tcpcsum::UniformPlan p = tcpcsum::plan_uniform((uintptr_t)base, stride, len, n, tu);
    *mode = p.mode;
    *shape = p.shape;
    *unroll = p.unroll;
    *max_blocks = p.max_blocks;
    return TCPCSUM_OK;
}

int tcpcsum_batch_uniform_dev(const void* d_base, uint64_t stride, uint32_t len, const uint32_t* d_sum_start,
                              uint32_t sum_start, uint16_t* d_out, uint64_t n, void* stream,
                              const tcpcsum_tuning_t* tune) {
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!d_base || !d_out || len > (uint32_t)INT_MAX) return TCPCSUM_EINVAL;
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    tcpcsum::launch_uniform((const uint8_t*)d_base, stride, len, d_sum_start, sum_start, d_out, n,
                            (hipStream_t)stream, tu);
    return check_launch();
}

int tcpcsum_batch_desc_dev(const void* d_base, const tcpcsum_desc_t* d_desc, uint64_t n, uint32_t max_len,
                           uint16_t* d_out, void* stream, const tcpcsum_tuning_t* tune) {
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!d_base || !d_desc || !d_out || max_len > (uint32_t)INT_MAX) return TCPCSUM_EINVAL;
    if (((uintptr_t)d_desc) & 15u) return TCPCSUM_EINVAL;   // descriptors are read as one 16-B load
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    tcpcsum::launch_desc((const uint8_t*)d_base, d_desc, n, max_len, d_out, (hipStream_t)stream, tu);
    return check_launch();
}

int tcpcsum_ipv4_batch_dev(void* d_pkts, uint64_t region_bytes, const uint64_t* d_pkt_off, uint64_t n, uint32_t cap,
                           int mode, uint16_t* d_out, uint8_t* d_status, void* stream, const tcpcsum_tuning_t* tune) {
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!d_pkts || !d_pkt_off || !region_bytes || (mode & ~3)) return TCPCSUM_EINVAL;
    if (cap > 65535u) cap = 65535u;   // tot_len is a u16
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    tcpcsum::launch_ipv4((uint8_t*)d_pkts, d_pkt_off, nullptr, n, cap, region_bytes, region_bytes, mode, d_out,
                         d_status, nullptr, (hipStream_t)stream, tu);
    return check_launch();
}

int tcpcsum_ipv4_batch_ptrs_dev(void* const* d_pkt_ptrs, const uint32_t* d_lens, uint64_t n, uint32_t cap, int mode,
                                uint16_t* d_out, uint8_t* d_status, void* stream, const tcpcsum_tuning_t* tune) {
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!d_pkt_ptrs || !d_lens || (mode & ~3) || (((uintptr_t)d_pkt_ptrs) & 7u) || (((uintptr_t)d_lens) & 3u))
        return TCPCSUM_EINVAL;
    if (cap > 65535u) cap = 65535u;
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    // addresses as offsets from 0, bounded per packet by d_lens
    tcpcsum::launch_ipv4(nullptr, (const uint64_t*)d_pkt_ptrs, d_lens, n, cap, ~0ull, n * (uint64_t)cap, mode, d_out,
                         d_status, nullptr, (hipStream_t)stream, tu);
    return check_launch();
}

int tcpcsum_tx_build_dev(const void* d_payload, const tcpcsum_txseg_t* d_segs, uint64_t n, uint32_t max_len,
                         void* d_out_pkts, int mode, uint16_t* d_check, void* stream, const tcpcsum_tuning_t* tune) {
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!d_segs || !d_out_pkts || (mode & ~TCPCSUM_IPV4_IPHDR) || (((uintptr_t)d_segs) & 15u))
        return TCPCSUM_EINVAL;
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    tcpcsum::launch_tx_build((const uint8_t*)d_payload, d_segs, n, max_len, (uint8_t*)d_out_pkts, mode, d_check,
                             (hipStream_t)stream, tu);
    return check_launch();
}

int tcpcsum_synth_fill_dev(void* d_dst, uint64_t stream_off, uint64_t nbytes, void* stream) {
    if (nbytes == 0) return TCPCSUM_OK;
    if (!d_dst) return TCPCSUM_EINVAL;
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    tcpcsum::launch_synth_fill((uint8_t*)d_dst, stream_off, nbytes, (hipStream_t)stream);
    return check_launch();
}

int tcpcsum_synth_pseudo_dev(uint32_t* d_sum_start, uint64_t seg0, uint64_t n, uint32_t seg_len, void* stream) {
    if (n == 0) return TCPCSUM_OK;
    if (!d_sum_start) return TCPCSUM_EINVAL;
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    tcpcsum::launch_synth_pseudo(d_sum_start, seg0, n, seg_len, (hipStream_t)stream);
    return check_launch();
}

int tcpcsum_stream_probe_dev(const void* d_src, uint64_t nbytes, uint64_t* d_partials, int* n_partials,
                             void* stream, const tcpcsum_tuning_t* tune) {
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    if (!d_src || !d_partials || !n_partials || (nbytes & 15u) || (((uintptr_t)d_src) & 15u))
        return TCPCSUM_EINVAL;
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    *n_partials = tcpcsum::launch_probe((const uint8_t*)d_src, nbytes, d_partials, (hipStream_t)stream, tu);
    return check_launch();
}

// ------------------------------------------------------------------ host path

struct tcpcsum_ctx {
    int device = 0;
    size_t scratch = 0;
    hipStream_t st[2] = {nullptr, nullptr};
    uint8_t* d_buf[2] = {nullptr, nullptr};
    size_t d_buf_bytes = 0;
    uint32_t* d_ss[2] = {nullptr, nullptr};
    uint16_t* d_out[2] = {nullptr, nullptr};
    size_t d_seg_cap = 0;   // entries of d_ss / d_out per slot
    // wire path
    uint8_t* d_region = nullptr;
    size_t d_region_bytes = 0;
    // pinned staging of the per-packet arrays (offsets in; results, status and
    // IPv4 header checks out), host views h_* and device views k_*: a pageable
    // caller array costs a CPU memcpy and the kernel reads / writes the staging
    // over PCIe, instead of a staged pageable hipMemcpy per array per batch
    uint64_t* h_off = nullptr;
    uint16_t* h_wout = nullptr;
    uint8_t* h_wstat = nullptr;
    uint16_t* h_wip = nullptr;
    uint64_t* k_off = nullptr;
    uint16_t* k_wout = nullptr;
    uint8_t* k_wstat = nullptr;
    uint16_t* k_wip = nullptr;
    uint32_t* h_len = nullptr;   // scatter-gather batches: per-packet readable bytes
    uint32_t* k_len = nullptr;
    // two pinned bounce buffers for every copy from / to host memory that is not
    // page-locked as a whole: pageable memory never reaches a HIP copy (whose
    // pageable path pins the user pages in place, under the same pages this
    // context registers for scatter-gather batches), and ranges only partly
    // page-locked would make HIP copy them as locked from their first page.
    // bounce_ev[i]: the last copy through h_bounce[i] (recorded on its stream)
    uint8_t* h_bounce[2] = {nullptr, nullptr};
    hipEvent_t bounce_ev[2] = {nullptr, nullptr};
    bool bounce_busy[2] = {false, false};
    size_t pkt_cap = 0;
    // launch shapes of this context's batches (tcpcsum_ctx_set_tuning)
    tcpcsum::Tuning tune;
    // host pages this context page-locked for scatter-gather batches
    tcpcsum::HipHostBackend backend;
    tcpcsum::HostRegistry<tcpcsum::HipHostBackend> reg{backend};
    std::mutex mu;
};

namespace {

void ctx_free_buffers(tcpcsum_ctx* c) {
    for (int i = 0; i < 2; ++i) {
        if (c->d_buf[i]) hipFree(c->d_buf[i]);
        if (c->d_ss[i]) hipFree(c->d_ss[i]);
        if (c->d_out[i]) hipFree(c->d_out[i]);
        c->d_buf[i] = nullptr;
        c->d_ss[i] = nullptr;
        c->d_out[i] = nullptr;
    }
    c->d_buf_bytes = 0;
    c->d_seg_cap = 0;
}

int ctx_ensure(tcpcsum_ctx* c, size_t buf_bytes, size_t segs) {
    if (buf_bytes > c->d_buf_bytes || segs > c->d_seg_cap) {
        for (int i = 0; i < 2; ++i) hipStreamSynchronize(c->st[i]);
        const size_t nb = buf_bytes > c->d_buf_bytes ? buf_bytes : c->d_buf_bytes;
        const size_t ns = segs > c->d_seg_cap ? segs : c->d_seg_cap;
        ctx_free_buffers(c);
        for (int i = 0; i < 2; ++i) {
            hipError_t e = hipMalloc(&c->d_buf[i], nb);
            if (e == hipSuccess) e = hipMalloc(&c->d_ss[i], ns * sizeof(uint32_t));
            if (e == hipSuccess) e = hipMalloc(&c->d_out[i], ns * sizeof(uint16_t));
            if (e != hipSuccess) {
                ctx_free_buffers(c);
                g_last_hip_error.store((int)e);
                return TCPCSUM_ENOMEM;
            }
        }
        c->d_buf_bytes = nb;
        c->d_seg_cap = ns;
    }
    return TCPCSUM_OK;
}

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

}  // namespace

int tcpcsum_ctx_create(int device, size_t scratch_bytes, tcpcsum_ctx_t** out) {
    if (!out) return TCPCSUM_EINVAL;
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || device < 0 || device >= count) {
        g_last_hip_error.store((int)e);
        return TCPCSUM_ENODEV;
    }
    DeviceGuard g(device);
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    tcpcsum_ctx* c = new (std::nothrow) tcpcsum_ctx();
    if (!c) return TCPCSUM_ENOMEM;
    c->device = device;
    c->scratch = scratch_bytes ? scratch_bytes : (64u << 20);
    for (int i = 0; i < 2; ++i) {
        e = hipStreamCreateWithFlags(&c->st[i], hipStreamNonBlocking);
        if (e != hipSuccess) {
            tcpcsum_ctx_destroy(c);
            return hip_fail(e);
        }
    }
    *out = c;
    return TCPCSUM_OK;
}

void tcpcsum_ctx_destroy(tcpcsum_ctx_t* c) {
    if (!c) return;
    DeviceGuard g(c->device);
    for (int i = 0; i < 2; ++i)
        if (c->st[i]) hipStreamSynchronize(c->st[i]);
    ctx_free_buffers(c);
    if (c->d_region) hipFree(c->d_region);
    if (c->h_off) hipHostFree(c->h_off);
    if (c->h_wout) hipHostFree(c->h_wout);
    if (c->h_wstat) hipHostFree(c->h_wstat);
    if (c->h_wip) hipHostFree(c->h_wip);
    if (c->h_len) hipHostFree(c->h_len);
    for (int i = 0; i < 2; ++i) {
        if (c->h_bounce[i]) hipHostFree(c->h_bounce[i]);
        if (c->bounce_ev[i]) hipEventDestroy(c->bounce_ev[i]);
    }
    c->reg.release(0, 0);
    for (int i = 0; i < 2; ++i)
        if (c->st[i]) hipStreamDestroy(c->st[i]);
    delete c;
}

int tcpcsum_ctx_set_tuning(tcpcsum_ctx_t* c, const tcpcsum_tuning_t* tune) {
    if (!c) return TCPCSUM_EINVAL;
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->tune = tu;
    return TCPCSUM_OK;
}

void* tcpcsum_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (!bytes) return nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        g_last_hip_error.store((int)e);
        return nullptr;
    }
    return p;
}

void tcpcsum_host_free(void* p) {
    if (p) hipHostFree(p);
}

namespace {

// Device-visible address of page-locked (hipHostMalloc / hipHostRegister'ed)
// host memory [p, p + bytes), or nullptr when any of it is pageable. Kernels
// read and write such memory directly over PCIe ("zero-copy"): no staging copy,
// only the bytes the kernel touches cross the link. The whole range must lie in
// ONE page-locked allocation or registration — a region only partly locked
// (its first page locked by a neighbouring registration, say) takes the copy
// path instead of letting a kernel touch unlocked pages.
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

constexpr size_t kBounce = 4u << 20;

hipError_t ensure_bounce(tcpcsum_ctx* c) {
    for (int i = 0; i < 2; ++i) {
        if (!c->h_bounce[i]) {
            hipError_t e = hipHostMalloc((void**)&c->h_bounce[i], kBounce, hipHostMallocDefault);
            if (e != hipSuccess) return e;
        }
        if (!c->bounce_ev[i]) {
            hipError_t e = hipEventCreateWithFlags(&c->bounce_ev[i], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

// Bounce buffer i is free again (its last copy, on whatever stream, is done).
hipError_t bounce_wait(tcpcsum_ctx* c, int i) {
    if (!c->bounce_busy[i]) return hipSuccess;
    c->bounce_busy[i] = false;
    return hipEventSynchronize(c->bounce_ev[i]);
}

// Host -> device on st. Page-locked source: one async DMA. Otherwise chunks of
// at most 4 MiB alternate between the two bounce buffers: the CPU copy of
// chunk k+1 overlaps the DMA of chunk k. Returns with the DMAs queued on st.
hipError_t copy_h2d(tcpcsum_ctx* c, void* d, const void* h, size_t n, hipStream_t st) {
    if (pinned_dev_ptr(h, n)) return hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st);
    hipError_t e = ensure_bounce(c);
    int i = 0;
    for (size_t o = 0; o < n && e == hipSuccess; o += kBounce, i ^= 1) {
        const size_t k = n - o < kBounce ? n - o : kBounce;
        e = bounce_wait(c, i);
        if (e != hipSuccess) break;
        memcpy(c->h_bounce[i], (const uint8_t*)h + o, k);
        e = hipMemcpyAsync((uint8_t*)d + o, c->h_bounce[i], k, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipEventRecord(c->bounce_ev[i], st);
        if (e == hipSuccess) c->bounce_busy[i] = true;
    }
    return e;
}

// Device -> host on st. Page-locked destination: one async DMA, queued on st.
// Otherwise through the bounce buffers, the DMA of chunk k+1 overlapping the
// CPU copy-out of chunk k, and complete on return.
hipError_t copy_d2h(tcpcsum_ctx* c, void* h, const void* d, size_t n, hipStream_t st) {
    if (pinned_dev_ptr(h, n)) return hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, st);
    hipError_t e = ensure_bounce(c);
    size_t prev_o = 0, prev_k = 0;
    int i = 0;
    for (size_t o = 0; o < n && e == hipSuccess; o += kBounce, i ^= 1) {
        const size_t k = n - o < kBounce ? n - o : kBounce;
        e = bounce_wait(c, i);
        if (e != hipSuccess) break;
        e = hipMemcpyAsync(c->h_bounce[i], (const uint8_t*)d + o, k, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipEventRecord(c->bounce_ev[i], st);
        if (e != hipSuccess) break;
        c->bounce_busy[i] = true;
        if (prev_k) {   // the previous chunk, while this one is in flight
            e = bounce_wait(c, i ^ 1);
            if (e == hipSuccess) memcpy((uint8_t*)h + prev_o, c->h_bounce[i ^ 1], prev_k);
        }
        prev_o = o;
        prev_k = k;
    }
    if (e == hipSuccess && prev_k) {
        e = bounce_wait(c, i ^ 1);
        if (e == hipSuccess) memcpy((uint8_t*)h + prev_o, c->h_bounce[i ^ 1], prev_k);
    }
    return e;
}

// One call's page locks of pageable host ranges: the pages under each range
// are registered for the call, the kernel reads (FILL: writes) them in place
// over PCIe, and they are unregistered once the call's streams have drained —
// never a HIP copy from pageable memory (whose pin-in-place is HIP's own,
// under pages this library also registers) and no staging copy of the bytes.
// Registering costs about 120 us for 32 MiB on MI355X hosts
// (tools/pin_cache_probe.cpp). Ranges come in increasing address order (the
// chunks of one batch): pages an earlier range already locked are not locked
// again. Requires the mapping at the host address (as every registration on
// MI355X hosts is), since a range may span two registrations. When a range
// cannot be registered (some page locked by someone else, a mapping that
// refuses it, a mapping elsewhere), pin() returns nullptr and the caller
// copies through the bounce buffers instead.
struct PinSet {
    hipStream_t st[2];
    std::vector<uintptr_t> los;
    uintptr_t lo = 0, hi = 0;   // [lo, hi): pages locked so far, contiguous
    PinSet(hipStream_t a, hipStream_t b) : st{a, b} {}
    PinSet(const PinSet&) = delete;
    PinSet& operator=(const PinSet&) = delete;
    ~PinSet() { release(); }
    const void* pin(const void* p, size_t n) {
        uintptr_t a = (uintptr_t)p & ~(uintptr_t)4095;
        const uintptr_t b = ((uintptr_t)p + n + 4095) & ~(uintptr_t)4095;
        const bool joins = !los.empty() && a >= lo && a <= hi;   // continues the locked run
        if (joins) a = hi;
        if (a < b) {
            void* d = nullptr;
            if (hipHostRegister((void*)a, b - a, hipHostRegisterMapped) != hipSuccess) {
                (void)hipGetLastError();
                return nullptr;
            }
            if (hipHostGetDevicePointer(&d, (void*)a, 0) != hipSuccess || (uintptr_t)d != a) {
                (void)hipGetLastError();
                (void)hipHostUnregister((void*)a);
                (void)hipGetLastError();
                return nullptr;
            }
            los.push_back(a);
            if (!joins) lo = a;
            hi = b;
        }
        return p;   // mapped at its host address
    }
    // after every kernel that reads the pages (queued on st[0] / st[1]) is done
    void release() {
        if (los.empty()) return;
        for (hipStream_t s : st)
            if (s) (void)hipStreamSynchronize(s);
        for (uintptr_t a : los)
            if (hipHostUnregister((void*)a) != hipSuccess) (void)hipGetLastError();
        los.clear();
        lo = hi = 0;
    }
};

// Pageable ranges at least this large are page-locked for the call rather than
// copied through the bounce buffers.
constexpr size_t kTempPinMin = 64u << 10;

int ensure_pkt_staging(tcpcsum_ctx* c, uint64_t n, hipStream_t st) {
    if (n <= c->pkt_cap) return TCPCSUM_OK;
    (void)hipStreamSynchronize(st);
    if (c->h_off) (void)hipHostFree(c->h_off);
    if (c->h_wout) (void)hipHostFree(c->h_wout);
    if (c->h_wstat) (void)hipHostFree(c->h_wstat);
    if (c->h_wip) (void)hipHostFree(c->h_wip);
    if (c->h_len) (void)hipHostFree(c->h_len);
    c->h_off = nullptr; c->h_wout = nullptr; c->h_wstat = nullptr; c->h_wip = nullptr; c->h_len = nullptr;
    c->pkt_cap = 0;
    size_t cap = 1024;
    while (cap < n) cap *= 2;
    hipError_t e = hipHostMalloc((void**)&c->h_off, cap * sizeof(uint64_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_wout, cap * sizeof(uint16_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_wstat, cap, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_wip, cap * sizeof(uint16_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_len, cap * sizeof(uint32_t), hipHostMallocDefault);
    if (e != hipSuccess) { g_last_hip_error.store((int)e); return TCPCSUM_ENOMEM; }
    c->k_off = (uint64_t*)pinned_dev_ptr(c->h_off);
    c->k_wout = (uint16_t*)pinned_dev_ptr(c->h_wout);
    c->k_wstat = (uint8_t*)pinned_dev_ptr(c->h_wstat);
    c->k_wip = (uint16_t*)pinned_dev_ptr(c->h_wip);
    c->k_len = (uint32_t*)pinned_dev_ptr(c->h_len);
    if (!c->k_off || !c->k_wout || !c->k_wstat || !c->k_wip || !c->k_len) return TCPCSUM_ENOMEM;
    c->pkt_cap = cap;
    return TCPCSUM_OK;
}

}  // namespace

// Pinned input: one launch reads the segments in host memory directly.
// Pageable input: chunks of segments alternate between two slots (stream +
// device buffers), each page-locked for the call and read in place (or copied
// through the bounce buffers), so locking chunk k+1 overlaps the kernel of
// chunk k and collecting chunk k's results overlaps the kernel of chunk k+1.
int tcpcsum_batch_uniform_host(tcpcsum_ctx_t* c, const void* h_base, uint64_t stride, uint32_t len,
                               const uint32_t* h_sum_start, uint32_t sum_start, uint16_t* h_out, uint64_t n) {
    if (!c) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!h_base || !h_out || len > (uint32_t)INT_MAX) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    const tcpcsum::Tuning tu = c->tune;
    hipError_t e;
    int rc;
    const size_t span = (size_t)((n - 1) * stride + len);
    if (const uint8_t* zb = (const uint8_t*)pinned_dev_ptr(h_base, span)) {
        hipStream_t st = c->st[0];
        const uint32_t* zss = nullptr;
        if (h_sum_start) zss = (const uint32_t*)pinned_dev_ptr(h_sum_start, n * sizeof(uint32_t));
        uint16_t* zout = (uint16_t*)pinned_dev_ptr(h_out, n * sizeof(uint16_t));
        if ((h_sum_start && !zss) || !zout) {   // stage the small arrays
            rc = ctx_ensure(c, 16, (size_t)n);
            if (rc) return rc;
        }
        if (h_sum_start && !zss) {
            e = copy_h2d(c, c->d_ss[0], h_sum_start, n * sizeof(uint32_t), st);
            if (e != hipSuccess) return hip_fail(e);
            zss = c->d_ss[0];
        }
        tcpcsum::launch_uniform(zb, stride, len, zss, sum_start, zout ? zout : c->d_out[0], n, st, tu);
        rc = check_launch();
        if (rc) return rc;
        if (!zout) {
            e = copy_d2h(c, h_out, c->d_out[0], n * sizeof(uint16_t), st);
            if (e != hipSuccess) return hip_fail(e);
        }
        e = hipStreamSynchronize(st);
        return e == hipSuccess ? TCPCSUM_OK : hip_fail(e);
    }
    // segments per chunk: (cnt-1)*stride + len <= scratch (at least one segment)
    uint64_t per = 1;
    if (stride == 0) per = n;
    else if (c->scratch > len) per = (c->scratch - len) / stride + 1;
    if (per > n) per = n;
    const uint64_t chunk_bytes = (per - 1) * stride + len;
    rc = ctx_ensure(c, (size_t)chunk_bytes + 16, (size_t)per);
    if (rc) return rc;
    // Chunks alternate between two streams. Each chunk's bytes are page-locked
    // for the call and read in place (else copied through the bounce buffers);
    // locking chunk k and collecting chunk k-1's results overlap kernel k-1 / k.
    uint16_t* zout = (uint16_t*)pinned_dev_ptr(h_out, n * sizeof(uint16_t));
    PinSet pins(c->st[0], c->st[1]);
    uint64_t prev_s0 = 0, prev_cnt = 0;
    int prev_slot = -1;
    uint64_t k = 0;
    for (uint64_t s0 = 0; s0 < n; s0 += per, ++k) {
        const int slot = (int)(k & 1);
        hipStream_t st = c->st[slot];
        const uint64_t cnt = (n - s0) < per ? (n - s0) : per;
        const uint64_t bytes = (cnt - 1) * stride + len;
        const uint8_t* src = (const uint8_t*)h_base + s0 * stride;
        // slot's previous chunk (k-2) finished when its results were collected
        const uint8_t* in = bytes >= kTempPinMin ? (const uint8_t*)pins.pin(src, bytes) : nullptr;
        if (!in) {
            // keep the device-side start alignment mod 16 equal to the host's so
            // the kernel shape matches what the same batch gets on device memory
            const size_t mis = (uintptr_t)src & 15u;
            e = copy_h2d(c, c->d_buf[slot] + mis, src, bytes, st);
            if (e != hipSuccess) return hip_fail(e);
            in = c->d_buf[slot] + mis;
        }
        if (h_sum_start) {
            e = copy_h2d(c, c->d_ss[slot], h_sum_start + s0, cnt * sizeof(uint32_t), st);
            if (e != hipSuccess) return hip_fail(e);
        }
        tcpcsum::launch_uniform(in, stride, len, h_sum_start ? c->d_ss[slot] : nullptr, sum_start,
                                zout ? zout + s0 : c->d_out[slot], cnt, st, tu);
        rc = check_launch();
        if (rc) return rc;
        if (prev_slot >= 0 && !zout) {   // chunk k-1's results, while chunk k runs
            e = copy_d2h(c, h_out + prev_s0, c->d_out[prev_slot], prev_cnt * sizeof(uint16_t), c->st[prev_slot]);
            if (e != hipSuccess) return hip_fail(e);
        }
        prev_s0 = s0;
        prev_cnt = cnt;
        prev_slot = slot;
    }
    if (prev_slot >= 0 && !zout) {
        e = copy_d2h(c, h_out + prev_s0, c->d_out[prev_slot], prev_cnt * sizeof(uint16_t), c->st[prev_slot]);
        if (e != hipSuccess) return hip_fail(e);
    }
    for (int i = 0; i < 2; ++i) {
        e = hipStreamSynchronize(c->st[i]);
        if (e != hipSuccess) return hip_fail(e);
    }
    return TCPCSUM_OK;
}

// Pinned packet pool: the kernel reads each packet's bytes over PCIe and (FILL)
// stores the check field in place in host memory — no staging of the packets.
// A pageable pool is page-locked for the call and read the same way; one that
// cannot be (or a small one) is copied H2D through pinned bounce buffers,
// checksummed, and the results are stored at TCP+16 on the host. Either way
// the per-packet arrays (offsets in,
// results and status out) go through the context's pinned staging when the
// caller's are pageable: a CPU memcpy and zero-copy kernel access instead of a
// pageable hipMemcpy (a staged, synchronous copy) per array per batch.
int tcpcsum_ipv4_batch_host(tcpcsum_ctx_t* c, void* h_pkts, size_t region_bytes, const uint64_t* h_pkt_off,
                            uint64_t n, uint32_t cap, int mode, uint16_t* h_out, uint8_t* h_status) {
    if (!c) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!h_pkts || !h_pkt_off || !region_bytes || (mode & ~3)) return TCPCSUM_EINVAL;
    if (cap > 65535u) cap = 65535u;
    // every packet header must lie inside the region; packets whose tot_len
    // runs past its end are SKIPPED by the kernel (limit = region_bytes)
    for (uint64_t i = 0; i < n; ++i)
        if (h_pkt_off[i] + 20u > region_bytes) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t st = c->st[0];
    int rc = ensure_pkt_staging(c, n, st);
    if (rc) return rc;
    const uint64_t* koff = (const uint64_t*)pinned_dev_ptr(h_pkt_off, n * sizeof(uint64_t));
    if (!koff) {
        memcpy(c->h_off, h_pkt_off, n * sizeof(uint64_t));
        koff = c->k_off;
    }
    uint16_t* zout = h_out ? (uint16_t*)pinned_dev_ptr(h_out, n * sizeof(uint16_t)) : nullptr;
    uint8_t* zst = h_status ? (uint8_t*)pinned_dev_ptr(h_status, n) : nullptr;
    uint16_t* kout = zout ? zout : c->k_wout;
    uint8_t* kst = zst ? zst : c->k_wstat;
    const bool fill = (mode & TCPCSUM_IPV4_VERIFY) == 0;
    hipError_t e;
    PinSet tp(st, nullptr);
    uint8_t* zp = (uint8_t*)pinned_dev_ptr(h_pkts, region_bytes);
    if (!zp && region_bytes >= kTempPinMin) zp = (uint8_t*)const_cast<void*>(tp.pin(h_pkts, region_bytes));
    if (zp) {
        // zero-copy over PCIe: 16-lane groups, 512 B per round (more waves with
        // reads in flight) beat the HBM-tuned MTU shape — 1024 x 1500-B FILL
        // batch 49 vs 59 us on MI355X (tools/e2e.py --sweep)
        tcpcsum::Tuning tu = c->tune;
        if (tu.shape < 0 && n < 65536u) tu.shape = 3;
        tcpcsum::launch_ipv4(zp, koff, nullptr, n, cap, (uint64_t)region_bytes, (uint64_t)region_bytes, mode, kout,
                             kst, nullptr, st, tu);
        rc = check_launch();
        if (rc) return rc;
        e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_fail(e);
        tp.release();
    } else {
        const size_t mis = (uintptr_t)h_pkts & 15u;
        const size_t need = region_bytes + mis + 16u;
        if (need > c->d_region_bytes) {
            (void)hipStreamSynchronize(st);
            if (c->d_region) (void)hipFree(c->d_region);
            c->d_region = nullptr;
            c->d_region_bytes = 0;
            e = hipMalloc(&c->d_region, need);
            if (e != hipSuccess) { g_last_hip_error.store((int)e); return TCPCSUM_ENOMEM; }
            c->d_region_bytes = need;
        }
        e = copy_h2d(c, c->d_region + mis, h_pkts, region_bytes, st);
        if (e != hipSuccess) return hip_fail(e);
        const bool ipfill = fill && (mode & TCPCSUM_IPV4_IPHDR);
        tcpcsum::launch_ipv4(c->d_region + mis, koff, nullptr, n, cap, (uint64_t)region_bytes,
                             (uint64_t)region_bytes, mode, kout, kst, ipfill ? c->k_wip : nullptr, st, c->tune);
        rc = check_launch();
        if (rc) return rc;
        e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_fail(e);
        if (fill) {
            // store each result at TCP+16 (native u16, as context.c:208), and the IP
            // header checksum the kernel computed — no arithmetic here
            const uint16_t* o = zout ? h_out : c->h_wout;
            const uint8_t* s = zst ? h_status : c->h_wstat;
            uint8_t* base = (uint8_t*)h_pkts;
            for (uint64_t i = 0; i < n; ++i) {
                if (s[i] != TCPCSUM_PKT_OK) continue;
                uint8_t* ip = base + h_pkt_off[i];
                uint8_t* tcp = ip + (ip[0] & 15u) * 4u;
                memcpy(tcp + 16, &o[i], 2);
                if (ipfill) memcpy(ip + 10, &c->h_wip[i], 2);
            }
        }
    }
    if (h_out && !zout) memcpy(h_out, c->h_wout, n * sizeof(uint16_t));
    if (h_status && !zst) memcpy(h_status, c->h_wstat, n);
    return TCPCSUM_OK;
}


// ------------------------------------------------- scatter-gather host batches

int tcpcsum_ipv4_batch_ptrs_host(tcpcsum_ctx_t* c, void* const* h_pkts, const uint32_t* h_lens, uint64_t n, int mode,
                                 uint16_t* h_out, uint8_t* h_status) {
    if (!c) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!h_pkts || !h_lens || (mode & ~3)) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    hipStream_t st = c->st[0];
    int rc = ensure_pkt_staging(c, n, st);
    if (rc) return rc;
    // per-packet device addresses and bounds, straight into the pinned staging
    // the kernel reads (no copy of packet bytes anywhere); memory pinned by
    // someone else is looked up afresh each batch (its owner may have freed it)
    c->reg.forget_foreign();
    uint64_t foot = 0;
    uint32_t cap = 20;
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t len = h_lens[i] > 65535u ? 65535u : h_lens[i];   // tot_len is a u16
        const uintptr_t p = (uintptr_t)h_pkts[i];
        uintptr_t dev = 0;
        if (len >= 20u && p) {
            rc = c->reg.resolve(p, len, &dev);
            if (rc == TCPCSUM_EHIP) g_last_hip_error.store(c->backend.last_error);
            if (rc) return rc == TCPCSUM_EHIP ? rc : TCPCSUM_EINVAL;
        } else {
            len = 0;   // too short for an IP header: SKIPPED, nothing is read
        }
        c->h_off[i] = dev;
        c->h_len[i] = len;
        foot += len;
        cap = len > cap ? len : cap;
    }
    uint16_t* zout = h_out ? (uint16_t*)pinned_dev_ptr(h_out, n * sizeof(uint16_t)) : nullptr;
    uint8_t* zst = h_status ? (uint8_t*)pinned_dev_ptr(h_status, n) : nullptr;
    // zero-copy over PCIe: the 16-lane group shape for latency-bound batches
    // (as tcpcsum_ipv4_batch_host on a pinned pool)
    tcpcsum::Tuning tu = c->tune;
    if (tu.shape < 0 && n < 65536u) tu.shape = 3;
    tcpcsum::launch_ipv4(nullptr, c->k_off, c->k_len, n, cap, ~0ull, foot, mode, zout ? zout : c->k_wout,
                         zst ? zst : c->k_wstat, nullptr, st, tu);
    rc = check_launch();
    if (rc) return rc;
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e);
    if (h_out && !zout) memcpy(h_out, c->h_wout, n * sizeof(uint16_t));
    if (h_status && !zst) memcpy(h_status, c->h_wstat, n);
    return TCPCSUM_OK;
}

int tcpcsum_ctx_register_host(tcpcsum_ctx_t* c, void* p, size_t bytes) {
    if (!c || !p || !bytes) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    const int rc = c->reg.lock_range((uintptr_t)p, bytes);
    if (rc == TCPCSUM_EHIP) g_last_hip_error.store(c->backend.last_error);
    return rc;
}

int tcpcsum_ctx_unregister_host(tcpcsum_ctx_t* c, void* p, size_t bytes) {
    if (!c) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    for (int i = 0; i < 2; ++i) (void)hipStreamSynchronize(c->st[i]);
    c->reg.release((uintptr_t)p, bytes);
    return TCPCSUM_OK;
}

int tcpcsum_ctx_registered(tcpcsum_ctx_t* c, uint64_t* ranges, uint64_t* bytes) {
    if (!c) return TCPCSUM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (ranges) *ranges = c->reg.owned_ranges();
    if (bytes) *bytes = c->reg.owned_bytes();
    return TCPCSUM_OK;
}

}  // extern "C"
