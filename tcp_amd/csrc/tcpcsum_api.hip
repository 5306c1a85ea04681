// tcpcsum_api.hip — the device half of the C ABI declared in include/tcpcsum.h.
//
// Argument checking, device checks, error mapping, the device batch entry
// points and the synthetic-workload / measurement helpers. The host-memory
// paths (tcpcsum_ctx_*, *_host) are in tcpcsum_host.hip. All checksum
// arithmetic on the batch paths runs in the gfx950 kernels of
// tcpcsum_kernels.hip; this file never computes a checksum itself.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <climits>

#include "tcpcsum.h"
#include "tcpcsum_internal.h"

#if TCPCSUM_MEASUREMENT_BUILD
#define TCPCSUM_PRODUCT_JSON false
#else
#define TCPCSUM_PRODUCT_JSON true
#endif

static_assert(sizeof(tcpcsum_desc_t) == 16, "descriptor is read as one 16-B load");
static_assert(sizeof(tcpcsum_txseg_t) == 48, "tx descriptor is read as three 16-B loads");
static_assert(sizeof(tcpcsum_ubatch_t) == 48 && sizeof(tcpcsum::UniformMultiEntry) == 48, "batch descriptor layout");

namespace {

// Diagnostics only (the hipError_t behind the last TCPCSUM_EHIP) and the
// per-device arch cache below; nothing that changes what a launch does.
std::atomic<int> g_last_hip_error{0};

constexpr int kMaxDevices = 64;
std::atomic<int> g_dev_ok[kMaxDevices];   // 0 unknown, 1 gfx950, -1 unusable

}  // namespace

namespace tcpcsum {

void note_hip_error(int e) { g_last_hip_error.store(e); }

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
            t->shape > 14 || (t->flags & ~8191) || (t->flags & 3) == 3 || (t->flags & 12) == 12)
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

}  // namespace tcpcsum

using tcpcsum::check_launch;
using tcpcsum::get_tuning;
using tcpcsum::hip_fail;
using tcpcsum::require_device;

extern "C" {

int tcpcsum_abi_version(void) { return TCPCSUM_ABI_VERSION; }

#define TCPCSUM_STR2(x) #x
#define TCPCSUM_STR(x) TCPCSUM_STR2(x)
const char* tcpcsum_build_info(void) {
    static const char info[] =
        "{\"abi\": " TCPCSUM_STR(TCPCSUM_ABI_VERSION) ", \"src_sha256\": \"" TCPCSUM_SRC_HASH
        "\", \"arch\": \"gfx950\", \"product\": " TCPCSUM_STR(TCPCSUM_PRODUCT_JSON)
        ", \"knobs\": {\"TCPCSUM_MEASUREMENT_BUILD\": " TCPCSUM_STR(TCPCSUM_MEASUREMENT_BUILD)
        ", \"TCPCSUM_TUNING_VARIANTS\": " TCPCSUM_STR(TCPCSUM_TUNING_VARIANTS)
        ", \"TCPCSUM_TX_KNOCKOUT\": " TCPCSUM_STR(TCPCSUM_TX_KNOCKOUT)
        ", \"TCPCSUM_WIRE_WAVES\": " TCPCSUM_STR(TCPCSUM_WIRE_WAVES)
        ", \"TCPCSUM_TX_WAVES\": " TCPCSUM_STR(TCPCSUM_TX_WAVES)
        ", \"TCPCSUM_LINE_CPOL\": " TCPCSUM_STR(TCPCSUM_LINE_CPOL)
        ", \"TCPCSUM_LOAD_CPOL\": " TCPCSUM_STR(TCPCSUM_LOAD_CPOL)
        ", \"TCPCSUM_XCD_REMAP\": " TCPCSUM_STR(TCPCSUM_XCD_REMAP)
        ", \"TCPCSUM_XCD_CHUNK\": " TCPCSUM_STR(TCPCSUM_XCD_CHUNK)
        ", \"TCPCSUM_UNIFORM_WPB\": " TCPCSUM_STR(TCPCSUM_UNIFORM_WPB)
        ", \"TCPCSUM_DESC_LB_WAVES\": " TCPCSUM_STR(TCPCSUM_DESC_LB_WAVES)
        ", \"TCPCSUM_SS_LOAD\": " TCPCSUM_STR(TCPCSUM_SS_LOAD)
        ", \"TCPCSUM_LB_VARIANT\": " TCPCSUM_STR(TCPCSUM_LB_VARIANT)
        ", \"TCPCSUM_LB_HEAD\": " TCPCSUM_STR(TCPCSUM_LB_HEAD)
        ", \"TCPCSUM_LB_HDR_X4\": " TCPCSUM_STR(TCPCSUM_LB_HDR_X4) "}"
        ", \"runtime_knobs\": [" TCPCSUM_RUNTIME_KNOBS_JSON "]}";
    return info;
}

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

int tcpcsum_batch_uniform_multi_dev(const tcpcsum_ubatch_t* b, uint32_t k, void* stream,
                                    const tcpcsum_tuning_t* tune) {
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    if (k == 0) return TCPCSUM_OK;
    if (!b) return TCPCSUM_EINVAL;
    for (uint32_t i = 0; i < k; ++i)
        if (b[i].n && (!b[i].d_base || !b[i].d_out || b[i].len > (uint32_t)INT_MAX)) return TCPCSUM_EINVAL;
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    for (uint32_t i = 0; i < k; i += TCPCSUM_MULTI_MAX) {
        tcpcsum::launch_uniform_multi(b + i, std::min<uint32_t>(TCPCSUM_MULTI_MAX, k - i), (hipStream_t)stream, tu);
        rc = check_launch();
        if (rc) return rc;
    }
    return TCPCSUM_OK;
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

int tcpcsum_ipv4_batch_ptrs_dev(void* const* d_pkt_ptrs, const uint32_t* d_lens, uint64_t n, uint32_t cap,
                                uint64_t bytes_hint, int mode, uint16_t* d_out, uint8_t* d_status, void* stream,
                                const tcpcsum_tuning_t* tune) {
    tcpcsum::Tuning tu;
    if (get_tuning(tune, &tu)) return TCPCSUM_EINVAL;
    if (n == 0) return TCPCSUM_OK;
    if (!d_pkt_ptrs || !d_lens || (mode & ~3) || (((uintptr_t)d_pkt_ptrs) & 7u) || (((uintptr_t)d_lens) & 3u))
        return TCPCSUM_EINVAL;
    if (cap > 65535u) cap = 65535u;
    int rc = require_device(nullptr, 0);
    if (rc) return rc;
    // addresses as offsets from 0, bounded per packet by d_lens
    tcpcsum::launch_ipv4(nullptr, (const uint64_t*)d_pkt_ptrs, d_lens, n, cap, ~0ull,
                         bytes_hint ? bytes_hint : n * (uint64_t)cap, mode, d_out, d_status, nullptr,
                         (hipStream_t)stream, tu);
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

}  // extern "C"
