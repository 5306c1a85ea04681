// copy_probe.hip — round 3: how fast can this chip move bytes HBM -> HBM (read + write) in the
// segment builder's access shape, i.e. what bounds tcpcsum_tx_build_dev (k_tx_build)?
// Copies 1M x 1456-B payloads (1.53 GB) into a second buffer, wave-contiguous 16-B loads
// (non-temporal) and 16-B stores, C chunks in flight per lane; one JSON line per variant
// (median / min ms of 7 x 10 launches after 3 warm-ups, GB/s counting read + write bytes).
//   store   default (write-back in L2), nt (streaming), wt (write-through, sc0 sc1)
//   shift   0: destination at the same offset; 44: destination 44 bytes further on (the
//           builder's payload position behind the 44-B header), every store still a whole
//           aligned 16-B chunk assembled from two source chunks (v_alignbyte), as k_tx_build does
//   grid    workgroups (0 = one tile per wave)
// Vector stores only.
//   hipcc -O3 --offload-arch=gfx950 -o tools/copy_probe tools/copy_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

template <class T>
using gptr = __attribute__((address_space(1))) T*;

__device__ __forceinline__ u32x4 ldnt(const uint8_t* p) { return __builtin_nontemporal_load((gptr<const u32x4>)p); }

// S: 0 default store, 1 nt store, 2 write-through (sc0 sc1). SH: destination byte shift (multiple of 4).
// dst chunk d (16-B aligned, d >= 1 when SH) takes source bytes [16d - SH, 16d - SH + 16).
template <int S, int SH, int C>
__global__ __launch_bounds__(256) void k_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                              uint64_t nchunks) {
    const uint64_t lane = threadIdx.x & 63, wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * 4u, per = 64u * C;
    constexpr uint32_t q = (SH & 15) / 4;             // dwords of shift inside a chunk
    constexpr uint64_t cs = (SH + 15) / 16;           // source chunk offset
    for (uint64_t t = wave * per; t < nchunks; t += nw * per) {
        u32x4 a[C], b[C];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint64_t c = t + (uint64_t)k * 64u + lane;
            const uint64_t s = c >= cs ? c - cs : 0;
            a[k] = ldnt(src + (c < nchunks ? s : 0) * 16u);
            if constexpr (SH % 16 != 0) b[k] = ldnt(src + (c < nchunks ? s + 1 : 0) * 16u);
        }
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint64_t c = t + (uint64_t)k * 64u + lane;
            if (c >= nchunks) continue;
            u32x4 v = a[k];
            if constexpr (SH % 16 != 0) {   // the 16 bytes starting 4q dwords from the end of a
                const uint32_t w[8] = {a[k].x, a[k].y, a[k].z, a[k].w, b[k].x, b[k].y, b[k].z, b[k].w};
                v = u32x4{w[4 - q], w[5 - q], w[6 - q], w[7 - q]};
            }
            uint8_t* p = dst + c * 16u;
            if constexpr (S == 0) *(gptr<u32x4>)p = v;
            else if constexpr (S == 1) __builtin_nontemporal_store(v, (gptr<u32x4>)p);
            else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 3" ::"v"(p), "v"(v) : "memory");
        }
    }
}

template <int S, int SH, int C>
static int run(const char* name, const uint8_t* src, uint8_t* dst, uint64_t nchunks, int blocks) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t waves = (nchunks + 64u * C - 1) / (64u * C);
    const int grid = blocks ? blocks : (int)((waves + 3) / 4);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_copy<S, SH, C>), dim3(grid), dim3(256), 0, 0, src, dst, nchunks);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < 10; ++k)
            hipLaunchKernelGGL((k_copy<S, SH, C>), dim3(grid), dim3(256), 0, 0, src, dst, nchunks);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t / 10);
    }
    std::sort(ms.begin(), ms.end());
    const double bytes = 2.0 * (double)nchunks * 16.0;
    std::printf("{\"variant\": \"%s\", \"C\": %d, \"grid\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f, "
                "\"GB/s_rw_median\": %.1f}\n",
                name, C, grid, ms[3], ms[0], bytes / (ms[3] * 1e-3) / 1e9);
    std::fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 0;
}

int main() {
    const uint64_t bytes = (uint64_t)(1u << 20) * 1456u, nchunks = bytes / 16;
    uint8_t *src, *dst;
    CK(hipMalloc(&src, bytes + 64));
    CK(hipMalloc(&dst, bytes + 64));
    CK(hipMemset(src, 0x5a, bytes + 64));
    for (int rep = 0; rep < 2; ++rep) {
        int rc = 0;
        for (int g : {0, 4096}) {
            rc |= run<0, 0, 4>("default_shift0", src, dst, nchunks, g);
            rc |= run<1, 0, 4>("nt_shift0", src, dst, nchunks, g);
            rc |= run<2, 0, 4>("wt_shift0", src, dst, nchunks, g);
            rc |= run<0, 0, 8>("default_shift0", src, dst, nchunks, g);
            rc |= run<1, 0, 8>("nt_shift0", src, dst, nchunks, g);
            rc |= run<0, 44, 4>("default_shift44", src, dst, nchunks, g);
            rc |= run<1, 44, 4>("nt_shift44", src, dst, nchunks, g);
            rc |= run<2, 44, 4>("wt_shift44", src, dst, nchunks, g);
        }
        if (rc) return 1;
    }
    return 0;
}
