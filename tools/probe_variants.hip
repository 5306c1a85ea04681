// probe_variants.hip — is there a faster way to stream HBM than the checksum
// kernels' access shape? Read-only kernels over a 2 x 2 GiB rotation (beyond
// the 256 MiB Infinity Cache), each summing what it reads (v_sad_u16, as the
// checksum does) into one u64 per workgroup:
//   wave    — the shipped shape: each load instruction reads 1 KiB contiguous
//             across the wave (16 B per lane), C in flight per lane, grid stride,
//             non-temporal (nt) or default policy
//   lane64  — each lane reads 64 contiguous bytes (4 x 16 B), C/4 such runs
//   glds    — global_load_lds_dwordx4 into LDS (no VGPR destination), C per
//             wave in flight, then ds_read_b128 and sum
// "_tile" variants launch one tile per wave (no grid-stride loop), as the
// shipped uniform kernel does for segments up to 1.5 KiB since round 2.
// Prints one JSON line per variant: GB/s (median of 5 x 10 launches).
//   hipcc -O3 --offload-arch=gfx950 -o tools/probe_variants tools/probe_variants.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

__device__ __forceinline__ uint32_t sad16(uint32_t d, uint32_t acc) { return __builtin_amdgcn_sad_u16(d, 0u, acc); }
__device__ __forceinline__ uint32_t sum4(u32x4 v, uint32_t a) { return sad16(v.w, sad16(v.z, sad16(v.y, sad16(v.x, a)))); }

template <int C, bool NT>
__global__ __launch_bounds__(256) void k_wave(const uint8_t* __restrict__ src, uint64_t nchunks, uint64_t* out) {
    const uint64_t lane = threadIdx.x & 63, wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * 4u, per = 64u * C;
    uint64_t acc = 0;
    for (uint64_t t = wave * per; t < nchunks; t += nw * per) {
        u32x4 v[C];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint64_t c = t + (uint64_t)k * 64u + lane;
            const u32x4* p = reinterpret_cast<const u32x4*>(src + (c < nchunks ? c : 0) * 16u);
            v[k] = NT ? __builtin_nontemporal_load(p) : *p;
        }
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < C; ++k) w = sum4(v[k], w);
        acc += w;
    }
    for (int s = 32; s >= 1; s >>= 1) acc += __shfl_xor(acc, s, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(out + (blockIdx.x & 8191u)), (unsigned long long)acc);
}

template <int C>
__global__ __launch_bounds__(256) void k_lane64(const uint8_t* __restrict__ src, uint64_t nchunks, uint64_t* out) {
    // a wave's tile: 64 lanes x C chunks, lane l owns chunks [l*C, l*C + C) of it
    const uint64_t lane = threadIdx.x & 63, wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * 4u, per = 64u * C;
    uint64_t acc = 0;
    for (uint64_t t = wave * per; t < nchunks; t += nw * per) {
        u32x4 v[C];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint64_t c = t + lane * C + k;
            v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + (c < nchunks ? c : 0) * 16u));
        }
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < C; ++k) w = sum4(v[k], w);
        acc += w;
    }
    for (int s = 32; s >= 1; s >>= 1) acc += __shfl_xor(acc, s, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(out + (blockIdx.x & 8191u)), (unsigned long long)acc);
}

template <int C>
__global__ __launch_bounds__(256) void k_glds(const uint8_t* __restrict__ src, uint64_t nchunks, uint64_t* out) {
    __shared__ u32x4 buf[4][C][64];
    const int wv = threadIdx.x >> 6;
    const uint64_t lane = threadIdx.x & 63, wave = blockIdx.x * 4u + wv;
    const uint64_t nw = (uint64_t)gridDim.x * 4u, per = 64u * C;
    uint64_t acc = 0;
    for (uint64_t t = wave * per; t < nchunks; t += nw * per) {
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint64_t c = t + (uint64_t)k * 64u + lane;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (c < nchunks ? c : 0) * 16u),
                                             (__attribute__((address_space(3))) void*)(&buf[wv][k][0]),
                                             16, 0, 2);
        }
        __builtin_amdgcn_s_waitcnt(0);   // vmcnt(0) lgkmcnt(0): the LDS writes landed
        __builtin_amdgcn_wave_barrier();
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < C; ++k) w = sum4(buf[wv][k][lane], w);
        __builtin_amdgcn_wave_barrier();
        acc += w;
    }
    for (int s = 32; s >= 1; s >>= 1) acc += __shfl_xor(acc, s, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(out + (blockIdx.x & 8191u)), (unsigned long long)acc);
}

typedef void (*kfn)(const uint8_t*, uint64_t, uint64_t*);

int main() {
    const uint64_t bytes = 2ull << 30, nch = bytes / 16;
    uint8_t* buf[2];
    uint64_t* out;
    for (int i = 0; i < 2; ++i) {
        CK(hipMalloc(&buf[i], bytes));
        CK(hipMemset(buf[i], 0x5a + i, bytes));
    }
    CK(hipMalloc(&out, 8192 * sizeof(uint64_t)));
    struct V { const char* name; kfn f; int blocks; };
    std::vector<V> vs = {
        {"wave_C16_nt_b512", k_wave<16, true>, 512},   {"wave_C16_nt_b1024", k_wave<16, true>, 1024},
        {"wave_C8_nt_b1024", k_wave<8, true>, 1024},   {"wave_C8_nt_b2048", k_wave<8, true>, 2048},
        {"wave_C24_nt_b512", k_wave<24, true>, 512},   {"wave_C16_def_b512", k_wave<16, false>, 512},
        {"lane64_C8_b1024", k_lane64<8>, 1024},       {"lane64_C16_b512", k_lane64<16>, 512},
        {"lane64_C4_b2048", k_lane64<4>, 2048},       {"glds_C8_b1024", k_glds<8>, 1024},
        {"glds_C16_b512", k_glds<16>, 512},           {"glds_C16_b1024", k_glds<16>, 1024},
        {"glds_C32_b512", k_glds<32>, 512},
        // one tile per wave (no grid-stride loop): 2 GiB / (1 KiB x C) waves
        {"wave_C4_nt_tile", k_wave<4, true>, 131072},  {"wave_C8_nt_tile", k_wave<8, true>, 65536},
        {"wave_C16_nt_tile", k_wave<16, true>, 32768}, {"wave_C24_nt_tile", k_wave<24, true>, 21846},
        {"glds_C8_tile", k_glds<8>, 65536},            {"glds_C16_tile", k_glds<16>, 32768},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {   // round 0 warms up every kernel
        for (const auto& v : vs) {
            std::vector<float> ms;
            for (int r = 0; r < 5; ++r) {
                CK(hipMemset(out, 0, 8192 * sizeof(uint64_t)));
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < 10; ++i)
                    hipLaunchKernelGGL(v.f, dim3(v.blocks), dim3(256), 0, 0, buf[i & 1], nch, out);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t = 0;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms.push_back(t / 10);
            }
            std::sort(ms.begin(), ms.end());
            const int slots = v.blocks < 8192 ? v.blocks : 8192;   // blocks fold onto 8192 partials
            std::vector<uint64_t> h(slots);
            CK(hipMemcpy(h.data(), out, slots * sizeof(uint64_t), hipMemcpyDeviceToHost));
            uint64_t s = 0;
            for (auto x : h) s += x;
            if (rep)
                std::printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GB/s\": %.1f, \"sum_per_launch\": %llu}\n", v.name,
                            ms[2], bytes / (ms[2] * 1e-3) / 1e9, (unsigned long long)(s / 10));
        }
    }
    return 0;
}
