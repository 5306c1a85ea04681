// tcpcsum_kernels.hip — gfx950 (MI355X / CDNA4) kernels for the TCP checksum
// hot path of uNetworking/tcp (context.c:104-145, called at context.c:208-209).
//
// Arithmetic contract, for every segment:
//   S   = sum_start + sum_{k < len} byte[k] * (k even ? 1 : 256)      (exact)
//   s1  = (S >> 16) + (S & 0xffff);  s2 = s1 + (s1 >> 16);  out = ~s2 & 0xffff
// The first line is csum_continue's loop (context.c:130-133) over native
// little-endian u16 words plus its odd-byte rule (context.c:134-138: a trailing
// byte sits at an even offset and is added as a low byte). The second line is
// its fold (context.c:140-144). S is never reduced early, so results are bit
// exact for every length, including sums >= 2^32 where the two-fold differs
// from a full RFC 1071 fold.
//
// How the bytes are read (all kernels): a segment is covered by the 16-byte
// aligned chunks that overlap it. Lanes of a "group" (G lanes per segment)
// load consecutive chunks with one 16-B non-temporal load each
// (global_load_dwordx4 nt), so every wave-instruction reads contiguous memory.
// Bytes outside the segment are masked in registers. Per chunk the sum of its
// four dwords' u16 halves is taken with v_sad_u16 (|a.lo-0| + |a.hi-0| + acc),
// one VALU op per dword. Word parity is absolute-address parity; for a segment
// starting at an odd address the relative even/odd roles swap, which is exact
// with E = W - 256*O (W: sum of absolute-aligned words, O: sum of odd-address
// bytes): S = sum_start + O + 256*E.
//
// Groups are reduced with DPP row ops (<=16 lanes) and ds_swizzle / bpermute
// (32/64 lanes). No LDS staging and no MFMA: this is an HBM-bound integer
// reduction (~1 VALU op per 4 bytes) and each byte is read exactly once.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "tcpcsum.h"
#include "tcpcsum_internal.h"

// The compile-time knobs (TCPCSUM_TUNING_VARIANTS, TCPCSUM_TX_KNOCKOUT,
// TCPCSUM_WIRE_WAVES, TCPCSUM_TX_WAVES) live in tcpcsum_internal.h: a product
// build refuses any of them set, tcpcsum_build_info() reports them.

namespace tcpcsum {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));   // 4-B aligned dwordx4

enum : int { M16 = 0, M4 = 1, M1 = 2 };

// Every pointer the kernels dereference is a global-memory address (HBM, or
// page-locked host memory mapped into the device's address space), never LDS
// or scratch: loads and stores go through address space 1, so the compiler
// emits global_* rather than flat_* instructions. A flat load counts against
// lgkmcnt as well as vmcnt, so the s_waitcnt lgkmcnt(0) of the next
// ds_bpermute / LDS access would wait for it too and serialise the loads.
template <class T>
using gptr = __attribute__((address_space(1))) T*;

template <class T>
__device__ __forceinline__ T ldg(const void* p) {
    return *(gptr<const T>)(p);
}
template <class T>
__device__ __forceinline__ void stg(void* p, T v) {
    *(gptr<T>)(p) = v;
}

__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
    return __builtin_nontemporal_load((gptr<const u32x4>)(p));
}

// Zero-filled device memory: lanes with nothing to load read it instead of
// predicating the load. A predicated load in a tile becomes a branch whose
// join point drains vmcnt, which serialises the tile's loads; an address
// select keeps every load unconditional and in flight together.
__device__ __attribute__((aligned(64))) uint8_t g_zero[64];

__device__ __forceinline__ const uint8_t* zsel(bool use, const uint8_t* p) { return use ? p : g_zero; }

// context.c:140-144, on the exact sum.
__device__ __forceinline__ uint16_t fold_ref(uint64_t S) {
    uint64_t s = (S >> 16) + (S & 0xffffu);
    s = s + (s >> 16);
    return (uint16_t)(~s & 0xffffu);
}

__device__ __forceinline__ uint32_t sad16(uint32_t d, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(d, 0u, acc);   // lo16(d) + hi16(d) + acc
}
__device__ __forceinline__ uint32_t sad8(uint32_t d, uint32_t acc) {
    return __builtin_amdgcn_sad_u8(d, 0u, acc);    // sum of the 4 bytes + acc
}

// ---------------------------------------------------------------- reductions
// Sum over the G lanes of an aligned lane group; result valid in every lane
// of the group. DPP for 2..16 lanes, swizzle/bpermute above.
template <int G>
__device__ __forceinline__ uint32_t group_sum32(uint32_t x) {
    if constexpr (G >= 2)  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
    if constexpr (G >= 4)  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
    if constexpr (G >= 8)  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false); // row_half_mirror
    if constexpr (G >= 16) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false); // row_mirror
    if constexpr (G >= 32) x += (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);                    // xor 16 within 32
    if constexpr (G >= 64) x += (uint32_t)__shfl_xor((int)x, 32, 64);
    return x;
}

template <int G>
__device__ __forceinline__ uint64_t group_sum64(uint64_t x) {
#pragma unroll
    for (int s = G / 2; s >= 1; s >>= 1) x += __shfl_xor(x, s, 64);
    return x;
}

// ---------------------------------------------------------------- chunk sums
// One 16-B chunk whose first byte sits at segment-relative offset rel
// (negative for the leading partial chunk; two's complement in a u32).
// M16: chunk entirely inside the segment (masking done by the load predicate).
// M4 : segment start and length are multiples of 4 — dword-granular mask.
template <int MODE>
__device__ __forceinline__ uint32_t chunk_w(u32x4 v, uint32_t rel, uint32_t len) {
    if constexpr (MODE == M16) {
        uint32_t w = sad16(v.x, 0u);
        w = sad16(v.y, w);
        w = sad16(v.z, w);
        return sad16(v.w, w);
    } else {
        uint32_t w = sad16((rel + 0u) < len ? v.x : 0u, 0u);
        w = sad16((rel + 4u) < len ? v.y : 0u, w);
        w = sad16((rel + 8u) < len ? v.z : 0u, w);
        return sad16((rel + 12u) < len ? v.w : 0u, w);
    }
}

__device__ __forceinline__ uint64_t bytemask64(int64_t nbytes) {   // low nbytes bytes set, nbytes in [0,8]
    return nbytes >= 8 ? ~0ull : ((1ull << (8 * nbytes)) - 1ull);
}

// Byte-granular: valid bytes of the chunk are [lo, hi) with lo = -rel and
// hi = len - rel clamped to [0,16]. Adds the aligned-word sum to W and the
// odd-address byte sum to O (O only when want_odd).
__device__ __forceinline__ void chunk_wo_bytes(u32x4 v, int64_t rel, int64_t len, bool want_odd,
                                               uint32_t& W, uint32_t& O) {
    int64_t lo = -rel;       lo = lo < 0 ? 0 : (lo > 16 ? 16 : lo);
    int64_t hi = len - rel;  hi = hi < 0 ? 0 : (hi > 16 ? 16 : hi);
    int64_t lo0 = lo < 8 ? lo : 8, hi0 = hi < 8 ? hi : 8;
    int64_t lo1 = lo > 8 ? lo - 8 : 0, hi1 = hi > 8 ? hi - 8 : 0;
    const uint64_t m0 = bytemask64(hi0) & ~bytemask64(lo0);
    const uint64_t m1 = bytemask64(hi1) & ~bytemask64(lo1);
    const uint32_t d0 = v.x & (uint32_t)m0, d1 = v.y & (uint32_t)(m0 >> 32);
    const uint32_t d2 = v.z & (uint32_t)m1, d3 = v.w & (uint32_t)(m1 >> 32);
    W = sad16(d0, W); W = sad16(d1, W); W = sad16(d2, W); W = sad16(d3, W);
    if (want_odd) {
        O = sad8(d0 & 0xff00ff00u, O); O = sad8(d1 & 0xff00ff00u, O);
        O = sad8(d2 & 0xff00ff00u, O); O = sad8(d3 & 0xff00ff00u, O);
    }
}

__device__ __forceinline__ uint64_t combine(uint64_t start, uint64_t W, uint64_t O, bool odd_start) {
    // even start: relative parity == absolute parity -> S = start + W.
    // odd start : relative even bytes are the absolute odd ones.
    return odd_start ? start + O + 256ull * (W - 256ull * O) : start + W;
}

// ---------------------------------------------------------------- XCD order
// Workgroups are dispatched to the 8 XCDs round-robin (workgroup b on XCD b % 8). When a
// launch gives every unit of work (a wave tile, or a segment per workgroup) its own
// workgroup slot — nb >= units_per_block-rounded need — and its grid is a whole number
// of XCD rounds, workgroup b takes block-run (b % 8) * nb/8 + b / 8 instead of b: each
// XCD then sweeps one contiguous eighth of the batch through its own L2 and the HBM
// channels see eight long streams instead of an interleave of small tiles
// (TCPCSUM_XCD_REMAP; measured per kernel). Grid-stride launches keep
// block order (remapped, the 64-B config's 1024 looping workgroups ran 14.8 instead of
// 12.6 us, profiles/r05_xcd_remap_ab.jsonl).
__device__ __forceinline__ uint64_t xcd_block(uint64_t blocks_needed) {
    const uint32_t nb = gridDim.x, bx = blockIdx.x;
    const bool remap = TCPCSUM_XCD_REMAP && nb % 8u == 0u && (uint64_t)nb >= blocks_needed;
#if TCPCSUM_XCD_CHUNK > 0   // measurement builds: XCDs take runs of CHUNK blocks in turn
    if (remap && (nb / 8u) % TCPCSUM_XCD_CHUNK == 0u) {
        const uint64_t j = bx / 8u;
        return ((j / TCPCSUM_XCD_CHUNK) * 8u + bx % 8u) * TCPCSUM_XCD_CHUNK + j % TCPCSUM_XCD_CHUNK;
    }
#endif
    return remap ? (uint64_t)(bx % 8u) * (nb / 8u) + bx / 8u : (uint64_t)bx;
}

// ---------------------------------------------------------------- uniform
// Segment i at base + i*stride, all of length len; n segments.
// G lanes per segment, C chunk loads per lane per segment (G*C >= chunks a
// segment can touch), U segments per group in flight per tile.
// A wave tile = (64/G)*U consecutive segments; load instruction (u, k) of the
// wave reads chunk k*G+gl of segments tile+u*(64/G)+q — consecutive segments
// across groups, i.e. one contiguous run of memory.
template <bool NT>
__device__ __forceinline__ u32x4 ldq(const uint8_t* p) {
    if constexpr (NT) return ld16(p);
    else return ldg<u32x4>(p);
}

template <int G, int C, int U, int MODE, bool NT>
struct UniformTile {
    static constexpr int GPW = 64 / G;
    static constexpr int SPT = GPW * U;
    // start values: one dword per group lane 0 (0, 1: non-temporal), or one coalesced dword per
    // lane for the whole tile, handed to each group by ds_bpermute (2, 3: non-temporal)
    static constexpr int SSL = (TCPCSUM_SS_LOAD >= 2 && SPT <= 64) ? TCPCSUM_SS_LOAD : (TCPCSUM_SS_LOAD & 1);
    u32x4 v[U][C];
    uint32_t st[U], mm[U];
    uint32_t sv;

    // issue every load of tile t (chunks, and the start values for lane 0 of each group)
    __device__ __forceinline__ void load(uint64_t t, const uint8_t* __restrict__ base, uint64_t stride,
                                         uint32_t len, const uint32_t* __restrict__ ss, uint32_t ss_scalar,
                                         uint64_t n, int q, int gl) {
        if constexpr (SSL >= 2) {
            const uint64_t sl = t * SPT + (uint64_t)(q * G + gl);
            const bool in = ss && (q * G + gl) < SPT && sl < n;
            if constexpr (SSL == 3) sv = in ? __builtin_nontemporal_load((gptr<const uint32_t>)(ss + sl)) : ss_scalar;
            else sv = in ? ss[sl] : ss_scalar;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t seg = t * SPT + (uint64_t)(u * GPW + q);
            const bool live = seg < n;
            const uint8_t* p = base + seg * stride;
            const uint32_t m = (uint32_t)((uintptr_t)p & 15u);
            const uint8_t* a0 = p - m;
            const uint32_t nch = (m + len + 15u) >> 4;
            mm[u] = m;
            if constexpr (SSL == 1)
                st[u] = (live && gl == 0) ? (ss ? __builtin_nontemporal_load((gptr<const uint32_t>)(ss + seg)) : ss_scalar) : 0u;
            else if constexpr (SSL == 0)
                st[u] = (live && gl == 0) ? (ss ? ss[seg] : ss_scalar) : 0u;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = (uint32_t)(k * G + gl);
#if TCPCSUM_LOAD_CPOL >= 0   // measurement builds: buffer loads with chosen cache-policy bits
                const uint8_t* b0 = reinterpret_cast<const uint8_t*>((uintptr_t)base & ~(uintptr_t)15u);
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(b0), 0, -1, 0x00020000);
                v[u][k] = (live && idx < nch)
                              ? __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(uint32_t)(a0 - b0) + (int)(idx * 16u), 0,
                                                                       TCPCSUM_LOAD_CPOL)
                              : u32x4{0u, 0u, 0u, 0u};
#else
                v[u][k] = (live && idx < nch) ? ldq<NT>(a0 + (uint64_t)idx * 16u) : u32x4{0u, 0u, 0u, 0u};
#endif
            }
        }
    }

    // sum, reduce over each group, fold, store
    __device__ __forceinline__ void finish(uint64_t t, const uint8_t* __restrict__ base, uint64_t stride,
                                           uint32_t len, uint16_t* __restrict__ out, uint64_t n, int q,
                                           int gl) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t seg = t * SPT + (uint64_t)(u * GPW + q);
            uint32_t w = 0, o = 0;
            bool odd = false;
            if constexpr (MODE == M1) odd = ((uintptr_t)(base + seg * stride)) & 1u;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t rel = (uint32_t)((k * G + gl) * 16) - mm[u];
                if constexpr (MODE == M1)
                    chunk_wo_bytes(v[u][k], (int64_t)(int32_t)rel, (int64_t)len, odd, w, o);
                else
                    w += chunk_w<MODE>(v[u][k], rel, len);
            }
            w = group_sum32<G>(w);
            if constexpr (MODE == M1) o = group_sum32<G>(o);
            uint32_t s0;
            if constexpr (SSL >= 2) s0 = (uint32_t)__shfl((int)sv, u * GPW + q, 64);
            else s0 = st[u];
            if (gl == 0 && seg < n) out[seg] = fold_ref(combine(s0, w, o, odd));
        }
    }
};

// PIPE: software-pipelined over the wave's tiles — the loads of tile t+nwaves
// are in flight while tile t is summed and stored (two register tiles).
template <int G, int C, int U, int MODE, bool PIPE, bool NT>
__global__ __launch_bounds__(256) void k_uniform(const uint8_t* __restrict__ base, uint64_t stride,
                                                 uint32_t len, const uint32_t* __restrict__ ss,
                                                 uint32_t ss_scalar, uint16_t* __restrict__ out,
                                                 uint64_t n, int blocked) {
    using Tile = UniformTile<G, C, U, MODE, NT>;
    constexpr uint32_t WPB = TCPCSUM_UNIFORM_WPB;   // waves per workgroup
    const int lane = threadIdx.x & 63;
    const int q = lane / G, gl = lane % G;
    const uint64_t nwaves = (uint64_t)gridDim.x * WPB;
    const uint64_t ntiles = (n + Tile::SPT - 1) / Tile::SPT;
    // tiles XCD by XCD (xcd_block): 1M x 1500 B 0.34 / 0.38 % faster at eight segments in
    // flight, HBM bytes unchanged (profiles/r05_xcd_remap_ab.jsonl); with it smaller tiles
    // win (plan_uniform)
    const uint64_t wave = xcd_block((ntiles + WPB - 1) / WPB) * WPB + (threadIdx.x >> 6);
    uint64_t t = wave;
    if constexpr (!PIPE) {
        Tile a;
        if (blocked) {   // each wave a contiguous run of tiles instead of a grid stride
            const uint64_t per = (ntiles + nwaves - 1) / nwaves;
            const uint64_t t1 = (wave + 1) * per < ntiles ? (wave + 1) * per : ntiles;
            for (t = wave * per; t < t1; ++t) {
                a.load(t, base, stride, len, ss, ss_scalar, n, q, gl);
                a.finish(t, base, stride, len, out, n, q, gl);
            }
            return;
        }
        for (; t < ntiles; t += nwaves) {
            a.load(t, base, stride, len, ss, ss_scalar, n, q, gl);
            a.finish(t, base, stride, len, out, n, q, gl);
        }
    } else {
        Tile a, b;
        if (t < ntiles) a.load(t, base, stride, len, ss, ss_scalar, n, q, gl);
        while (t < ntiles) {
            const uint64_t t2 = t + nwaves;
            if (t2 < ntiles) b.load(t2, base, stride, len, ss, ss_scalar, n, q, gl);
            a.finish(t, base, stride, len, out, n, q, gl);
            if (t2 >= ntiles) break;
            const uint64_t t3 = t2 + nwaves;
            if (t3 < ntiles) a.load(t3, base, stride, len, ss, ss_scalar, n, q, gl);
            b.finish(t2, base, stride, len, out, n, q, gl);
            t = t3;
        }
    }
}

// Several independent uniform batches in one launch (tcpcsum_batch_uniform_multi_dev):
// batch b is grid row blockIdx.y, so the batch index is a scalar from the
// dispatcher — no search — and its descriptor is read straight out of the
// kernel-argument segment with scalar loads. A 64 MiB batch of 64-B segments
// streams in ~8.4 us at peak; launched alone it takes ~13 us, the rest being
// the grid's ramp and drain, which one launch over K batches
// pays once. Rows are dispatched in order, so batch b+1's first waves fill the
// CUs batch b's last waves leave.
template <int G, int C, int U, int MODE>
__global__ __launch_bounds__(256) void k_uniform_multi(UniformMultiArgs args) {
    using Tile = UniformTile<G, C, U, MODE, true>;
    const __attribute__((address_space(4))) UniformMultiArgs* A =
        (const __attribute__((address_space(4))) UniformMultiArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    const __attribute__((address_space(4))) UniformMultiEntry& e = A->e[blockIdx.y];
    const uint8_t* base = e.base;
    const uint64_t stride = e.stride, n = e.n;
    const uint32_t len = e.len;
    const int lane = threadIdx.x & 63;
    const int q = lane / G, gl = lane % G;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t ntiles = (n + Tile::SPT - 1) / Tile::SPT;
    // XCD order within the row (a row of nb % 8 == 0 workgroups starts on XCD 0)
    for (uint64_t t = xcd_block((ntiles + 3) / 4) * 4u + (threadIdx.x >> 6); t < ntiles; t += nwaves) {
        Tile a;
        a.load(t, base, stride, len, e.ss, e.ss0, n, q, gl);
        a.finish(t, base, stride, len, e.out, n, q, gl);
    }
}

// Long segments (more than 512 chunks): one wave per segment, C chunk loads
// per lane per round (C KiB per wave-round), u32 lane partials flushed to u64
// every round so any length <= INT32_MAX is exact. The wave's work is the flat
// sequence of (segment, round) items; with PIPE the loads of item j+1 are in
// flight while item j is summed, across segment boundaries too.
template <int C, int MODE, bool PIPE, bool NT>
__global__ __launch_bounds__(256) void k_uniform_long(const uint8_t* __restrict__ base, uint64_t stride,
                                                      uint32_t len, uint32_t rounds,
                                                      const uint32_t* __restrict__ ss, uint32_t ss_scalar,
                                                      uint16_t* __restrict__ out, uint64_t n) {
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    // block order: XCD order measured no better for one segment per wave (byte-granular
    // 12301 / 20001 B, profiles/r05_xcd_kernels_ab.jsonl); the 64 KiB config's grid loops
    uint64_t seg = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (seg >= n) return;
    uint32_t r = 0;
    uint64_t W = 0, O = 0;
    u32x4 va[C], vb[C];
    auto load = [&](u32x4 (&v)[C], uint64_t sg, uint32_t rr) {
        const uint8_t* p = base + sg * stride;
        const uint32_t m = (uint32_t)((uintptr_t)p & 15u);
        const uint8_t* a0 = p - m;
        const uint32_t nch = (uint32_t)(((uint64_t)m + len + 15u) >> 4);
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint32_t idx = rr * (64u * C) + (uint32_t)(k * 64 + lane);
            v[k] = idx < nch ? ldq<NT>(a0 + (uint64_t)idx * 16u) : u32x4{0u, 0u, 0u, 0u};
        }
    };
    // sum item (sg, rr); on its last round reduce, fold and store
    auto consume = [&](const u32x4 (&v)[C], uint64_t sg, uint32_t rr) {
        const uint8_t* p = base + sg * stride;
        const uint32_t m = (uint32_t)((uintptr_t)p & 15u);
        const bool odd = (MODE == M1) && ((uintptr_t)p & 1u);
        uint32_t w = 0, o = 0;
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint32_t idx = rr * (64u * C) + (uint32_t)(k * 64 + lane);
            if constexpr (MODE == M1)
                chunk_wo_bytes(v[k], (int64_t)idx * 16 - (int64_t)m, (int64_t)len, odd, w, o);
            else
                w += chunk_w<MODE>(v[k], idx * 16u - m, len);
        }
        W += w;
        O += o;
        if (rr + 1 == rounds) {
            const uint64_t Wt = group_sum64<64>(W);
            const uint64_t Ot = (MODE == M1) ? group_sum64<64>(O) : 0;
            if (lane == 0) out[sg] = fold_ref(combine(ss ? ss[sg] : ss_scalar, Wt, Ot, odd));
            W = 0;
            O = 0;
        }
    };
    auto next = [&](uint64_t& sg, uint32_t& rr) {
        if (++rr == rounds) { rr = 0; sg += nwaves; }
    };
    if constexpr (!PIPE) {
        for (; seg < n; next(seg, r)) {
            load(va, seg, r);
            consume(va, seg, r);
        }
    } else {
        uint64_t s1 = seg;
        uint32_t r1 = r;
        load(va, seg, r);
        while (true) {
            next(s1, r1);
            if (s1 < n) load(vb, s1, r1);
            consume(va, seg, r);
            if (s1 >= n) break;
            seg = s1; r = r1;
            next(s1, r1);
            if (s1 < n) load(va, s1, r1);
            consume(vb, seg, r);
            if (s1 >= n) break;
            seg = s1; r = r1;
        }
    }
}

// Split segments (long segments, shape 13): one workgroup of four waves per
// segment, one segment per workgroup (grid-stride only past 2^24 segments).
// Round r, load k of thread t reads chunk r*256*C + k*256 + t, so each wave
// instruction is one contiguous 1 KiB and the workgroup's instruction 4 KiB;
// all C loads of a round are unconditional (zsel) and in flight together.
// Lane partials are u32 per round (C*8 words of <= 0xffff), flushed to u64;
// the four wave totals meet in LDS.
template <int C, int MODE>
__global__ __launch_bounds__(256) void k_uniform_split(const uint8_t* __restrict__ base, uint64_t stride,
                                                       uint32_t len, uint32_t rounds,
                                                       const uint32_t* __restrict__ ss, uint32_t ss_scalar,
                                                       uint16_t* __restrict__ out, uint64_t n) {
    __shared__ uint64_t part[4][2];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // block order: XCD order measured 3.8 % slower at 12300 B, even at 8192 / 9000 B
    // (profiles/r05_xcd_kernels_ab.jsonl)
    for (uint64_t seg = blockIdx.x; seg < n; seg += gridDim.x) {
        const uint8_t* p = base + seg * stride;
        const uint32_t m = (uint32_t)((uintptr_t)p & 15u);
        const uint8_t* a0 = p - m;
        const uint32_t nch = (uint32_t)(((uint64_t)m + len + 15u) >> 4);
        const bool odd = (MODE == M1) && ((uintptr_t)p & 1u);
        uint64_t W = 0, O = 0;
        for (uint32_t r = 0; r < rounds; ++r) {
            u32x4 v[C];
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = r * (256u * C) + (uint32_t)(k * 256 + tid);
                v[k] = ld16(zsel(idx < nch, a0 + (uint64_t)idx * 16u));
            }
            uint32_t w = 0, o = 0;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = r * (256u * C) + (uint32_t)(k * 256 + tid);
                if constexpr (MODE == M1)
                    chunk_wo_bytes(v[k], (int64_t)idx * 16 - (int64_t)m, (int64_t)len, odd, w, o);
                else
                    w += chunk_w<MODE>(v[k], idx * 16u - m, len);
            }
            W += w;
            O += o;
        }
        W = group_sum64<64>(W);
        if constexpr (MODE == M1) O = group_sum64<64>(O);
        if (lane == 0) {
            part[wv][0] = W;
            part[wv][1] = O;
        }
        __syncthreads();
        if (tid == 0) {
            const uint64_t Wt = part[0][0] + part[1][0] + part[2][0] + part[3][0];
            const uint64_t Ot = part[0][1] + part[1][1] + part[2][1] + part[3][1];
            out[seg] = fold_ref(combine(ss ? ss[seg] : ss_scalar, Wt, Ot, odd));
        }
        __syncthreads();
    }
}

// One workgroup of WPB waves per segment, the headline's tile plan carried to long
// segments (shape 14): each wave reads one contiguous tile of C KiB per round — wave v,
// load k, lane l reads chunk r*WPB*64*C + v*64*C + k*64 + l — so at 64 KiB with (16, 4)
// every wave holds exactly one 4 KiB tile and the workgroup the whole segment in one
// round. Segments are taken XCD by XCD (xcd_block), one per workgroup, so each XCD
// sweeps one contiguous eighth of the batch. All C loads of a round are unconditional
// (zsel) and in flight together; u32 lane partials per round (C*8 words of <= 0xffff)
// flushed to u64; the WPB wave totals meet in LDS. Exact for any length <= INT32_MAX.
template <int WPB, int C, int MODE>
__global__ __launch_bounds__(WPB * 64) void k_uniform_wg(const uint8_t* __restrict__ base, uint64_t stride,
                                                         uint32_t len, uint32_t rounds,
                                                         const uint32_t* __restrict__ ss, uint32_t ss_scalar,
                                                         uint16_t* __restrict__ out, uint64_t n) {
    static_assert(MODE != M1, "byte-granular segments keep one wave per segment");
    __shared__ uint64_t part[WPB];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t first = xcd_block(n);
    for (uint64_t seg = first; seg < n; seg += gridDim.x) {
        const uint8_t* p = base + seg * stride;
        const uint32_t m = (uint32_t)((uintptr_t)p & 15u);
        const uint8_t* a0 = p - m;
        const uint32_t nch = (uint32_t)(((uint64_t)m + len + 15u) >> 4);
        uint64_t W = 0;
        for (uint32_t r = 0; r < rounds; ++r) {
            u32x4 v[C];
            const uint32_t c0 = r * (uint32_t)(WPB * 64 * C) + (uint32_t)(wv * 64 * C + lane);
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = c0 + (uint32_t)(k * 64);
                v[k] = ld16(zsel(idx < nch, a0 + (uint64_t)idx * 16u));
            }
            uint32_t w = 0;
#pragma unroll
            for (int k = 0; k < C; ++k) w += chunk_w<MODE>(v[k], (c0 + (uint32_t)(k * 64)) * 16u - m, len);
            W += w;
        }
        W = group_sum64<64>(W);
        if (lane == 0) part[wv] = W;
        __syncthreads();
        if (tid == 0) {
            uint64_t Wt = 0;
#pragma unroll
            for (int i = 0; i < WPB; ++i) Wt += part[i];
            out[seg] = fold_ref((ss ? ss[seg] : ss_scalar) + Wt);
        }
        if (seg + gridDim.x < n) __syncthreads();
    }
}

// Flat tiles (segments of >= 1 KiB, 4-byte aligned): a wave takes SPT
// consecutive segments and reads their byte span as one contiguous stream —
// lane l loads chunk c0 + 64k + l, so every load instruction is one contiguous
// 1 KiB (the read probe's access shape). Instruction k covers at most two
// segments (stride >= 1 KiB): the lanes split its dwords into the first /
// second segment, two wave reductions give their sums, and lane j of the wave
// accumulates the sum of the tile's segment j; at the end lane j folds and
// stores segment j (coalesced start-value loads and result stores).
__device__ __forceinline__ uint32_t wave_sum32(uint32_t x) {
    x = group_sum32<16>(x);   // every lane holds its row's sum
    return __builtin_amdgcn_readlane(x, 0) + __builtin_amdgcn_readlane(x, 16) + __builtin_amdgcn_readlane(x, 32) +
           __builtin_amdgcn_readlane(x, 48);
}

template <int C>
__global__ __launch_bounds__(256) void k_flat(const uint8_t* __restrict__ base, uint32_t stride, uint32_t len,
                                              const uint32_t* __restrict__ ss, uint32_t ss_scalar,
                                              uint16_t* __restrict__ out, uint64_t n, uint32_t spt) {
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t ntiles = (n + spt - 1) / spt;
    const uint32_t bm = (uint32_t)((uintptr_t)base & 15u);
    const uint8_t* b0 = base - bm;   // 16-B aligned
    for (uint64_t t = xcd_block((ntiles + 3) / 4) * 4u + (threadIdx.x >> 6); t < ntiles; t += nwaves) {
        const uint64_t s_first = t * spt;
        const uint32_t nseg = (uint32_t)((n - s_first) < spt ? (n - s_first) : spt);
        const uint64_t tbase = s_first * (uint64_t)stride + bm;        // tile's first byte, from b0
        const uint64_t tend = tbase + (uint64_t)(nseg - 1) * stride + len;
        const uint64_t c0 = tbase >> 4, c1 = (tend + 15) >> 4;
        // start value for the segment this lane will own
        const uint32_t st = lane < (int)nseg ? (ss ? ss[s_first + lane] : ss_scalar) : 0u;
        u32x4 v[C];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint64_t ci = c0 + (uint64_t)(k * 64 + lane);
            v[k] = ci < c1 ? ld16(b0 + ci * 16u) : u32x4{0u, 0u, 0u, 0u};
        }
        uint32_t acc = 0;
        const int32_t x0 = (int32_t)((int64_t)(c0 * 16) - (int64_t)tbase);   // in (-16, 0]
        int32_t ja = x0 < 0 ? -1 : 0;   // tile segment holding instruction k's first dword
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const int32_t xk = x0 + k * 1024;
            if (xk >= (ja + 1) * (int32_t)stride) ++ja;   // wave-uniform; at most one step (stride >= 1 KiB)
            const int32_t bnd = (ja + 1) * (int32_t)stride;
            const int32_t x = xk + lane * 16;
            const uint32_t d[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
            uint32_t a = 0, b = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int32_t xd = x + 4 * j;
                const bool in_a = xd < bnd;
                const int32_t js = in_a ? ja : ja + 1;
                const int32_t r = xd - js * (int32_t)stride;
                const bool valid = js >= 0 && js < (int32_t)nseg && r >= 0 && r < (int32_t)len;
                const uint32_t w = valid ? d[j] : 0u;
                if (in_a) a = sad16(w, a); else b = sad16(w, b);
            }
            const uint32_t sa = wave_sum32(a), sb = wave_sum32(b);
            acc += lane == ja ? sa : 0u;
            acc += lane == ja + 1 ? sb : 0u;
        }
        if (lane < (int)nseg) out[s_first + lane] = fold_ref((uint64_t)st + acc);
    }
}

// ---------------------------------------------------------------- ragged
// Sum of one round of C chunks already in registers (chunk r + k*G + gl).
template <int G, int C>
__device__ __forceinline__ void round_sum(const u32x4 (&v)[C], uint32_t r, uint32_t m, uint32_t len, bool a4,
                                          bool odd, int gl, uint32_t& w, uint32_t& o) {
    if (a4) {
#pragma unroll
        for (int k = 0; k < C; ++k) w += chunk_w<M4>(v[k], (r + (uint32_t)(k * G + gl)) * 16u - m, len);
    } else {
#pragma unroll
        for (int k = 0; k < C; ++k)
            chunk_wo_bytes(v[k], (int64_t)(r + (uint32_t)(k * G + gl)) * 16 - (int64_t)m, (int64_t)len, odd, w, o);
    }
}

// Ragged descriptors in tiles of U segments per lane group: all descriptor
// loads of the tile, then the first round of chunk loads of all U segments,
// then the sums (longer segments take further rounds).
template <int G, int C, int U>
__global__ __launch_bounds__(256) void k_desc(const uint8_t* __restrict__ base,
                                              const tcpcsum_desc_t* __restrict__ desc, uint64_t n,
                                              uint16_t* __restrict__ out) {
    constexpr int GPW = 64 / G;
    constexpr int SPT = GPW * U;
    const int lane = threadIdx.x & 63;
    const int q = lane / G, gl = lane % G;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t ntiles = (n + SPT - 1) / SPT;
    // block order: XCD order measured 0.7-2 % slower on ragged batches in two runs
    // (profiles/r05_xcd_kernels_ab.jsonl)
    uint64_t t = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    // one 16-B load per descriptor; slots past n read zeros (len 0)
    auto load_desc = [&](uint64_t tile, u32x4 (&dst)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t seg = tile * SPT + (uint64_t)(u * GPW + q);
            dst[u] = ldg<u32x4>(zsel(seg < n, reinterpret_cast<const uint8_t*>(desc + seg)));
        }
    };
    u32x4 dn[U];
    load_desc(t, dn);
    for (; t < ntiles; t += nwaves) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = dn[u];
        u32x4 v[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint8_t* p = base + ((uint64_t)d[u].x | ((uint64_t)d[u].y << 32));
            const uint32_t m = (uint32_t)((uintptr_t)p & 15u);
            const uint32_t nch = (uint32_t)(((uint64_t)m + d[u].z + 15u) >> 4);   // 0 for dead slots (len 0)
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = (uint32_t)(k * G + gl);
                v[u][k] = ld16(zsel(idx < nch, p - m + (uint64_t)idx * 16u));
            }
        }
        // the next tile's descriptors, in flight while this tile is summed
        load_desc(t + nwaves, dn);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t seg = t * SPT + (uint64_t)(u * GPW + q);
            if (seg >= n) continue;   // group-uniform
            const uint8_t* p = base + ((uint64_t)d[u].x | ((uint64_t)d[u].y << 32));
            const uint32_t len = d[u].z;
            const uint32_t m = (uint32_t)((uintptr_t)p & 15u);
            const uint32_t nch = (uint32_t)(((uint64_t)m + len + 15u) >> 4);
            const bool a4 = (((uintptr_t)p | len) & 3u) == 0;
            const bool odd = ((uintptr_t)p & 1u) != 0;
            uint32_t w = 0, o = 0;
            round_sum<G, C>(v[u], 0u, m, len, a4, odd, gl, w, o);
            uint64_t W = w, O = o;
            for (uint32_t r = (uint32_t)(G * C); r < nch; r += (uint32_t)(G * C)) {
                u32x4 x[C];
#pragma unroll
                for (int k = 0; k < C; ++k) {
                    const uint32_t idx = r + (uint32_t)(k * G + gl);
                    x[k] = idx < nch ? ld16(p - m + (uint64_t)idx * 16u) : u32x4{0u, 0u, 0u, 0u};
                }
                uint32_t w2 = 0, o2 = 0;
                round_sum<G, C>(x, r, m, len, a4, odd, gl, w2, o2);
                W += w2;
                O += o2;
            }
            W = group_sum64<G>(W);
            O = odd ? group_sum64<G>(O) : 0;
            if (gl == 0) out[seg] = fold_ref(combine((uint64_t)d[u].w, W, O, odd));
        }
    }
}

// ---------------------------------------------------------------- balanced
// Mixed-length batches. A lane group per segment wastes lanes and loads when
// lengths vary (a 64-B segment in a 96-chunk group). Here a wave takes 64
// segments (one per lane), lays their aligned hulls end to end in a "chunk
// space" by a wave prefix sum, and sweeps that space 64 chunks per load
// instruction: lane l of sub-round k loads chunk R + 64k + l whatever segment
// it belongs to, so every instruction does 64 useful 16-B loads. Each lane
// finds its segment from the segments that start inside its 64-chunk window
// (a short scalar loop over a ballot), masks its chunk to the segment's byte
// range, and the per-segment sums come from a wave inclusive scan of the chunk
// sums: the lane holding a segment's last chunk in the window adds
// X[end] - X[run start - 1] to the segment's LDS accumulator.

// Inclusive prefix sum over the 64 lanes, all DPP: row shifts 1/2/4/8 scan
// each row of 16, row_bcast:15 adds row 0's (row 2's) total into row 1 (row 3),
// row_bcast:31 adds lane 31's running total into rows 2 and 3 (GFX9 DPP).
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return x;
}

// N independent inclusive scans stepped in lockstep: each DPP step of one scan
// fills the other scans' DPP read-after-write wait states (one scan alone pads
// every step with s_nop).
template <int N>
__device__ __forceinline__ void wave_scan_incl_n(uint32_t (&x)[N]) {
#define TC_SCAN_STEP(ctrl, rmask)                                                                        \
    _Pragma("unroll") for (int i = 0; i < N; ++i) x[i] +=                                                 \
        (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x[i], ctrl, rmask, 0xF, false);
    TC_SCAN_STEP(0x111, 0xF)   // row_shr:1
    TC_SCAN_STEP(0x112, 0xF)   // row_shr:2
    TC_SCAN_STEP(0x114, 0xF)   // row_shr:4
    TC_SCAN_STEP(0x118, 0xF)   // row_shr:8
    TC_SCAN_STEP(0x142, 0xA)   // row_bcast:15 -> rows 1, 3
    TC_SCAN_STEP(0x143, 0xC)   // row_bcast:31 -> rows 2, 3
#undef TC_SCAN_STEP
}

__device__ __forceinline__ uint32_t bperm(uint32_t x, uint32_t src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)x);
}

constexpr uint32_t kNoHole = 0x40000000u;   // a hole offset past any segment (int32-safe)

// Bytes [lo, hi) of a 16-byte chunk as two 64-bit byte masks.
__device__ __forceinline__ void range_mask(int32_t lo, int32_t hi, uint64_t& m0, uint64_t& m1) {
    lo = lo < 0 ? 0 : (lo > 16 ? 16 : lo);
    hi = hi < 0 ? 0 : (hi > 16 ? 16 : hi);
    const int32_t lo0 = lo < 8 ? lo : 8, hi0 = hi < 8 ? hi : 8;
    const int32_t lo1 = lo > 8 ? lo - 8 : 0, hi1 = hi > 8 ? hi - 8 : 0;
    m0 = bytemask64(hi0) & ~bytemask64(lo0);
    m1 = bytemask64(hi1) & ~bytemask64(lo1);
}

// The chunk's bytes at segment-relative offsets [0, len) except the two-byte
// hole [hole, hole + 2) (the zeroed check of a FILL; hole >= len: none);
// rel = segment-relative offset of the chunk's first byte. W: aligned-word sum,
// O: odd-address byte sum (only when want_odd).
__device__ __forceinline__ void chunk_masked(u32x4 v, int32_t rel, int32_t len, int32_t hole, bool want_odd,
                                             uint32_t& W, uint32_t& O) {
    uint64_t m0, m1;
    range_mask(-rel, len - rel, m0, m1);
    if (hole != (int32_t)kNoHole) {   // kernel-uniform
        uint64_t h0, h1;
        range_mask(hole - rel, hole + 2 - rel, h0, h1);
        m0 &= ~h0;
        m1 &= ~h1;
    }
    const uint32_t d0 = v.x & (uint32_t)m0, d1 = v.y & (uint32_t)(m0 >> 32);
    const uint32_t d2 = v.z & (uint32_t)m1, d3 = v.w & (uint32_t)(m1 >> 32);
    W = sad16(d0, W); W = sad16(d1, W); W = sad16(d2, W); W = sad16(d3, W);
    if (want_odd) {
        O = sad8(d0 & 0xff00ff00u, O); O = sad8(d1 & 0xff00ff00u, O);
        O = sad8(d2 & 0xff00ff00u, O); O = sad8(d3 & 0xff00ff00u, O);
    }
}

// One round of the balanced sweep: for each of its C windows of 64 chunks, every lane's owner
// segment, the owner's first chunk, the chunk's index in the owner's hull, and the chunk itself
// (its load issued here, consumed by lb_consume).
template <int C>
struct LbRound {
    uint32_t own[C], pc[C], po[C];
    u32x4 v[C];
};

// The owner search of window [W0, W0 + 64): a scalar loop over the segments that start in the
// window (a ballot), one readlane each — ~12 instructions per start, most of them scalar.
__device__ __forceinline__ uint32_t lb_owner_loop(uint32_t W0, uint32_t P, uint32_t nj, uint32_t lane,
                                                  uint32_t& carry) {
    // segments starting inside [W0, W0 + 64), in lane (= start) order
    uint64_t M = __ballot(nj != 0 && P - W0 < 64u && P >= W0);
    uint32_t o = carry;
    while (M) {
        const int j = __builtin_ctzll(M);
        M &= M - 1;
        const uint32_t st = (uint32_t)__builtin_amdgcn_readlane((int)P, j) - W0;
        o = lane >= st ? (uint32_t)j : o;
    }
    carry = (uint32_t)__builtin_amdgcn_readlane((int)o, 63);
    return o;
}

// The loop-free owner search (measurement variant, TCPCSUM_LB_VARIANT bit 0): once per tile the
// segments' first chunks are marked in a per-wave LDS bitmap over the chunk space (T <= 8192
// bits) and a permute makes `inv`: rank among the non-empty segments -> lane. Per window one
// broadcast LDS read gives the 64 start bits S; chunk W0 + l belongs to the segment of rank
// base + popcount(S & bits [0, l]) - 1 (base: starts in the windows before), found by one
// bpermute. No loop, whatever the number of starts (small packets: ~20 per window).
__device__ __forceinline__ uint32_t lb_owner_bitmap(uint32_t W0, uint32_t lane, uint32_t inv, uint32_t& base,
                                                    const uint32_t* bm) {
    const uint64_t S = *(const volatile uint64_t*)(bm + (W0 >> 5));   // W0 % 64 == 0: 8-B aligned
    const uint64_t pre = S & ((2ull << lane) - 1ull);                  // lane 63: every bit
    const uint32_t rank = base + (uint32_t)__builtin_popcountll(pre) - 1u;
    base += (uint32_t)__builtin_popcountll(S);
    return bperm(inv, rank);
}

// Per-lane segment [a, a + len) (len <= 1 MiB: the chunk space stays < 2^32),
// hole (the same segment-relative offset for every segment, kNoHole: none) as
// above. On return accW[lane] / accO[lane] hold the lane's segment sums W and O
// (O only when want_odd, wave-uniform). acc: the wave's 2 x 64 u64 LDS slots;
// mark: its 256 u32 LDS slots (the bitmap owner search).
// A4: every segment of the tile 4-B aligned in start and length (packed
// IPv4/TCP packets of 4-B multiples, IMIX) — dword-granular masks, no byte
// masks. A template parameter, not a branch in the sweep: a branch there joins
// after the masks, and the join waits for every load of the round.
// TCPCSUM_LB_VARIANT bit 0: the bitmap owner search; bit 1: software-pipelined rounds — the
// owner search and the loads of round r + 1 are issued before round r is summed (two LbRound
// register sets), so a round's loads no longer wait for the previous round's scans and atomics.
template <int C, bool A4>
__device__ __forceinline__ void lb_sums_t(const uint8_t* a, uint32_t len, uint32_t hole, bool want_odd,
                                          uint64_t* accW, uint64_t* accO, uint32_t* mark) {
    constexpr bool BITMAP = (TCPCSUM_LB_VARIANT & 1) != 0;
    constexpr bool PIPE = (TCPCSUM_LB_VARIANT & 2) != 0;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t m = (uint32_t)((uintptr_t)a & 15u);
    const uint32_t nj = len ? (m + len + 15u) >> 4 : 0u;   // chunks of the aligned hull
    const uint32_t lm = len | (m << 27);                     // len < 2^27
    const uint32_t incl = wave_scan_incl(nj);
    const uint32_t P = incl - nj;                           // first chunk in the chunk space
    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint64_t a0 = (uint64_t)(uintptr_t)a - m;
    const uint32_t a_lo = (uint32_t)a0, a_hi = (uint32_t)(a0 >> 32);
    accW[lane] = 0;
    if (want_odd) accO[lane] = 0;
    uint32_t carry = 0;   // segment owning the next window's first chunk (loop search)
    uint32_t base = 0, inv = 0;   // bitmap search
    const bool bitmap = BITMAP && T <= 8192u;
    if (bitmap) {
        volatile uint32_t* bm = mark;
#pragma unroll
        for (int q = 0; q < 4; ++q) bm[lane * 4u + q] = 0u;
        __builtin_amdgcn_wave_barrier();
        if (nj != 0) atomicOr(mark + (P >> 5), 1u << (P & 31u));
        __builtin_amdgcn_wave_barrier();
        const uint64_t NZ = __ballot(nj != 0);
        const uint32_t below =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(NZ >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)NZ, 0u));
        const uint32_t K = (uint32_t)__builtin_popcountll(NZ);
        // a permutation: non-empty segments to their ranks, empty ones after them
        const uint32_t dest = nj != 0 ? below : K + (lane - below);
        inv = (uint32_t)__builtin_amdgcn_ds_permute((int)(dest << 2), (int)lane);
    }
    auto issue = [&](LbRound<C>& r, uint32_t R) {
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint32_t W0 = R + 64u * k;
            const uint32_t g = W0 + lane;
#if TCPCSUM_LB_VARIANT & 8   // knock-out (results WRONG): no owner search, what it costs
            const uint32_t o = carry;
#else
            const uint32_t o = bitmap ? lb_owner_bitmap(W0, lane, inv, base, mark) : lb_owner_loop(W0, P, nj, lane, carry);
#endif
            r.own[k] = o;
            r.po[k] = bperm(P, o);
            r.pc[k] = g - r.po[k];   // chunk index inside the owner's hull
            const uint64_t base = (uint64_t)bperm(a_lo, o) | ((uint64_t)bperm(a_hi, o) << 32);
            r.v[k] = ld16(zsel(g < T, reinterpret_cast<const uint8_t*>(base + (uint64_t)r.pc[k] * 16u)));
        }
    };
    auto consume = [&](const LbRound<C>& r, uint32_t R) {
        uint32_t w[C], od[C], sr[C];
        bool end[C];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint32_t W0 = R + 64u * k;
            const uint32_t g = W0 + lane;
            const uint32_t o = r.own[k];
            const uint32_t lmo = bperm(lm, o);
            const uint32_t lo = lmo & ((1u << 27) - 1u), mo = lmo >> 27;
            const uint32_t no = (mo + lo + 15u) >> 4;
            w[k] = 0;
            od[k] = 0;
            // lanes past the chunk space (g >= T) loaded the zero buffer: they sum 0
            if constexpr (A4) {
                const uint32_t rel = r.pc[k] * 16u - mo;   // dwords at rel + 4j: inside iff < lo (unsigned)
                const u32x4 x = r.v[k];
                uint32_t t = sad16(rel < lo ? x.x : 0u, 0u);
                t = sad16(rel + 4u < lo ? x.y : 0u, t);
                t = sad16(rel + 8u < lo ? x.z : 0u, t);
                w[k] = sad16(rel + 12u < lo ? x.w : 0u, t);
            } else {
                chunk_masked(r.v[k], (int32_t)(r.pc[k] * 16u) - (int32_t)mo, (int32_t)lo, (int32_t)hole, want_odd,
                             w[k], od[k]);
            }
            end[k] = g < T && (r.pc[k] + 1u == no || lane == 63u || g + 1u == T);
            sr[k] = r.po[k] > W0 ? r.po[k] - W0 : 0u;   // the run's first lane in this window
        }
        // the C windows' scans interleaved (their DPP steps fill each other's wait states)
        wave_scan_incl_n<C>(w);
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint32_t Xp = bperm(w[k], sr[k] ? sr[k] - 1u : 0u);
            if (end[k])
                atomicAdd(reinterpret_cast<unsigned long long*>(accW + r.own[k]),
                          (unsigned long long)(w[k] - (sr[k] ? Xp : 0u)));
        }
        if (want_odd) {   // wave-uniform
            wave_scan_incl_n<C>(od);
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t Yp = bperm(od[k], sr[k] ? sr[k] - 1u : 0u);
                if (end[k])
                    atomicAdd(reinterpret_cast<unsigned long long*>(accO + r.own[k]),
                              (unsigned long long)(od[k] - (sr[k] ? Yp : 0u)));
            }
        }
    };
    constexpr uint32_t STEP = 64u * C;
    if constexpr (!PIPE) {
        for (uint32_t R = 0; R < T; R += STEP) {
            LbRound<C> r;
            issue(r, R);
            consume(r, R);
        }
    } else {
        LbRound<C> ra, rb;
        if (T) issue(ra, 0);
        for (uint32_t R = 0; R < T; R += 2u * STEP) {
            if (R + STEP < T) issue(rb, R + STEP);
            consume(ra, R);
            if (R + STEP >= T) break;
            if (R + 2u * STEP < T) issue(ra, R + 2u * STEP);
            consume(rb, R + STEP);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// Every segment of the tile starting 4-B aligned (TCP segments of packets in malloc'd or
// 16-B packed buffers: TCP at ip + 20): the sweep takes the dword-granular A4 path over each
// segment's first len & ~3 bytes, and its last len & 3 bytes (at an even offset: low bytes
// of their words) come from one aligned dword per segment, loaded before the sweep. The
// byte-granular masks of the A4 = false path cost ~45 VALU per 1 KiB window: the flush mix
// VERIFY ran at 133 VALU instructions per KiB (rocprofv3 SQ_INSTS_VALU,
// profiles/r06_wire_mix_pmc.json).
template <int C>
__device__ __forceinline__ void lb_sums(const uint8_t* a, uint32_t len, uint32_t hole, bool want_odd,
                                        uint64_t* accW, uint64_t* accO, uint32_t* mark) {
    const bool a4 = __ballot(len != 0 && ((uint32_t)(uintptr_t)a & 3u) != 0) == 0 && hole == kNoHole;
    if (a4 && __ballot((len & 3u) != 0) == 0) {   // lengths too: nothing left over
        lb_sums_t<C, true>(a, len, hole, want_odd, accW, accO, mark);
    } else if (a4) {
        const uint32_t body = len & ~3u, tail = len & 3u;
        // the dword holding the tail bytes: inside the segment's last aligned dword, so on a
        // page the segment is on
        const uint32_t td = ldg<uint32_t>(zsel(tail != 0u, a + body));
        lb_sums_t<C, true>(a, body, hole, want_odd, accW, accO, mark);
        if (tail)
            atomicAdd(reinterpret_cast<unsigned long long*>(accW + (threadIdx.x & 63)),
                      (unsigned long long)sad16(td & ((1u << (8u * tail)) - 1u), 0u));
        __builtin_amdgcn_wave_barrier();
    } else {
        lb_sums_t<C, false>(a, len, hole, want_odd, accW, accO, mark);
    }
}

// One segment summed by the whole wave (wave-uniform a, len): 64 chunks per
// load instruction, u32 lane partials flushed to u64 every 8 rounds. For the
// rare segments too long for the balanced chunk space.
__device__ __forceinline__ void wave_seg_sums(const uint8_t* a, uint32_t len, bool want_odd, uint64_t& W,
                                              uint64_t& O) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t m = (uint32_t)((uintptr_t)a & 15u);
    const uint8_t* a0 = a - m;
    const uint64_t nch = ((uint64_t)m + len + 15u) >> 4;
    uint64_t w64 = 0, o64 = 0;
    for (uint64_t r = 0; r < nch; r += 512) {
        uint32_t w = 0, o = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint64_t idx = r + 64u * k + lane;
            const u32x4 v = ld16(zsel(idx < nch, a0 + idx * 16u));
            if (idx < nch) chunk_wo_bytes(v, (int64_t)idx * 16 - m, (int64_t)len, want_odd, w, o);
        }
        w64 += w;
        o64 += o;
    }
    W = group_sum64<64>(w64);
    O = want_odd ? group_sum64<64>(o64) : 0;
}

// Ragged descriptors, balanced: 64 descriptors per wave tile. Segments longer
// than 1 MiB (chunk space kept < 2^32) are summed one at a time by the wave.
template <int C>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TCPCSUM_DESC_LB_WAVES, 8))) void k_desc_lb(const uint8_t* __restrict__ base,
                                                 const tcpcsum_desc_t* __restrict__ desc, uint64_t n,
                                                 uint16_t* __restrict__ out, uint32_t spw) {
    // spw: segments per wave tile (1..64; lanes >= spw hold no segment) — fewer
    // for long segments, so a batch of them still spreads over enough waves
    __shared__ uint64_t acc[4][2][64];
    __shared__ __attribute__((aligned(8))) uint32_t marks[(TCPCSUM_LB_VARIANT & 1) ? 4 : 1][(TCPCSUM_LB_VARIANT & 1) ? 256 : 2];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* mark = marks[(TCPCSUM_LB_VARIANT & 1) ? wv : 0];
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t ntiles = (n + spw - 1) / spw;
    for (uint64_t t = (uint64_t)blockIdx.x * 4u + wv; t < ntiles; t += nwaves) {   // block order, as k_desc
        const uint64_t seg = t * spw + (uint64_t)lane;
        const bool mine = (uint32_t)lane < spw && seg < n;
        const u32x4 d = ldg<u32x4>(zsel(mine, reinterpret_cast<const uint8_t*>(desc + seg)));
        const uint8_t* p = base + ((uint64_t)d.x | ((uint64_t)d.y << 32));
        const uint32_t len = d.z;   // 0 past n
        const bool odd = ((uintptr_t)p & 1u) != 0;
        const bool any_odd = __ballot(len != 0 && odd) != 0;
        const bool big = len > (1u << 20);
        uint64_t bw = 0, bo = 0;
        for (uint64_t M = __ballot(big); M; M &= M - 1) {   // wave-uniform, rare
            const int j = __builtin_ctzll(M);
            const uint64_t pj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uintptr_t)p, j) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uintptr_t)p >> 32), j) << 32);
            const uint32_t lj = (uint32_t)__builtin_amdgcn_readlane((int)len, j);
            uint64_t W, O;
            wave_seg_sums(reinterpret_cast<const uint8_t*>(pj), lj, any_odd, W, O);
            if (lane == j) { bw = W; bo = O; }
        }
        lb_sums<C>(p, big ? 0u : len, kNoHole, any_odd, acc[wv][0], acc[wv][1], mark);
        const uint64_t W = big ? bw : acc[wv][0][lane];
        const uint64_t O = !any_odd ? 0 : big ? bo : acc[wv][1][lane];
        if (mine) out[seg] = fold_ref(combine((uint64_t)d.w, W, O, odd));
    }
}

// ---------------------------------------------------------------- wire (IPv4)
// Packet i at pkts + off[i] (see tcpcsum.h). Tiles of U packets per lane
// group; the offsets of the next tile are in flight while a tile is summed.
// Each packet costs one memory round trip: the group loads the aligned hull of
// [ip, ip + span) speculatively (up to its G*C chunks; span = cap, bounded by
// the region and by the next packet's offset when that lies ahead — a hint:
// a packet longer than its span takes fix-up loads), and the IP header
// fields and the TCP check are then read out of the first G chunks — lane gl
// holds chunk gl, so a field is a group-local ds_bpermute plus v_alignbyte,
// not a global byte load (G >= 8 covers bytes [0, 113): any IHL and the check
// at ihl*4 + 16). The TCP range [ihl*4, tot_len) and (IPHDR) the IP header
// range [0, ihl*4) are summed from registers with byte masks at their ends.
// Longer packets take extra rounds. FILL subtracts the check word (what
// zeroing it does: TCP+16 is an even offset) and stores the result in place.
struct IpPkt {
    uint8_t* ip;
    uint64_t o;
    uint32_t m;      // ip & 15
    uint32_t spec;   // chunks loaded speculatively
    uint32_t room;   // readable bytes at ip: min(region end, the packet's own bound), clamped
    bool live;    // a packet of the batch
    bool hdr;     // its 20-byte IP header is readable
};

// x, computed here: an identity DPP move (quad_perm 0,1,2,3) is convergent, so
// the compiler can neither sink the computation of x past control flow nor
// rematerialize it from its operands later — it holds one VGPR from here on.
__device__ __forceinline__ uint32_t pin_vgpr(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xE4, 0xF, 0xF, false);
}

// A native u16 at p: one 2-byte store when p is even, two byte stores otherwise.
__device__ __forceinline__ void store_u16(uint8_t* p, uint16_t v) {
    if (((uintptr_t)p & 1u) == 0) {
        stg<uint16_t>(p, v);
    } else {
        stg<uint8_t>(p, (uint8_t)(v & 0xffu));
        stg<uint8_t>(p + 1, (uint8_t)(v >> 8));
    }
}

// Write-through (sc0 sc1) stores, rather than lines left dirty in L2 — all
// compiler-visible, so the hazard recognizer owns the store-data wait states
// (round 3's inline-asm stores hid them: the compiler reused a dwordx4 store's
// data VGPRs one instruction later and 4 of 1M packets were corrupted until a
// hand-counted s_nop went in). A relaxed atomic store at system scope is
// exactly global_store_{byte,short} sc0 sc1 on gfx950 (the memory model's
// system-scope store: no wait, no fence); a 16-byte one is a raw buffer store
// with cache policy sc0|sc1 (CPol bits 1 | 16).
constexpr int kCpolSc0Sc1 = TCPCSUM_LINE_CPOL;   // 1 | 16 (measurement builds may change it)

template <class T>
__device__ __forceinline__ void stg_wt(uint8_t* p, T v) {
    __hip_atomic_store((gptr<T>)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 16 bytes at the 16-B aligned p, written through. A buffer store's base sits in
// scalar registers, so it is the wave's: its first active lane's address less
// 2 GiB, and each lane stores at its 32-bit offset from there. A lane whose
// address lies outside that 4 GiB window (never, for the packets of one wave
// tile in any batch layout tested; possible only for pointer batches scattered
// over more than 2 GiB) takes a default-policy store — same bytes, only not
// written through.
__device__ __forceinline__ void stg_wt16(uint8_t* p, u32x4 v) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint64_t first = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                           (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint64_t base = first > 0x80000000ull ? first - 0x80000000ull : 0ull;
    const uint64_t rel = a - base;
    if (a >= base && rel <= 0xFFFFFF00ull) {
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uintptr_t)base), 0, -1, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(uint32_t)rel, 0, kCpolSc0Sc1);
    } else {
        *(gptr<u32x4>)(p) = v;
    }
}

// 16 bytes at the 16-B aligned p, written through, relative to a wave-uniform
// base: a kernel argument, or a readfirstlane taken in converged code before the
// (divergent) store branch — stg_wt16 builds its base from the first active lane
// inside the branch, a readfirstlane pair and the descriptor per store. A lane
// outside [base, base + 4 GiB) takes a default-policy store (same bytes).
__device__ __forceinline__ void stg_wt16_at(uint8_t* p, u32x4 v, uint64_t base) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint64_t rel = a - base;
    if (a >= base && rel <= 0xFFFFFF00ull) {
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uintptr_t)base), 0, -1, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(uint32_t)rel, 0, kCpolSc0Sc1);
    } else {
        *(gptr<u32x4>)(p) = v;
    }
}

// The write-through base for a wave whose stores land near addr (any lane's, taken
// where the wave is converged): 2 GiB below it, so the window covers addr +- 2 GiB.
__device__ __forceinline__ uint64_t wt_base_near(uint64_t addr) {
    const uint64_t first = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32)) << 32) |
                           (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)addr);
    return first > 0x80000000ull ? first - 0x80000000ull : 0ull;
}

// A native u16 at p, written through: a lone 2-byte store per packet in the
// middle of a read stream costs less that way (tools/fill_store_probe.hip: +62
// vs +72 us per 1M stores).
__device__ __forceinline__ void store_u16_wt(uint8_t* p, uint16_t v) {
    if (((uintptr_t)p & 1u) == 0) {
        stg_wt<uint16_t>(p, v);
    } else {
        stg_wt<uint8_t>(p, (uint8_t)(v & 0xffu));
        stg_wt<uint8_t>(p + 1, (uint8_t)(v >> 8));
    }
}

// Dword D (counted from the aligned start of the packet's window) out of the
// group's first-round chunks c0 (lane gbase + k holds chunk k).
__device__ __forceinline__ uint32_t grp_dword(const u32x4 c0, int gbase, uint32_t D) {
    const uint32_t j = D & 3u;
    const uint32_t mine = j == 0 ? c0.x : j == 1 ? c0.y : j == 2 ? c0.z : c0.w;
    return (uint32_t)__shfl((int)mine, gbase + (int)(D >> 2), 64);
}

// Dword D out of the group's first two rounds of chunks (lane gbase + k holds
// chunk k in c0 and chunk G + k in c1): windows of 2*G chunks for G = 8.
template <int G>
__device__ __forceinline__ uint32_t grp_dword2(const u32x4 c0, const u32x4 c1, int gbase, uint32_t D) {
    const uint32_t j = D >> 2;
    const bool hi = j >= (uint32_t)G;
    const u32x4 c = hi ? c1 : c0;
    const uint32_t q = D & 3u;
    const uint32_t mine = q == 0 ? c.x : q == 1 ? c.y : q == 2 ? c.z : c.w;
    return (uint32_t)__shfl((int)mine, gbase + (int)(hi ? j - (uint32_t)G : j), 64);
}

// The 4 packet bytes at window offset a (little-endian dword), out of the
// group's first round (C == 1 or G >= 16) or first two rounds of chunks.
template <int G, int C>
__device__ __forceinline__ uint32_t grp_bytes4(const u32x4 (&v)[C], int gbase, uint32_t a) {
    uint32_t lo, hi;
    if constexpr (C == 1 || G >= 16) {
        lo = grp_dword(v[0], gbase, a >> 2);
        hi = grp_dword(v[0], gbase, (a >> 2) + 1u);
    } else {
        lo = grp_dword2<G>(v[0], v[1], gbase, a >> 2);
        hi = grp_dword2<G>(v[0], v[1], gbase, (a >> 2) + 1u);
    }
    return __builtin_amdgcn_alignbyte(hi, lo, a & 3u);
}

// One packet's results, committed by the group's lane 0.
struct IpDone {
    uint8_t* ip;
    uint64_t i;
    uint32_t th;
    uint32_t urg;   // urg_ptr (TCP+18) in the high half, for a check|urg_ptr dword store
    uint16_t c, ic;
    uint8_t st;
    bool w;     // a packet of the batch: out / status are written
    bool fill;  // checks are stored in place
};

// plen (nullable): per-packet readable bytes (scatter-gather batches: pkts = 0,
// off[i] = the packet's address, limit = ~0). A packet never reads past
// min(limit - off[i], plen[i]).
// VER: VERIFY (the launch's mode has TCPCSUM_IPV4_VERIFY) as a compile-time
// constant — the FILL stores and their live registers compiled out of the
// VERIFY kernel (k_ipv4<8,4,1>: 120 -> 88 VGPRs, 4 -> 5 waves per SIMD).
// FILL with (8,4) lane groups, one packet per group — the default MTU shape — asks the
// compiler for 5 waves per SIMD: it needs 102 VGPRs (4 waves) and fits in 96 with two
// spilled to scratch (12 bytes per lane, off the summation loop); 1M x 1500-B packets
// packed 0.343 -> 0.330 ms, 1024-B slots 0.212 -> 0.206, 1536-B slots 0.297 -> 0.293
// (tools/wire_lib_ab.py, profiles/r03_wire_verify_template_ab.jsonl). Elsewhere the
// compiler's choice (TCPCSUM_WIRE_WAVES, a measurement knob, default 1) — forced
// unrolls would spill dozens of registers at 5 waves.
constexpr int wire_waves(int G, int C, int U, bool VER) {
    return (!VER && G == 8 && C == 4 && U == 1 && TCPCSUM_WIRE_WAVES < 5) ? 5 : TCPCSUM_WIRE_WAVES;
}

template <int G, int C, int U, bool NT, bool PL, bool VER>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(wire_waves(G, C, U, VER), 8))) void k_ipv4(uint8_t* __restrict__ pkts, const uint64_t* __restrict__ off,
                                              const uint32_t* __restrict__ plen,
                                              uint64_t n, uint32_t cap, uint64_t limit, int mode,
                                              uint16_t* __restrict__ out, uint8_t* __restrict__ status,
                                              uint16_t* __restrict__ ipout, uint32_t amask, int store_mode) {
    // amask: window alignment - 1. Lane gl of a group loads window chunks k*G+gl,
    // so with 128-B windows every group load instruction covers whole 128-B
    // lines however the packet is aligned. Header fields lie in window bytes
    // [0, amask + 81): 16-B windows need G >= 8, 128-B windows G >= 16 or C >= 2.
    static_assert(G >= 8, "the header and TCP check are read from the group's first chunks");
    if constexpr (C == 1 && G < 16) amask = 15u;
    constexpr int GPW = 64 / G;
    constexpr int SPT = GPW * U;
    const int lane = threadIdx.x & 63;
    const int q = lane / G, gl = lane % G;
    const int gbase = lane - gl;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t ntiles = (n + SPT - 1) / SPT;
    constexpr bool verify = VER;
    const bool iphdr = (mode & TCPCSUM_IPV4_IPHDR) != 0;
    // XCD order for MTU-size packets: 1536 / 2048-B slots and packed 1500-B packets VERIFY
    // -2.4 / -3.4 / -2.4 %, FILL -1..-2 % where it moved; 9216-B jumbo slots VERIFY +3 %, so
    // batches whose cap passes 4 KiB keep block order (profiles/r05_xcd_kernels_ab.jsonl)
    uint64_t t = xcd_block(cap <= 4096u ? (ntiles + 3) / 4 : ~0ull) * 4u + (threadIdx.x >> 6);
    // offsets of packet i and of packet i + 1 (0 past the end: no bound)
    uint64_t on[U], on1[U];
    uint32_t pn[U];
    auto load_off = [&](uint64_t tile) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = tile * SPT + (uint64_t)(u * GPW + q);
            on[u] = ldg<uint64_t>(zsel(i < n, reinterpret_cast<const uint8_t*>(off + i)));
            on1[u] = ldg<uint64_t>(zsel(i + 1 < n, reinterpret_cast<const uint8_t*>(off + i + 1)));
            if constexpr (PL)
                pn[u] = ldg<uint32_t>(zsel(i < n, reinterpret_cast<const uint8_t*>(plen + i)));
            else
                pn[u] = 0xffffffffu;
        }
    };
    IpPkt p[U];
    u32x4 v[U][C];
    // the tile's speculative packet loads (offsets already in on / on1)
    auto issue = [&](uint64_t tile) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = tile * SPT + (uint64_t)(u * GPW + q);
            p[u].live = i < n;
            p[u].o = on[u];
            // scatter-gather (PL): pkts is 0 and off[i] the address — integer
            // arithmetic, not a pointer offset from null
            uint8_t* ip = PL ? reinterpret_cast<uint8_t*>((uintptr_t)pkts + p[u].o) : pkts + p[u].o;
            p[u].ip = ip;
            p[u].m = (uint32_t)((uintptr_t)ip & amask);
            uint64_t span;
            if constexpr (PL) {   // bounded by the region and by the packet's own length
                const uint64_t rr = p[u].live && p[u].o < limit ? limit - p[u].o : 0u;
                const uint32_t room = (uint32_t)(rr < (uint64_t)pn[u] ? rr : (uint64_t)pn[u]);
                p[u].hdr = room >= 20u;
                p[u].room = room;
                span = p[u].hdr ? (room < cap ? room : cap) : 0u;
            } else {              // bounded by the region
                p[u].hdr = p[u].live && p[u].o < limit && limit - p[u].o >= 20u;
                const uint64_t room = p[u].hdr ? limit - p[u].o : 0u;
                span = room < cap ? room : cap;
            }
            const bool live = p[u].hdr;   // a dead slot reads zeros: ver 0, skipped
            // speculative payload chunks: the aligned hull of [ip, ip + span); at
            // least 80 bytes (any IP header and the TCP check) when the packet has them
            const uint64_t gap = on1[u] > p[u].o ? on1[u] - p[u].o : ~0ull;
            const uint64_t hint = gap > 80u ? gap : 80u;
            span = span < hint ? span : hint;
            const uint32_t nch = (p[u].m + (uint32_t)span + 15u) >> 4;
            p[u].spec = nch;
            const uint8_t* a0 = ip - p[u].m;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = (uint32_t)(k * G + gl);
                // chunks wholly before the packet (128-B windows) are not read
                v[u][k] = ldq<NT>(zsel(live && idx < nch && idx * 16u + 16u > p[u].m, a0 + (uint64_t)idx * 16u));
            }
        }
    };
    // FILL's line stores go out written through relative to a wave-uniform base
    // (stg_wt16_at): the region's start (rounded down to its 128-B window) when the
    // whole region lies within 4 GiB of it — a kernel argument, no per-store setup —
    // else 2 GiB below the tile's first packet, taken once per tile where the wave
    // is converged, not inside the divergent store branch.
    const bool region_base = !PL && limit <= 0xFFFFFE00ull;
    uint64_t wt_base = region_base ? ((uint64_t)(uintptr_t)pkts & ~(uint64_t)127u) : 0u;
    const __amdgpu_buffer_rsrc_t wt_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uintptr_t)wt_base), 0, -1, 0x00020000);
    auto process = [&](int u, uint64_t i) -> IpDone {
        IpDone d;
        d.w = false;
        d.fill = false;
        d.i = i;
        d.ip = p[u].ip;
        d.th = 0;
        d.urg = 0;
        d.c = 0;
        d.ic = 0;
        d.st = TCPCSUM_PKT_SKIPPED;
        if (!p[u].live) return d;   // group-uniform
        d.w = true;
        uint8_t* ip = p[u].ip;
        const uint32_t m = p[u].m;
        const uint32_t h0 = grp_bytes4<G, C>(v[u], gbase, m);        // ver/ihl, tos, tot_len
        const uint32_t h8 = grp_bytes4<G, C>(v[u], gbase, m + 8u);   // ttl, protocol, check
        const uint32_t ver = (h0 >> 4) & 15u, ihl = h0 & 15u;
        const uint32_t tot = ((h0 >> 8) & 0xff00u) | (h0 >> 24);
        const uint32_t proto = (h8 >> 8) & 0xffu;
        const bool fits = PL ? tot <= p[u].room : p[u].o + tot <= limit;
        const bool ok = p[u].hdr && ver == 4u && proto == 6u && ihl >= 5u && tot >= ihl * 4u + 20u && tot <= cap &&
                        fits;
        if (!ok) return d;   // group-uniform: skipped, out = 0
        const uint32_t th = ihl * 4u;   // TCP start, packet-relative (even)
        const bool odd = (m & 1u) != 0;
        const uint32_t sa = grp_bytes4<G, C>(v[u], gbase, m + 12u), da = grp_bytes4<G, C>(v[u], gbase, m + 16u);
        const uint32_t tcp_len = tot - th;
        const uint32_t len_be = ((tcp_len & 0xffu) << 8) | ((tcp_len >> 8) & 0xffu);   // htons
        // context.c:104-119 closed form: six native u16 words of the pseudo header.
        // Pinned here (pin_vgpr): left to itself the compiler computes it — and the
        // check word — after the long-packet rounds below, keeping the two raw
        // dwords of each field live across them, which spilled two VGPRs of the
        // FILL kernel to scratch at its 5 waves per SIMD.
        const uint32_t ps32 = pin_vgpr((sa & 0xffffu) + (sa >> 16) + (da & 0xffffu) + (da >> 16) + 0x0600u + len_be);
        const uint32_t check_dw = pin_vgpr(grp_bytes4<G, C>(v[u], gbase, m + th + 16u));   // check | urg_ptr
        const uint32_t check_word = check_dw & 0xffffu;
        const uint32_t nch_tot = (m + tot + 15u) >> 4;
        if (nch_tot > p[u].spec) {   // longer than its span hint (group-uniform, rare)
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = (uint32_t)(k * G + gl);
                if (idx >= p[u].spec && idx < nch_tot) v[u][k] = ldq<NT>(ip - m + (uint64_t)idx * 16u);
            }
        }
        uint32_t w = 0, o = 0, wi = 0, oi = 0;
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const int32_t pos = (int32_t)((uint32_t)(k * G + gl) * 16u) - (int32_t)m;   // chunk start, packet-relative
            const u32x4 x = v[u][k];
            // whole chunks of [th, tot): no masks (select the chunk's sum in or out)
            const bool full = pos >= (int32_t)th && pos + 16 <= (int32_t)tot;
            const uint32_t wk = sad16(x.w, sad16(x.z, sad16(x.y, sad16(x.x, 0u))));
            w += full ? wk : 0u;
            if (odd) {
                const uint32_t ok8 = sad8(x.w & 0xff00ff00u, sad8(x.z & 0xff00ff00u,
                                          sad8(x.y & 0xff00ff00u, sad8(x.x & 0xff00ff00u, 0u))));
                o += full ? ok8 : 0u;
            }
            // the (at most two) edge chunks of a packet: masked, behind a wave-uniform
            // branch — on MTU slots only one or two of the C rounds hold any
            const bool part = !full && pos + 16 > (int32_t)th && pos < (int32_t)tot;
            if (__builtin_amdgcn_ballot_w64(part) != 0) {
                if (part) chunk_wo_bytes(x, (int64_t)pos - th, (int64_t)(tot - th), odd, w, o);
            }
            if (iphdr && pos < (int32_t)th) chunk_wo_bytes(x, (int64_t)pos, (int64_t)th, odd, wi, oi);
        }
        uint64_t W = w, O = o;
        // packets longer than the group's first G*C chunks (jumbo frames): the same
        // split — whole chunks unmasked, the tail chunk masked behind a wave-uniform
        // branch; chunks past the packet read the zero buffer (no predicated loads)
        for (uint32_t r = (uint32_t)(G * C); r < nch_tot; r += (uint32_t)(G * C)) {
            uint32_t w2 = 0, o2 = 0;
            u32x4 xs[C];
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = r + (uint32_t)(k * G + gl);
                xs[k] = ldq<NT>(zsel(idx < nch_tot, ip - m + (uint64_t)idx * 16u));
            }
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = r + (uint32_t)(k * G + gl);
                const int32_t pos = (int32_t)(idx * 16u) - (int32_t)m;
                const u32x4 x = xs[k];
                const bool full = idx < nch_tot && pos >= (int32_t)th && pos + 16 <= (int32_t)tot;
                const uint32_t wk = sad16(x.w, sad16(x.z, sad16(x.y, sad16(x.x, 0u))));
                w2 += full ? wk : 0u;
                if (odd) {
                    const uint32_t ok8 = sad8(x.w & 0xff00ff00u, sad8(x.z & 0xff00ff00u,
                                              sad8(x.y & 0xff00ff00u, sad8(x.x & 0xff00ff00u, 0u))));
                    o2 += full ? ok8 : 0u;
                }
                const bool part = idx < nch_tot && !full && pos + 16 > (int32_t)th && pos < (int32_t)tot;
                if (__builtin_amdgcn_ballot_w64(part) != 0) {
                    if (part) chunk_wo_bytes(x, (int64_t)pos - th, (int64_t)(tot - th), odd, w2, o2);
                }
            }
            W += w2;
            O += o2;
        }
        W = group_sum64<G>(W);
        O = odd ? group_sum64<G>(O) : 0;
        const uint64_t ps = ps32;
        uint64_t S = combine(ps, W, O, odd);
        // FILL: the reference sums with check == 0 (context.c:182); TCP+16 is an
        // even relative offset, so its native word contributes exactly check_word.
        if (!verify) S -= check_word;
        d.c = fold_ref(S);
        // IPv4 header checksum = csum_continue(0, ip, ihl*4) with check (IP+10) as
        // zero — the reference's commented-out context.c:179, over ihl*4 bytes.
        uint16_t ic_fill = 0;
        if (iphdr) {
            const uint64_t WI = group_sum64<G>((uint64_t)wi);
            const uint64_t OI = odd ? group_sum64<G>((uint64_t)oi) : 0;
            uint64_t IS = combine(0, WI, OI, odd);
            if (!verify) IS -= h8 >> 16;
            ic_fill = fold_ref(IS);
        }
        d.th = th;
        d.urg = check_dw & 0xffff0000u;
        d.fill = !verify;
        // FILL, line store (store_mode 2, the default): when the 128-B line holding
        // the check (and, with IPHDR, the IPv4 header checksum) lies inside this
        // packet and in the group's first-round registers, the group writes the
        // whole line back — the bytes it read, the checksums patched in — as
        // write-through (sc0 sc1) 16-B stores, instead of 2-byte stores that leave
        // partially dirty lines to be written back later: FILL on 1M x 1500-B
        // packets in 1536-B slots 0.328 -> 0.289 ms (VERIFY 0.246;
        // tools/fill_line_ab.py, profiles/r03_fill_line_ab.jsonl).
        // store_mode 3: the same with the 64-B block holding the checks (half the
        // bytes written; of packed packets more qualify, since a 64-B block inside
        // the packet is found for any start up to 64 B into a 128-B line).
        if ((store_mode == 2 || store_mode == 3) && !verify && amask == 127u && (m & 1u) == 0) {
            const uint32_t cpos = m + th + 16u;   // window offset of the check (even)
            const uint32_t ipos = m + 10u;        // ... of the IPv4 header checksum
            const uint32_t bsz = store_mode == 3 ? 64u : 128u;   // the block written (wave-uniform)
            const uint32_t b0 = cpos & ~(bsz - 1u);               // its window offset
            // Only the group's first round of registers stays live to the store (FILL
            // k_ipv4<8,4,1>: 108 VGPRs with two rounds kept, 102 with one): the block
            // must lie in the group's first G chunks (128 B for G = 8) — for 128-B
            // lines, packets starting on a 128-B boundary — the rest take the 2-byte store
            constexpr uint32_t KB = 16u * (uint32_t)G;
            if (b0 >= m && b0 + bsz <= m + tot && b0 + bsz <= KB && (!iphdr || (ipos & ~(bsz - 1u)) == b0)) {
                auto patch = [](u32x4& x, uint32_t pos, uint32_t v16) {
                    const uint32_t sh = (pos & 2u) * 8u, j = (pos >> 2) & 3u;
                    const uint32_t keep = ~(0xffffu << sh), val = v16 << sh;
                    x.x = j == 0u ? (x.x & keep) | val : x.x;
                    x.y = j == 1u ? (x.y & keep) | val : x.y;
                    x.z = j == 2u ? (x.z & keep) | val : x.z;
                    x.w = j == 3u ? (x.w & keep) | val : x.w;
                };
                const uint32_t idx = (uint32_t)gl;   // this lane's first-round chunk
                if (idx * 16u - b0 < bsz) {
                    u32x4 x = v[u][0];
                    if (idx == (cpos >> 4)) patch(x, cpos, (uint32_t)d.c);
                    if (iphdr && idx == (ipos >> 4)) patch(x, ipos, (uint32_t)ic_fill);
                    uint8_t* dst = ip - m + (uint64_t)idx * 16u;
                    if (region_base)   // wave-uniform: every line of the region is in the window
                        __builtin_amdgcn_raw_buffer_store_b128(
                            x, wt_rsrc, (int)(uint32_t)((uint64_t)(uintptr_t)dst - wt_base), 0, kCpolSc0Sc1);
                    else
                        stg_wt16_at(dst, x, wt_base);
                }
                d.fill = false;   // stored
            }
        }
        uint32_t st = TCPCSUM_PKT_OK;
        if (verify && d.c != 0 && check_word == (uint32_t)(uint16_t)~fold_ref(ps)) st |= TCPCSUM_PKT_CSUM_PARTIAL;
        if (iphdr) {
            d.ic = ic_fill;
            if (verify && d.ic != 0) st |= TCPCSUM_PKT_IPHDR_BAD;
        }
        d.st = (uint8_t)st;
        return d;
    };
    auto commit = [&](const IpDone& d) {
        if (!d.w || gl != 0) return;
        if (d.fill) {
            uint8_t* cp = d.ip + d.th + 16;
            if (store_mode == 1 && ((uintptr_t)cp & 3u) == 0)   // check and the unchanged urg_ptr in one dword
                stg<uint32_t>(cp, d.urg | d.c);
            else if (store_mode >= 2)
                store_u16_wt(cp, d.c);   // native u16 store, as context.c:208, written through
            else
                store_u16(cp, d.c);
            if (iphdr) {
                if (store_mode >= 2) store_u16_wt(d.ip + 10, d.ic);
                else store_u16(d.ip + 10, d.ic);
            }
        }
        if (iphdr && ipout && d.st != TCPCSUM_PKT_SKIPPED) ipout[d.i] = d.ic;
        if (out) out[d.i] = d.c;
        if (status) status[d.i] = d.st;
    };
    load_off(t);
    for (; t < ntiles; t += nwaves) {
        issue(t);
        if constexpr (!VER) {   // converged here: the line stores' base for this tile
            if (!region_base) wt_base = wt_base_near((uint64_t)(uintptr_t)p[0].ip);
        }
        // the next tile's offsets, in flight while this tile is summed
        load_off(t + nwaves);
#pragma unroll
        for (int u = 0; u < U; ++u) commit(process(u, t * SPT + (uint64_t)(u * GPW + q)));
    }
}

// Wire batches, balanced (mixed packet sizes, packed small packets): 64 packets
// per wave tile. Each lane reads its packet's IP header with aligned dword loads
// (fields funnel-shifted out of them: no dynamic register indexing), validates
// it exactly like k_ipv4, and the TCP ranges [ip + ihl*4, ip + tot_len) are
// summed by lb_sums — FILL then subtracts the check word (what zeroing it
// does). The IPv4 header checksum (IPHDR) is summed per lane from the
// header dwords: relative dwords, so its u16 halves are the reference's words.
template <int C, bool PL, bool HD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TCPCSUM_DESC_LB_WAVES, 8))) void k_ipv4_lb(uint8_t* __restrict__ pkts, const uint64_t* __restrict__ off,
                                                 const uint32_t* __restrict__ plen,
                                                 uint64_t n, uint32_t cap, uint64_t limit, int mode,
                                                 uint16_t* __restrict__ out, uint8_t* __restrict__ status,
                                                 uint16_t* __restrict__ ipout, uint32_t spw) {
    // spw: packets per wave tile (1..64; lanes >= spw hold none), as in k_desc_lb
    __shared__ uint64_t acc[4][2][64];
    __shared__ __attribute__((aligned(8))) uint32_t marks[(TCPCSUM_LB_VARIANT & 1) ? 4 : 1][(TCPCSUM_LB_VARIANT & 1) ? 256 : 2];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* mark = marks[(TCPCSUM_LB_VARIANT & 1) ? wv : 0];
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t ntiles = (n + spw - 1) / spw;
    const bool verify = (mode & TCPCSUM_IPV4_VERIFY) != 0;
    const bool iphdr = (mode & TCPCSUM_IPV4_IPHDR) != 0;
    // A tile's packet offsets (and PL lengths), then the header dwords under them: two
    // dependent loads before its sweep. TCPCSUM_LB_VARIANT bit 2: a grid-stride loop that
    // issues tile t + 2's offsets and tile t + 1's header loads before tile t is swept.
    struct Off {
        uint64_t o;
        uint32_t pl;
    };
    auto load_off = [&](uint64_t t) {
        const uint64_t i = t * spw + (uint64_t)lane;
        const bool live = (uint32_t)lane < spw && i < n;
        Off r;
        r.o = ldg<uint64_t>(zsel(live, reinterpret_cast<const uint8_t*>(off + i)));
        r.pl = PL ? ldg<uint32_t>(zsel(live, reinterpret_cast<const uint8_t*>(plen + i))) : 0u;
        return r;
    };
    // the readable bytes at the packet (PL: region end and its own length) and whether the
    // 20-byte header is among them
    auto room_of = [&](uint64_t t, const Off& f, uint32_t& room) {
        const uint64_t i = t * spw + (uint64_t)lane;
        const bool live = (uint32_t)lane < spw && i < n;
        if constexpr (PL) {
            const uint64_t rr = live && f.o < limit ? limit - f.o : 0u;
            room = (uint32_t)(rr < (uint64_t)f.pl ? rr : (uint64_t)f.pl);
            return room >= 20u;
        } else {
            room = 0;
            return live && f.o < limit && limit - f.o >= 20u;
        }
    };
    // the dwords under header bytes [0, 20): D[5] only when ip is not 4-B aligned
    // (an aligned dword holding a needed byte never crosses a page)
    auto load_hdr = [&](uint64_t t, const Off& f, uint32_t (&D)[6]) {
        uint32_t room;
        const bool hdr = room_of(t, f, room);
        const uint8_t* ip = PL ? reinterpret_cast<const uint8_t*>((uintptr_t)pkts + f.o) : pkts + f.o;
        const uint32_t sh = (uint32_t)((uintptr_t)ip & 3u);
        if (TCPCSUM_LB_HDR_X4 && __ballot(hdr && sh != 0) == 0) {
            // 4-B aligned headers: one dwordx4 and one dword load (the 20 bytes are readable)
            const uint8_t* hp = zsel(hdr, ip);
            const u32x4a4 q = *(gptr<const u32x4a4>)(hp);
            D[0] = q.x;
            D[1] = q.y;
            D[2] = q.z;
            D[3] = q.w;
            D[4] = ldg<uint32_t>(hp + 16);
            D[5] = 0;
            return;
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) D[k] = ldg<uint32_t>(zsel(hdr && (k < 5 || sh != 0), ip - sh + 4 * k));
    };
    auto process = [&](uint64_t t, const Off& f, const uint32_t (&D)[6]) {
        const uint64_t i = t * spw + (uint64_t)lane;
        const bool live = (uint32_t)lane < spw && i < n;
        const uint64_t o = f.o;
        uint32_t room;
        const bool hdr = room_of(t, f, room);
        uint8_t* ip = PL ? reinterpret_cast<uint8_t*>((uintptr_t)pkts + o) : pkts + o;
        const uint32_t sh = (uint32_t)((uintptr_t)ip & 3u);
        const uint8_t* d0 = ip - sh;
        auto rel4 = [&](int k) { return __builtin_amdgcn_alignbyte(D[k + 1], D[k], sh); };   // bytes [4k, 4k+4)
        const uint32_t h0 = rel4(0), h8 = rel4(2), sa = rel4(3), da = rel4(4);
        const uint32_t ver = (h0 >> 4) & 15u, ihl = h0 & 15u;
        const uint32_t tot = ((h0 >> 8) & 0xff00u) | (h0 >> 24);
        const uint32_t proto = (h8 >> 8) & 0xffu;
        const bool fits = PL ? tot <= room : o + tot <= limit;
        const bool ok = hdr && ver == 4u && proto == 6u && ihl >= 5u && tot >= ihl * 4u + 20u && tot <= cap && fits;
        const uint32_t th = ihl * 4u;
        const uint32_t len = ok ? tot - th : 0u;
        uint8_t* tcp = ip + th;
        const bool odd = ((uintptr_t)ip & 1u) != 0;   // th is even
        const bool any_odd = __ballot(ok && odd) != 0;
        lb_sums<C>(tcp, len, kNoHole, any_odd, acc[wv][0], acc[wv][1], mark);
        if (!live) return;
        if (!ok) {
            if (out) out[i] = 0;
            if (status) status[i] = TCPCSUM_PKT_SKIPPED;
            return;
        }
        const uint32_t len_be = ((len & 0xffu) << 8) | ((len >> 8) & 0xffu);   // htons
        // context.c:104-119 closed form
        const uint64_t ps = (sa & 0xffffu) + (sa >> 16) + (da & 0xffffu) + (da >> 16) + 0x0600u + len_be;
        uint64_t S = combine(ps, acc[wv][0][lane], any_odd ? acc[wv][1][lane] : 0, odd);
        // FILL sums with the check as zero (context.c:182): TCP+16 is an even offset,
        // so its native word (L2-hot: just summed) contributes exactly its value
        // (taking it from the sweep's registers instead, via LDS, measured slower: flush mix
        // FILL 0.1163 vs 0.1001 ms, VERIFY too, profiles/r06_wire_lb_chk_ab.jsonl)
        if (!verify) S -= (uint32_t)ldg<uint8_t>(tcp + 16) | ((uint32_t)ldg<uint8_t>(tcp + 17) << 8);
        const uint16_t c = fold_ref(S);
        uint32_t st = TCPCSUM_PKT_OK;
        if (verify && c != 0) {   // rare: was the check left as the bare pseudo-header sum?
            const uint32_t cw = (uint32_t)ldg<uint8_t>(tcp + 16) | ((uint32_t)ldg<uint8_t>(tcp + 17) << 8);
            if (cw == (uint32_t)(uint16_t)~fold_ref(ps)) st |= TCPCSUM_PKT_CSUM_PARTIAL;
        }
        if (iphdr) {
            // csum_continue(0, ip, ihl*4) with check (IP+10) as zero: the reference's
            // commented-out context.c:179
            uint32_t w = 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) w = sad16(rel4(k), w);
            for (uint32_t k = 5; k < ihl; ++k) {   // IP options
                const uint32_t lo = ldg<uint32_t>(d0 + 4 * k);
                const uint32_t hi = sh ? ldg<uint32_t>(d0 + 4 * k + 4) : 0u;
                w = sad16(__builtin_amdgcn_alignbyte(hi, lo, sh), w);
            }
            const uint16_t ic = fold_ref((uint64_t)w - (verify ? 0u : (h8 >> 16)));
            if (ipout) ipout[i] = ic;
            if (!verify) store_u16(ip + 10, ic);
            else if (ic != 0) st |= TCPCSUM_PKT_IPHDR_BAD;
        }
        if (!verify) store_u16(tcp + 16, c);   // native u16 store, as context.c:208
        if (out) out[i] = c;
        if (status) status[i] = (uint8_t)st;
    };
    // Tiles whose packets all start 4-B aligned (any real packet buffer), without IPHDR: the
    // packet's first 64 bytes from its 16-B aligned start come in with four 16-B loads — the
    // header fields, the first TCP bytes (a 44-B control segment entirely) and the FILL's
    // check word, all from registers — and only the rest of each segment, from the next 16-B
    // boundary past those 64 bytes, is swept: a control segment never enters the sweep and
    // the check word needs no load of its own. Taken by FILL only (its own instantiation,
    // see the launcher): 2M packed 576-B FILL -12.5 %, flush mix FILL -4 %.
    auto process_head = [&](uint64_t t, const Off& f) {
        const uint64_t i = t * spw + (uint64_t)lane;
        const bool live = (uint32_t)lane < spw && i < n;
        const uint64_t o = f.o;
        uint32_t room;
        const bool hdr = room_of(t, f, room);
        const uint64_t readable = !hdr ? 0u : PL ? (uint64_t)room : limit - o;
        uint8_t* ip = PL ? reinterpret_cast<uint8_t*>((uintptr_t)pkts + o) : pkts + o;
        const uint32_t sh = (uint32_t)((uintptr_t)ip & 15u);   // 0, 4, 8 or 12
        const uint8_t* al = ip - sh;
        u32x4 H[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)   // a 16-B chunk holding a readable byte never crosses a page
            H[k] = ldg<u32x4>(zsel(hdr && 16u * k < sh + readable, al + 16 * k));
        // dword j (0..15) of the 64 loaded bytes: register selects only
        auto dw = [&](uint32_t j) {
            const u32x4 c = j < 4u ? H[0] : j < 8u ? H[1] : j < 12u ? H[2] : H[3];
            const uint32_t r = j & 3u;
            return r == 0u ? c.x : r == 1u ? c.y : r == 2u ? c.z : c.w;
        };
        const uint32_t q = sh >> 2;
        const uint32_t h0 = dw(q), h8 = dw(q + 2u), sa = dw(q + 3u), da = dw(q + 4u);
        const uint32_t ver = (h0 >> 4) & 15u, ihl = h0 & 15u;
        const uint32_t tot = ((h0 >> 8) & 0xff00u) | (h0 >> 24);
        const uint32_t proto = (h8 >> 8) & 0xffu;
        const bool fits = PL ? tot <= room : o + tot <= limit;
        const bool ok = hdr && ver == 4u && proto == 6u && ihl >= 5u && tot >= ihl * 4u + 20u && tot <= cap && fits;
        const uint32_t th = ihl * 4u;
        const uint32_t len = ok ? tot - th : 0u;
        uint8_t* tcp = ip + th;
        // the TCP bytes among the 64 loaded: relative dwords [th / 4, in_regs / 4), the last
        // one cut at tot
        const uint32_t in_regs = 64u - sh;   // bytes of the packet in H
        const uint32_t head_end = ok ? (tot < in_regs ? tot : in_regs) : 0u;
        uint32_t wh = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t rel = 4u * (uint32_t)j - sh;   // wraps for dwords before the packet
            const uint32_t d = j < 4 ? (j == 0 ? H[0].x : j == 1 ? H[0].y : j == 2 ? H[0].z : H[0].w)
                             : j < 8 ? (j == 4 ? H[1].x : j == 5 ? H[1].y : j == 6 ? H[1].z : H[1].w)
                             : j < 12 ? (j == 8 ? H[2].x : j == 9 ? H[2].y : j == 10 ? H[2].z : H[2].w)
                                      : (j == 12 ? H[3].x : j == 13 ? H[3].y : j == 14 ? H[3].z : H[3].w);
            const uint32_t keep = head_end - rel;   // bytes of this dword before head_end
            const uint32_t m = keep >= 4u ? 0xffffffffu : (1u << (8u * keep)) - 1u;
            wh = sad16(rel >= th && rel < head_end ? d & m : 0u, wh);
        }
        const uint32_t len_be = ((len & 0xffu) << 8) | ((len >> 8) & 0xffu);   // htons
        // context.c:104-119 closed form
        const uint32_t ps = (sa & 0xffffu) + (sa >> 16) + (da & 0xffffu) + (da >> 16) + 0x0600u + len_be;
        // the check word (TCP+16, an even offset: its native u16), from the registers when
        // it lies among the loaded bytes — taken before the sweep, so that the 64 loaded bytes
        // are not held across it
        const uint32_t cpos = th + 16u;
        const bool cw_in = cpos + 2u <= in_regs;
        uint32_t cw = dw(q + ((cw_in ? cpos : 0u) >> 2)) & 0xffffu;
        // the rest of the segment, from the first 16-B boundary past the loaded bytes
        const uint32_t bstart = th > in_regs ? th : in_regs;
        const uint32_t blen = ok && tot > bstart ? tot - bstart : 0u;
        lb_sums<C>(ip + bstart, blen, kNoHole, false, acc[wv][0], acc[wv][1], mark);
        if (!live) return;
        if (!ok) {
            if (out) out[i] = 0;
            if (status) status[i] = TCPCSUM_PKT_SKIPPED;
            return;
        }
        if (!cw_in) cw = (uint32_t)ldg<uint8_t>(tcp + 16) | ((uint32_t)ldg<uint8_t>(tcp + 17) << 8);
        uint64_t S = (uint64_t)ps + wh + acc[wv][0][lane];
        if (!verify) S -= cw;   // FILL sums with the check as zero (context.c:182)
        const uint16_t c = fold_ref(S);
        uint32_t st = TCPCSUM_PKT_OK;
        if (verify && c != 0 && cw == (uint32_t)(uint16_t)~fold_ref(ps)) st |= TCPCSUM_PKT_CSUM_PARTIAL;
        if (!verify) store_u16(tcp + 16, c);   // native u16 store, as context.c:208
        if (out) out[i] = c;
        if (status) status[i] = (uint8_t)st;
    };
    // Measured and dropped: a span path sweeping a packed tile as one run of chunks (owners from
    // the offsets alone, the first round's loads issued beside the header loads): parity-exact
    // but flush mix VERIFY 0.119 ms against 0.078, 2M packed 576 B 0.287 against 0.190 — per-dword
    // owner masks and one wave per SIMD less cost more than the latency it hid (commit 976945f,
    // profiles/r06_lb_span_ab.jsonl).
    // block order: XCD order measured 1 % slower on 2M packed 576-B packets
    // (profiles/r05_xcd_kernels_ab.jsonl)
    uint64_t t = (uint64_t)blockIdx.x * 4u + wv;
    if constexpr ((TCPCSUM_LB_VARIANT & 4) == 0) {
        for (; t < ntiles; t += nwaves) {
            const Off f = load_off(t);
            const uint64_t i = t * spw + (uint64_t)lane;
            const bool live = (uint32_t)lane < spw && i < n;
            const uintptr_t ipa = PL ? (uintptr_t)pkts + f.o : (uintptr_t)(pkts + f.o);
            if (HD && __ballot(live && (ipa & 3u) != 0) == 0) {
                process_head(t, f);
                continue;
            }
            uint32_t D[6];
            load_hdr(t, f, D);
            process(t, f, D);
        }
    } else {
        if (t >= ntiles) return;
        Off f1 = load_off(t), f2 = load_off(t + nwaves);   // past the end: zero loads, no packet
        uint32_t D1[6];
        load_hdr(t, f1, D1);
        for (; t < ntiles; t += nwaves) {
            const Off f3 = load_off(t + 2 * nwaves);
            uint32_t D2[6];
            load_hdr(t + nwaves, f2, D2);
            process(t, f1, D1);
            f1 = f2;
            f2 = f3;
#pragma unroll
            for (int k = 0; k < 6; ++k) D1[k] = D2[k];
        }
    }
}

// ---------------------------------------------------------------- tx build
// Device-side context.c:150-213: write the IPv4/TCP packet of each descriptor
// and checksum it in the same pass. Phase 1 (all lanes of the group): the
// payload is copied in 16-byte destination chunks — each lane loads the (at
// most two) aligned 16-B source chunks under its destination chunk and funnel-
// shifts them into place (v_alignbyte), stores the chunk (one dwordx4 store,
// byte stores only at the two ragged ends) and sums it from registers. Phase 2
// (lanes 0..10): the 44 header bytes of context.c:169-206 as 11 dwords, the
// TCP and optional IP checks folded in, stored after the group reduction.
// The 16 bytes at byte offset 4q+r of the 32-byte window A:B (q, r uniform
// per packet): five selected dwords, four v_alignbyte. Register-only — a
// dynamically indexed window array would be placed in scratch.
__device__ __forceinline__ u32x4 funnel16(const u32x4 A, const u32x4 B, int q, uint32_t r) {
    const uint32_t w0 = q == 0 ? A.x : q == 1 ? A.y : q == 2 ? A.z : A.w;
    const uint32_t w1 = q == 0 ? A.y : q == 1 ? A.z : q == 2 ? A.w : B.x;
    const uint32_t w2 = q == 0 ? A.z : q == 1 ? A.w : q == 2 ? B.x : B.y;
    const uint32_t w3 = q == 0 ? A.w : q == 1 ? B.x : q == 2 ? B.y : B.z;
    const uint32_t w4 = q == 0 ? B.x : q == 1 ? B.y : q == 2 ? B.z : B.w;
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(w1, w0, r);
    v.y = __builtin_amdgcn_alignbyte(w2, w1, r);
    v.z = __builtin_amdgcn_alignbyte(w3, w2, r);
    v.w = __builtin_amdgcn_alignbyte(w4, w3, r);
    return v;
}

__device__ __forceinline__ uint32_t sum_halves(uint32_t d) { return (d & 0xffffu) + (d >> 16); }

// One packet of a tile, as decoded from its descriptor.
struct TxPkt {
    const uint8_t* src;     // payload
    const uint8_t* sbase;   // aligned source chunk under destination chunk 0
    uint8_t* ip;            // packet start
    uint8_t* dbase;         // aligned destination chunk holding the first payload byte
    uint32_t sa, da, seq, ack, ports, flags, len;
    uint32_t dm, sh, f0, f1;
    bool live, odd;
};

// the 48-byte record of segment i as three 16-byte loads; dead slots read
// zeros (g_zero is 64 bytes: covers the record)
struct TxRec {
    u32x4 d0, d1, d2;
};

__device__ __forceinline__ TxRec tx_load(const tcpcsum_txseg_t* segs, uint64_t i, uint64_t n) {
    const u32x4* dp = reinterpret_cast<const u32x4*>(zsel(i < n, reinterpret_cast<const uint8_t*>(segs + i)));
    return TxRec{dp[0], dp[1], dp[2]};
}

__device__ __forceinline__ void tx_decode(TxPkt& p, const TxRec& r, bool live, const uint8_t* payload,
                                          uint8_t* outp) {
    p.live = live;
    const u32x4 d0 = r.d0, d1 = r.d1, d2 = r.d2;
    const uint64_t payload_off = (uint64_t)d0.x | ((uint64_t)d0.y << 32);
    const uint64_t out_off = (uint64_t)d0.z | ((uint64_t)d0.w << 32);
    p.sa = d1.x; p.da = d1.y; p.seq = d1.z; p.ack = d1.w;
    p.ports = d2.x;
    p.flags = (d2.y >> 16) & 0xffu;
    p.len = (p.flags & TCPCSUM_TXF_DATA) ? (d2.y & 0xffffu) : 0u;
    if (p.len > 65491u) p.live = false;   // not written (d_check = 0)
    p.ip = outp + out_off;
    p.src = payload + payload_off;
    uint8_t* dst = p.ip + 44;
    p.odd = ((uintptr_t)p.ip & 1u) != 0;   // parity of the TCP start (ip + 20)
    p.dm = (uint32_t)((uintptr_t)dst & 15u);
    p.dbase = dst - p.dm;
    p.sh = (uint32_t)(((uintptr_t)p.src - p.dm) & 15u);
    // derived from the argument pointer (not an integer): keeps global_ loads
    p.sbase = p.src - (int64_t)(p.dm + p.sh);
    // destination chunks entirely inside the payload: [f0, f1)
    p.f0 = p.dm ? 1u : 0u;
    p.f1 = (p.dm + p.len) >> 4;
    if (!p.live) { p.len = 0; p.f0 = 0; p.f1 = 0; }
}

// chunk e of the packet's ragged ends for lane gl: 0 = head (lane 0), 1 = tail (lane 1); -1 none
__device__ __forceinline__ int tx_edge_chunk(const TxPkt& p, int gl) {
    if (!p.len || gl > 1) return -1;
    const bool head = p.dm != 0;
    const bool tail = ((p.dm + p.len) & 15u) != 0 && p.f1 >= p.f0 && !(head && p.f1 == 0);
    if (gl == 0) return head ? 0 : -1;
    return tail ? (int)p.f1 : -1;
}

__device__ __forceinline__ void tx_edge_load(const TxPkt& p, int e, u32x4& A, u32x4& B) {
    A = u32x4{0u, 0u, 0u, 0u};
    B = A;
    if (e < 0) return;
    const uint8_t* a = p.sbase + (uint64_t)e * 16u;
    const uintptr_t lo = (uintptr_t)p.src, hi = (uintptr_t)p.src + p.len;
    if ((uintptr_t)a < hi && (uintptr_t)a + 16 > lo) A = ld16(a);
    if (p.sh != 0 && (uintptr_t)a + 16 < hi && (uintptr_t)a + 32 > lo) B = ld16(a + 16);   // rare: ragged ends only
}

// Source chunk idx + 1 for lane gl's load k of a round (lane gl loads chunk
// base + k*G + gl): lane gl + 1's chunk of the same load, or for the group's
// last lane lane 0's chunk of load k + 1 — lane 0 offers that one instead of
// its own, which no lane of its group reads — or, after the round's last load,
// the chunk the last lane read itself (bl). Every lane runs the bpermutes (no
// divergence around them); unused when the packet needs no shift.
template <int G, int C>
__device__ __forceinline__ u32x4 tx_next_chunk(const u32x4 (&a)[C], int k, const u32x4 bl, int lane, int gl) {
    if constexpr ((TCPCSUM_TX_KNOCKOUT & 4) != 0) return a[k];
    const u32x4 x = (gl == 0 && k + 1 < C) ? a[k + 1 < C ? k + 1 : k] : a[k];
    const uint32_t src = (uint32_t)(gl < G - 1 ? lane + 1 : lane - (G - 1));
    u32x4 b;
    b.x = bperm(x.x, src);
    b.y = bperm(x.y, src);
    b.z = bperm(x.z, src);
    b.w = bperm(x.w, src);
    return (gl == G - 1 && k == C - 1) ? bl : b;
}

// Phase 1 for a full chunk already loaded: shift into place, store, sum.
// SP: store policy — 0 default (write-back in L2), 1 non-temporal, 2 written
// through (sc0 sc1, stg_wt16).
template <int SP>
__device__ __forceinline__ void tx_full_chunk(const TxPkt& p, uint32_t idx, const u32x4 A, const u32x4 B,
                                              uint32_t& wsum, uint32_t& osum) {
    const u32x4 v = funnel16(A, B, (int)(p.sh >> 2), p.sh & 3u);
    u32x4* d = reinterpret_cast<u32x4*>(p.dbase + (uint64_t)idx * 16u);
    if constexpr ((TCPCSUM_TX_KNOCKOUT & 8) != 0) {
    } else if constexpr (SP == 1) {
        __builtin_nontemporal_store(v, d);
    } else if constexpr (SP == 2) {
        stg_wt16(reinterpret_cast<uint8_t*>(d), v);
    } else {
        *d = v;
    }
    wsum = sad16(v.x, wsum); wsum = sad16(v.y, wsum);
    wsum = sad16(v.z, wsum); wsum = sad16(v.w, wsum);
    if (p.odd) {
        osum = sad8(v.x & 0xff00ff00u, osum); osum = sad8(v.y & 0xff00ff00u, osum);
        osum = sad8(v.z & 0xff00ff00u, osum); osum = sad8(v.w & 0xff00ff00u, osum);
    }
}

// Bytes [b0, b1) of the 16-byte chunk v to the 16-B aligned dc, in naturally
// aligned power-of-two pieces: rising from b0 (1, 2, 4, 8 bytes while the
// offset has that bit set), then falling (8, 4, 2, 1 while they fit) — at
// most eight store instructions for any range, instead of one per byte.
__device__ __forceinline__ void store_range16(uint8_t* dc, const u32x4 v, uint32_t b0, uint32_t b1) {
    auto dw = [&](uint32_t i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; };
    auto at = [&](uint32_t o) { return dw(o >> 2) >> (8u * (o & 3u)); };   // bytes from offset o (within its dword)
    uint32_t x = b0;
    if ((x & 1u) && x + 1u <= b1) { stg<uint8_t>(dc + x, (uint8_t)at(x)); x += 1u; }
    if ((x & 2u) && x + 2u <= b1) { stg<uint16_t>(dc + x, (uint16_t)at(x)); x += 2u; }
    if ((x & 4u) && x + 4u <= b1) { stg<uint32_t>(dc + x, dw(x >> 2)); x += 4u; }
    if ((x & 8u) && x + 8u <= b1) { stg<uint64_t>(dc + x, (uint64_t)v.z | ((uint64_t)v.w << 32)); x += 8u; }
    if (x + 8u <= b1) { stg<uint64_t>(dc + x, (uint64_t)v.x | ((uint64_t)v.y << 32)); x += 8u; }   // x == 0
    if (x + 4u <= b1) { stg<uint32_t>(dc + x, dw(x >> 2)); x += 4u; }
    if (x + 2u <= b1) { stg<uint16_t>(dc + x, (uint16_t)at(x)); x += 2u; }
    if (x + 1u <= b1) stg<uint8_t>(dc + x, (uint8_t)at(x));
}

// Ragged end: the payload bytes of chunk e stored, and summed.
__device__ __forceinline__ void tx_edge_chunk_store(const TxPkt& p, int e, const u32x4 A, const u32x4 B,
                                                    uint32_t& wsum, uint32_t& osum) {
    const u32x4 v = funnel16(A, B, (int)(p.sh >> 2), p.sh & 3u);
    const int64_t rel = (int64_t)e * 16 - (int64_t)p.dm;   // dest chunk start - first payload byte
    uint8_t* dc = p.dbase + (uint64_t)e * 16u;
    const int64_t lo = rel < 0 ? -rel : 0, hi = (int64_t)p.len - rel < 16 ? (int64_t)p.len - rel : 16;
    if (!(TCPCSUM_TX_KNOCKOUT & 1) && lo < hi) store_range16(dc, v, (uint32_t)lo, (uint32_t)hi);
    chunk_wo_bytes(v, rel, (int64_t)p.len, p.odd, wsum, osum);
}

// Phase 2: header (context.c:169-206) with the checks folded in; lanes store it.
template <int G>
__device__ __forceinline__ void tx_header(const TxPkt& p, uint64_t Spay, int mode, int gl, uint16_t* checks,
                                          uint64_t i) {
    const uint32_t tot = 44u + p.len;
    const uint32_t tcp_len = 24u + p.len;
    const uint32_t len_be = ((tcp_len & 0xffu) << 8) | ((tcp_len >> 8) & 0xffu);
    const uint32_t fl = p.flags;
    const uint32_t tflags = (fl & TCPCSUM_TXF_FIN ? 1u : 0u) | (fl & TCPCSUM_TXF_SYN ? 2u : 0u) |
                            (fl & TCPCSUM_TXF_RST ? 4u : 0u) | (fl & TCPCSUM_TXF_DATA ? 8u : 0u) |
                            (fl & TCPCSUM_TXF_ACK ? 16u : 0u);
    const uint32_t sport = p.ports & 0xffffu, dport = p.ports >> 16;
    uint32_t hd[11];
    hd[0] = 0x45u | ((tot >> 8) << 16) | ((tot & 0xffu) << 24);
    hd[1] = 0u;                                          // id = (u16)htonl(54321) = 0, frag_off 0
    hd[2] = 0xffu | (6u << 8);                           // ttl 255, IPPROTO_TCP, check 0
    hd[3] = p.sa;
    hd[4] = p.da;
    hd[5] = (sport >> 8) | ((sport & 0xffu) << 8) | ((dport >> 8) << 16) | ((dport & 0xffu) << 24);
    hd[6] = __builtin_bswap32(p.seq);
    hd[7] = __builtin_bswap32(p.ack);
    hd[8] = 0x60u | (tflags << 8) | (0x20u << 16);       // doff 6, flags, window 8192 (BE 20 00)
    hd[9] = 0u;                                          // check (below), urg_ptr 0
    hd[10] = 0x00050303u;                                // options 03 03 05 00
    uint64_t S = Spay + (p.sa & 0xffffu) + (p.sa >> 16) + (p.da & 0xffffu) + (p.da >> 16) + 0x0600u + len_be;
#pragma unroll
    for (int k = 5; k < 11; ++k) S += sum_halves(hd[k]);
    const uint16_t c = fold_ref(S);
    hd[9] = c;
    if (mode & TCPCSUM_IPV4_IPHDR) {
        uint32_t is = 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) is += sum_halves(hd[k]);
        hd[2] |= (uint32_t)fold_ref(is) << 16;
    }
    for (int j = gl; j < 11 && !(TCPCSUM_TX_KNOCKOUT & 2); j += G) {   // lane j stores header dword j
        uint32_t v = hd[0];
#pragma unroll
        for (int k = 1; k < 11; ++k) v = j == k ? hd[k] : v;
        uint8_t* hp = p.ip + 4 * j;
        if ((((uintptr_t)p.ip) & 3u) == 0) {
            *reinterpret_cast<uint32_t*>(hp) = v;
        } else {
            hp[0] = (uint8_t)v; hp[1] = (uint8_t)(v >> 8); hp[2] = (uint8_t)(v >> 16); hp[3] = (uint8_t)(v >> 24);
        }
    }
    if (gl == 0 && checks) checks[i] = c;
}

// Tile of (64/G)*U packets per wave: U packets per lane group in flight. All
// descriptor loads, then all payload loads (bulk chunks and both ragged ends)
// of the tile are issued before any is consumed. Payloads with more full
// chunks than G*C take extra (un-overlapped) rounds.
template <int G, int C, int U, int SP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TCPCSUM_TX_WAVES, 8))) void k_tx_build(const uint8_t* __restrict__ payload,
                                                  const tcpcsum_txseg_t* __restrict__ segs, uint64_t n,
                                                  uint8_t* __restrict__ outp, int mode,
                                                  uint16_t* __restrict__ checks) {
    constexpr int GPW = 64 / G;
    constexpr int SPT = GPW * U;
    const int lane = threadIdx.x & 63;
    const int q0 = lane / G, gl = lane % G;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t ntiles = (n + SPT - 1) / SPT;
    // block order: its 32768-workgroup loop beats one tile per wave in XCD order by 1-13 %
    // (200 B .. 3000 B payloads, interleaved; profiles/r05_tx_grid_ab.jsonl)
    uint64_t t = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    TxRec rn[U];
#pragma unroll
    for (int u = 0; u < U; ++u) rn[u] = tx_load(segs, t * SPT + (uint64_t)(u * GPW + q0), n);
    for (; t < ntiles; t += nwaves) {
        TxPkt p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = t * SPT + (uint64_t)(u * GPW + q0);
            tx_decode(p[u], rn[u], i < n, payload, outp);
        }
        // Source chunk idx + 1 (the upper half of a shifted destination chunk) is
        // the next lane's chunk idx' = idx + 1 of the same load: it comes over
        // from that lane (ds_bpermute), not from a second load of the same bytes —
        // the group's last lane takes lane 0's chunk of the next load, and only at
        // the round's last load does it read one chunk itself (Bl).
        u32x4 A[U][C], Bl[U], EA[U], EB[U];
        int e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int k = 0; k < C; ++k) {   // full chunks, and chunk f1 when the last one needs it
                const uint32_t idx = p[u].f0 + (uint32_t)(k * G + gl);
                const bool need = idx < p[u].f1 || (idx == p[u].f1 && p[u].sh && p[u].f1 > p[u].f0);
                A[u][k] = ld16(zsel(need, p[u].sbase + (uint64_t)idx * 16u));
            }
            const uint32_t il = p[u].f0 + (uint32_t)((C - 1) * G + gl);
            Bl[u] = ld16(zsel(gl == G - 1 && il < p[u].f1 && p[u].sh, p[u].sbase + (uint64_t)il * 16u + 16u));
            e[u] = tx_edge_chunk(p[u], gl);
            tx_edge_load(p[u], e[u], EA[u], EB[u]);
        }
        // the next tile's records, in flight while this tile is built
#pragma unroll
        for (int u = 0; u < U; ++u) rn[u] = tx_load(segs, (t + nwaves) * SPT + (uint64_t)(u * GPW + q0), n);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t wsum = 0, osum = 0;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint32_t idx = p[u].f0 + (uint32_t)(k * G + gl);
                const u32x4 B = tx_next_chunk<G, C>(A[u], k, Bl[u], lane, gl);
                if (idx < p[u].f1) tx_full_chunk<SP>(p[u], idx, A[u][k], B, wsum, osum);
            }
            uint64_t W = wsum, O = osum;
            // long payloads: further rounds of G*C full chunks
            for (uint32_t rr = p[u].f0 + (uint32_t)(G * C); rr < p[u].f1; rr += (uint32_t)(G * C)) {
                u32x4 a2[C];
#pragma unroll
                for (int k = 0; k < C; ++k) {
                    const uint32_t idx = rr + (uint32_t)(k * G + gl);
                    const bool need = idx < p[u].f1 || (idx == p[u].f1 && p[u].sh);
                    a2[k] = ld16(zsel(need, p[u].sbase + (uint64_t)idx * 16u));
                }
                const uint32_t il = rr + (uint32_t)((C - 1) * G + gl);
                const u32x4 bl = ld16(zsel(gl == G - 1 && il < p[u].f1 && p[u].sh, p[u].sbase + (uint64_t)il * 16u + 16u));
                uint32_t ws = 0, os = 0;
#pragma unroll
                for (int k = 0; k < C; ++k) {
                    const uint32_t idx = rr + (uint32_t)(k * G + gl);
                    const u32x4 B = tx_next_chunk<G, C>(a2, k, bl, lane, gl);
                    if (idx < p[u].f1) tx_full_chunk<SP>(p[u], idx, a2[k], B, ws, os);
                }
                W += ws;
                O += os;
            }
            if (e[u] >= 0) {
                uint32_t ws = 0, os = 0;
                tx_edge_chunk_store(p[u], e[u], EA[u], EB[u], ws, os);
                W += ws;
                O += os;
            }
            W = group_sum64<G>(W);
            O = p[u].odd ? group_sum64<G>(O) : 0;
            const uint64_t i = t * SPT + (uint64_t)(u * GPW + q0);
            if (p[u].live) {
                tx_header<G>(p[u], combine(0, W, O, p[u].odd), mode, gl, checks, i);
            } else if (i < n && gl == 0 && checks) {
                checks[i] = 0;
            }
        }
    }
}

// ---------------------------------------------------------------- synthetic
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// SURVEY.md Appendix B stream: byte b = byte (b % 8) of mix(SEED + (b/8 + 1) * gamma).
__global__ __launch_bounds__(256) void k_synth_fill(uint8_t* __restrict__ dst, uint64_t off, uint64_t nbytes) {
    const uint64_t w0 = off >> 3, w1 = (off + nbytes + 7) >> 3;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = w0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < w1; w += nthr) {
        const uint64_t v = mix64(0x5EEDC0DEull + (w + 1) * 0x9E3779B97F4A7C15ull);
        const uint64_t b0 = w << 3;
        uint8_t* d = dst + (int64_t)(b0 - off);
        if (b0 >= off && b0 + 8 <= off + nbytes && (((uintptr_t)d) & 7u) == 0) {
            *reinterpret_cast<uint64_t*>(d) = v;
        } else {
            for (int k = 0; k < 8; ++k) {
                const uint64_t b = b0 + k;
                if (b >= off && b < off + nbytes) dst[b - off] = (uint8_t)(v >> (8 * k));
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_synth_pseudo(uint32_t* __restrict__ ss, uint64_t seg0, uint64_t n,
                                                      uint32_t len_be) {
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += nthr) {
        const uint64_t i = seg0 + k;
        const uint32_t sa = __builtin_bswap32(0x0A000000u | (uint32_t)(i & 0xFFFFFFu));
        const uint32_t da = __builtin_bswap32(0xC0A80000u | (uint32_t)((i * 7u) & 0xFFFFu));
        ss[k] = (sa & 0xffffu) + (sa >> 16) + (da & 0xffffu) + (da >> 16) + 0x0600u + len_be;
    }
}

// ---------------------------------------------------------------- probe
// Read-only stream with the checksum kernels' access shape (each wave reads
// contiguous 1 KiB per load instruction, C in flight per lane; by default one
// 4 KiB tile per wave in XCD order, as the uniform kernel's plan), summed so it
// cannot be dead-code eliminated. Each wave adds its partial into slot
// wave % kProbeSlots (one atomic per wave, spread over the slots — 2048
// same-address atomics would cost ~25 us on this chip).
//
// WR (TCPCSUM_TUNE_PROBE_WRITE): also write back, through (sc0 sc1, as the wire
// FILL's line store), every `period`-th 128-B line it read — the bytes unchanged.
// With period 12 over 1536-B slots that is the wire FILL's HBM traffic (every line
// read, one whole line written per packet) without its arithmetic: the ceiling the
// FILL is held to.
// G: lanes per group — a group reads its own contiguous C x G x 16 bytes, G x 16 per
// instruction (G = 64: one contiguous 1 KiB per instruction; G = 32: two 512-B pieces,
// as the uniform kernel's (32, C) lane groups read two segments)
template <int C, bool WR, int G = 64>
__global__ __launch_bounds__(256) void k_probe(const uint8_t* __restrict__ src, uint64_t nchunks,
                                               uint64_t* __restrict__ partials, uint32_t period) {
    const int lane = threadIdx.x & 63;
    const int q = lane / G, gl = lane % G;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t ntiles = (nchunks + 64 * C - 1) / (64 * C);
    uint64_t acc = 0;
    for (uint64_t t = xcd_block((ntiles + 3) / 4) * 4u + (threadIdx.x >> 6); t < ntiles; t += nwaves) {
        u32x4 v[C];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint64_t idx = t * (64 * C) + (uint64_t)(q * G * C + k * G + gl);
            v[k] = idx < nchunks ? ld16(src + idx * 16u) : u32x4{0u, 0u, 0u, 0u};
        }
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < C; ++k) w += chunk_w<M16>(v[k], 0u, 0u);
        acc += w;
        if constexpr (WR) {
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint64_t idx = t * (64 * C) + (uint64_t)(q * G * C + k * G + gl);
                if (idx < nchunks && (idx >> 3) % period == 0u)
                    stg_wt16_at(const_cast<uint8_t*>(src) + idx * 16u, v[k], (uint64_t)(uintptr_t)src);
            }
        }
    }
    // each wave adds its own partial (no workgroup barrier: a wave retires as soon as its
    // tile is summed, as the checksum kernels' waves do) into slot wave % kProbeSlots
    acc = group_sum64<64>(acc);
    if (lane == 0)
        atomicAdd((unsigned long long*)&partials[((uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6)) % (uint64_t)kProbeSlots],
                  (unsigned long long)acc);
}

}  // namespace tcpcsum

// ============================================================== launchers
using namespace tcpcsum;

namespace {

// HIP bounds a launch at gridDim.x * blockDim.x < 2^32 threads: with 256-thread
// workgroups at most 2^24 - 1 of them (the kernels grid-stride past that).
constexpr uint64_t kMaxGrid = (1u << 24) - 1u;

// A grid that covers the work is rounded up to whole XCD rounds, so the kernels can take
// their tiles XCD by XCD (xcd_block): at most 7 idle workgroups.
inline uint64_t xcd_rounds(uint64_t blocks) {
    return (blocks + 7u) & ~(uint64_t)7u;
}

inline unsigned grid_for(uint64_t waves_needed, int max_blocks) {
    uint64_t blocks = (waves_needed + 3) / 4;
    if (blocks < 1) blocks = 1;
    if (blocks < (uint64_t)max_blocks) blocks = xcd_rounds(blocks);
    if (blocks > (uint64_t)max_blocks) blocks = (uint64_t)max_blocks;
    if (blocks > kMaxGrid) blocks = kMaxGrid;
    return (unsigned)blocks;
}

template <int G, int C, int U, int MODE, bool PIPE, bool NT>
void launch_uniform_t(const uint8_t* base, uint64_t stride, uint32_t len, const uint32_t* ss,
                      uint32_t ss0, uint16_t* out, uint64_t n, hipStream_t s, int max_blocks, int blocked) {
    // VGPR budget: at most 32 chunk quads per lane (16 per buffer when pipelined)
    constexpr int LIM = PIPE ? 16 : 32;
    constexpr int UE = (C * U > LIM) ? (LIM / C > 0 ? LIM / C : 1) : U;
    constexpr int SPT = (64 / G) * UE;
    const uint64_t ntiles = (n + SPT - 1) / SPT;
    // grid_for counts four waves per workgroup; TCPCSUM_UNIFORM_WPB (measurement builds) other sizes
    const uint64_t waves = TCPCSUM_UNIFORM_WPB == 4 ? ntiles : (ntiles * 4u + TCPCSUM_UNIFORM_WPB - 1) / TCPCSUM_UNIFORM_WPB;
    hipLaunchKernelGGL((k_uniform<G, C, UE, MODE, PIPE, NT>), dim3(grid_for(waves, max_blocks)),
                       dim3(64 * TCPCSUM_UNIFORM_WPB), 0, s, base, stride, len, ss, ss0, out, n, blocked);
}

template <int C, int MODE, bool PIPE, bool NT>
void launch_long_t(const uint8_t* base, uint64_t stride, uint32_t len, const uint32_t* ss, uint32_t ss0,
                   uint16_t* out, uint64_t n, hipStream_t s, int max_blocks) {
    // rounds per segment: enough for the worst start alignment in the batch
    uint64_t nch = 0;
    for (uint64_t i = 0; i < 16 && i < n; ++i) {
        const uint64_t c = ((((uintptr_t)base + i * stride) & 15u) + len + 15u) >> 4;
        if (c > nch) nch = c;
    }
    const uint32_t rounds = (uint32_t)((nch + 64u * C - 1) / (64u * C));
    if (rounds == 0) return;
    hipLaunchKernelGGL((k_uniform_long<C, MODE, PIPE, NT>), dim3(grid_for(n, max_blocks)), dim3(256), 0, s, base,
                       stride, len, rounds, ss, ss0, out, n);
}

// split segments: unroll selects C = 4 * unroll chunk loads per thread per round,
// halved while half of it still covers the segment in one round
template <int MODE>
void launch_split(const uint8_t* base, uint64_t stride, uint32_t len, const uint32_t* ss, uint32_t ss0,
                  uint16_t* out, uint64_t n, hipStream_t s, int max_blocks, int unroll) {
    uint64_t nch = 0;
    for (uint64_t i = 0; i < 16 && i < n; ++i) {
        const uint64_t c = ((((uintptr_t)base + i * stride) & 15u) + len + 15u) >> 4;
        if (c > nch) nch = c;
    }
    if (nch == 0) return;
    int C = unroll <= 1 ? 4 : unroll == 2 ? 8 : unroll == 4 ? 16 : 32;
    while (C > 4 && 256u * (uint64_t)(C / 2) >= nch) C /= 2;
    const uint32_t rounds = (uint32_t)((nch + 256u * C - 1) / (256u * C));
    uint64_t gb = n < (uint64_t)max_blocks ? xcd_rounds(n) : (uint64_t)max_blocks;
    if (gb > (uint64_t)max_blocks) gb = (uint64_t)max_blocks;
    if (gb > kMaxGrid) gb = kMaxGrid;
    const unsigned g = (unsigned)gb;
#define TC_S(CC)                                                                                             \
    hipLaunchKernelGGL((k_uniform_split<CC, MODE>), dim3(g), dim3(256), 0, s, base, stride, len, rounds, ss, \
                       ss0, out, n)
    if (C == 4) TC_S(4);
    else if (C == 8) TC_S(8);
    else if (C == 16) TC_S(16);
    else TC_S(32);
#undef TC_S
}

// a workgroup per segment (shape 14): unroll selects (waves per workgroup, loads per lane per
// round) = 1: one 4 KiB tile per wave, as many waves as the segment fills — (16, 4) past
// 32 KiB, (8, 4) past 16 KiB, else (4, 4); 2: (8, 8); 4: (16, 2); 8: (4, 16). The grid
// covers the batch in whole XCD rounds (segments XCD by XCD) unless max_blocks caps it.
template <int MODE>
void launch_wg(const uint8_t* base, uint64_t stride, uint32_t len, const uint32_t* ss, uint32_t ss0,
               uint16_t* out, uint64_t n, hipStream_t s, int max_blocks, int unroll) {
    uint64_t nch = 0;
    for (uint64_t i = 0; i < 16 && i < n; ++i) {
        const uint64_t c = ((((uintptr_t)base + i * stride) & 15u) + len + 15u) >> 4;
        if (c > nch) nch = c;
    }
    if (nch == 0) return;
    uint64_t gb = xcd_rounds(n);
    if (max_blocks > 0 && gb > (uint64_t)max_blocks) gb = (uint64_t)max_blocks;
    if (gb > kMaxGrid) gb = kMaxGrid & ~(uint64_t)7u;
    const unsigned g = (unsigned)gb;
#define TC_W(WPB, CC)                                                                                        \
    hipLaunchKernelGGL((k_uniform_wg<WPB, CC, MODE>), dim3(g), dim3(WPB * 64), 0, s, base, stride, len,      \
                       (uint32_t)((nch + WPB * 64u * CC - 1) / (WPB * 64u * CC)), ss, ss0, out, n)
    if (unroll <= 1) {
        if (nch > 2048u) TC_W(16, 4);
        else if (nch > 1024u) TC_W(8, 4);
        else TC_W(4, 4);
    } else if (unroll == 2) TC_W(8, 8);
    else if (unroll == 4) TC_W(16, 2);
    else TC_W(4, 16);
#undef TC_W
}

// flat tiles: unroll selects C (8 * unroll chunks per lane, 8 KiB * unroll per wave tile)
inline void launch_flat(const uint8_t* base, uint64_t stride, uint32_t len, const uint32_t* ss, uint32_t ss0,
                        uint16_t* out, uint64_t n, hipStream_t s, int max_blocks, int unroll) {
    int C = unroll <= 1 ? 8 : unroll == 2 ? 16 : unroll == 4 ? 24 : 32;
    // a tile must hold at least one segment: (stride + 30) / 16 + 1 <= 64 * C
    while (C < 32 && stride + 46u > (uint64_t)C * 1024u) C += 8;
    uint64_t spt = ((uint64_t)C * 1024u - 46u) / stride;
    if (spt > 64) spt = 64;
    if (spt < 1) spt = 1;
    const uint64_t ntiles = (n + spt - 1) / spt;
    const unsigned g = grid_for(ntiles, max_blocks);
    if (C == 8) hipLaunchKernelGGL(k_flat<8>, dim3(g), dim3(256), 0, s, base, (uint32_t)stride, len, ss, ss0, out, n, (uint32_t)spt);
    else if (C == 16) hipLaunchKernelGGL(k_flat<16>, dim3(g), dim3(256), 0, s, base, (uint32_t)stride, len, ss, ss0, out, n, (uint32_t)spt);
    else if (C == 24) hipLaunchKernelGGL(k_flat<24>, dim3(g), dim3(256), 0, s, base, (uint32_t)stride, len, ss, ss0, out, n, (uint32_t)spt);
    else hipLaunchKernelGGL(k_flat<32>, dim3(g), dim3(256), 0, s, base, (uint32_t)stride, len, ss, ss0, out, n, (uint32_t)spt);
}

template <int MODE, bool PIPE, bool NT>
void launch_uniform_mode(int shape, int unroll, const uint8_t* base, uint64_t stride, uint32_t len,
                         const uint32_t* ss, uint32_t ss0, uint16_t* out, uint64_t n, hipStream_t s,
                         int max_blocks, int blocked) {
#define TC_U(G, C, U) \
    launch_uniform_t<G, C, U, MODE, PIPE, NT>(base, stride, len, ss, ss0, out, n, s, max_blocks, blocked)
#define TC_U4(G, C)                          \
    do {                                     \
        if (unroll == 1) TC_U(G, C, 1);      \
        else if (unroll == 2) TC_U(G, C, 2); \
        else if (unroll == 4) TC_U(G, C, 4); \
        else TC_U(G, C, 8);                  \
    } while (0)
#define TC_L(C) launch_long_t<C, MODE, PIPE, NT>(base, stride, len, ss, ss0, out, n, s, max_blocks)
    switch (shape) {
        case 0: TC_U4(4, 1); break;    // <= 4 chunks   (64 B)
        case 1: TC_U4(8, 1); break;    // <= 8
        case 2: TC_U4(16, 1); break;   // <= 16
        case 3: TC_U4(32, 1); break;   // <= 32
        case 4: TC_U4(64, 1); break;   // <= 64
        case 5: TC_U4(32, 3); break;   // <= 96         (1500 B)
        case 6: TC_U4(64, 2); break;   // <= 128
        case 7: TC_U4(64, 4); break;   // <= 256
        case 8: TC_U4(64, 8); break;   // <= 512
        case 12: launch_flat(base, stride, len, ss, ss0, out, n, s, max_blocks, unroll); break;
        case 13: launch_split<MODE>(base, stride, len, ss, ss0, out, n, s, max_blocks, unroll); break;
        case 14:
            if constexpr (MODE != M1) launch_wg<MODE>(base, stride, len, ss, ss0, out, n, s, max_blocks, unroll);
            break;
        case 10: TC_U4(1, 5); break;   // <= 5: one lane per segment, no cross-lane reduction
        case 11: TC_U4(2, 4); break;   // <= 8: two lanes per segment
        default:                       // one wave per segment, 8*unroll chunks per lane per round
            if (unroll <= 1) TC_L(8);
            else if (unroll == 2 || PIPE) TC_L(16);
            else TC_L(32);
    }
#undef TC_L
#undef TC_U4
#undef TC_U
}

}  // namespace

namespace tcpcsum {

// Segment-group shapes: shape k covers up to kShapeChunks[k] 16-B chunks per
// segment. Defaults per shape (measured on MI355X, tools/sweep.py; see
// DESIGN.md): segments-in-flight per group and the resident grid — for the
// lane-group shapes 0..8 only where the tile plan in plan_uniform does not
// apply (byte-granular batches; forced max_blocks).
// Shapes 10/11 are the thin lane groups (1 or 2 lanes per segment) for tiny
// segments; shape 9 (one wave per segment) has no chunk limit.
// Shape 12 is the flat tile (segments of 1 KiB .. 32 KiB, 4-byte aligned, stride
// >= len), only used when forced or when kFlatAuto says so.
// Shape 13 is the split segment (a workgroup of four waves per segment, no chunk limit).
static const uint32_t kShapeChunks[15] = {4, 8, 16, 32, 64, 96, 128, 256, 512, 0xffffffffu, 5, 8, 2048, 0xffffffffu,
                                         0xffffffffu};
static const int kShapeUnroll[15] = {4, 8, 8, 8, 8, 8, 8, 8, 4, 2, 2, 2, 2, 2, 1};
static const int kShapeBlocks[15] = {4096, 512, 4096, 4096, 4096, 512, 4096, 1024, 2048, 256, 2048, 2048, 512, 1 << 24,
                                     1 << 24};
static const bool kShapePipe[15] = {false, false, false, false, false, false, false, false, false, false, false, false,
                                    false, false, false};
static const bool kShapeNt[15] = {true, true, true, true, true, true, true, true, true, true, true, true, true, true, true};

static bool flat_ok(uintptr_t b, uint64_t stride, uint32_t len, int mode) {
    return mode != M1 && stride >= 1024 && stride >= len && stride + 46u <= 32u * 1024u && len >= 1024 &&
           (b & 3u) == 0;
}

UniformPlan plan_uniform(uintptr_t b, uint64_t stride, uint32_t len, uint64_t n, const Tuning& tu) {
    UniformPlan p;
    p.mode = (((b | stride | len) & 15u) == 0) ? M16 : (((b | stride | len) & 3u) == 0) ? M4 : M1;
    // The chunks a segment touches depend on its start mod 16, which repeats
    // with period <= 16 over i: take the max over one period.
    uint64_t nch = 0;
    for (uint64_t i = 0; i < 16 && i < n; ++i) {
        const uint64_t m = (b + i * stride) & 15u;
        const uint64_t c = (m + len + 15u) >> 4;
        if (c > nch) nch = c;
    }
    p.shape = 9;
    for (int k = 0; k < 9; ++k)
        if (nch <= kShapeChunks[k]) { p.shape = k; break; }
    // Segments past 8 KiB, dword or chunk aligned: four waves per segment
    // (split) beat one wave per segment on MI355X — 9000 B -2 %, 12300 B -4 %,
    // 20004 B -6 %, 24 KiB -7 %, 48-128 KiB -2..-7 %, the 64 KiB config even
    // (profiles/r02_split_sweep.jsonl). Byte-granular segments keep one wave per
    // segment: their byte masks make the split VALU-bound (12301 B +30 %).
    // Multi-GiB batches of 64 KiB+ chunk-aligned segments keep the resident
    // one-wave-per-segment grid: 256K x 64 KiB 2.392-2.398 vs 2.405-2.408 ms
    // split, three same-process runs (profiles/r02_k64_check.jsonl).
    const bool huge = p.mode == M16 && len >= 65536u && (double)n * len >= 4.0 * (1u << 30);
    if (p.shape == 9 && p.mode != M1 && !huge) p.shape = 13;
    // Dword- or chunk-aligned segments past 32 KiB up to 128 KiB: a workgroup per segment,
    // one 4 KiB tile per wave (16 waves), segments XCD by XCD (shape 14) — the headline's tile
    // plan. Same process against the plan before it (split / resident one-wave grid), ~1.5 GB
    // batches: 48 KiB -2.6 %, 64 KiB -3.3 %, 128 KiB -1.5 %; the 16 GiB 64 KiB config 2.279 vs
    // 2.393 ms (-4.8 %) (profiles/r06_sweeplens.jsonl, r06_sweep64k.jsonl). At 12-32 KiB it was
    // within +-2.5 % either way and 256 KiB even, so those keep theirs.
    if (p.mode != M1 && nch > 2048u && nch <= 8193u) p.shape = 14;
    // 8 KiB chunk-aligned segments (exactly 512 chunks): the split is 9 % ahead of
    // (64,8) (0.208 vs 0.228 ms per 1.5 GB); 6.4-8 KiB otherwise within 2 % of the
    // best shape (tools/uniform_size_sweep*.sh, profiles/r02_uniform_size_sweep.jsonl)
    if (p.shape == 8 && p.mode == M16 && nch == 512) p.shape = 13;
    // a forced shape is honoured only if it covers the segment
    if (tu.shape == 12) {
        if (flat_ok(b, stride, len, p.mode)) p.shape = 12;
    } else if (tu.shape == 14) {
        if (p.mode != M1) p.shape = 14;
    } else if (tu.shape >= 0 && tu.shape <= 13 && nch <= kShapeChunks[tu.shape]) {
        p.shape = tu.shape;
    }
    p.unroll = tu.unroll ? tu.unroll : kShapeUnroll[p.shape];
    p.max_blocks = tu.max_blocks > 0 ? tu.max_blocks : kShapeBlocks[p.shape];
    // Byte-granular batches (odd starts or lengths) spend ~3x the VALU per chunk
    // on byte masks and odd-byte sums: more, shallower waves hide it better —
    // 16384 workgroups, at most 4 segments in flight per group (swept on MI355X at
    // 99, 577, 1499, 3001 and 8191 B: 6-25 % faster than the aligned shapes'
    // defaults with 4096 workgroups, profiles/r02_sweep_m1.jsonl; 16384 a further
    // 1-5 %, profiles/r02_grid_m1.jsonl)
    if (p.mode == M1) {
        if (!tu.unroll && p.shape != 9 && p.unroll > 4) p.unroll = 4;
        // (one tile per wave in XCD order, as below, loses here: 99 B +8 %, 577 B +11 %,
        // 1499 / 3001 B +1 %, profiles/r05_plan_ab.jsonl)
        if (tu.max_blocks <= 0) p.max_blocks = 16384;
    } else if (p.shape <= 8 && tu.max_blocks <= 0) {
        // Lane-group shapes, 4-B aligned: one tile per wave (no grid-stride loop), the
        // tiles taken XCD by XCD (k_uniform), and a tile of at most ~4.5 KiB of the
        // batch — the most segments in flight per group (1..8) whose span fits. Under
        // the XCD order smaller tiles stream faster; a sweep of every unroll and grid at
        // ten sizes picked exactly this tile (profiles/r05_tile_sweep_xcd.jsonl), and
        // against the round-5 plan before it (eight in flight; 1024 looping workgroups
        // for 64 B), same process: 1M x 1500 B 0.2189 -> 0.2089 ms, 64 B -3 %, 128 B
        // -2 %, 256 B -4 %, 512 / 1024 B -3 %, 2048 / 3000 B -7 %, 4096 B -4 %, 6000 B -3 %
        // (profiles/r05_plan_ab.jsonl). Before the XCD order, eight in flight won
        // (profiles/r02_grid_sweep.jsonl).
        p.max_blocks = 1 << 24;
        if (!tu.unroll) {
            static const uint32_t kGroupsPerWave[9] = {16, 8, 4, 2, 1, 2, 1, 1, 1};
            const uint64_t span = (uint64_t)kGroupsPerWave[p.shape] * (stride > len ? stride : len);
            int u = 8;
            while (u > 1 && span * (uint64_t)u > 4608u) u >>= 1;
            p.unroll = u;
        }
    } else if (p.shape == 9 && tu.max_blocks <= 0 && (p.mode != M16 || len < 12288u)) {
        // one wave per segment: segments of one round (jumbo frames, 8-12 KiB)
        // and the dword-masked path want more waves than the 64 KiB config's
        // grid — one segment per wave, no loop (9000 B: 0.356 -> 0.234 ms at 1024
        // workgroups, 0.225 uncapped; 12300 B: 0.323 -> 0.242 -> 0.224; 20004 B
        // 0.239 -> 0.228; 16-64 KiB aligned keep 256; profiles/r02_sweep_long.jsonl,
        // r02_grid_long.jsonl)
        p.max_blocks = 1 << 24;
    }
    p.pipe = tu.flags & TCPCSUM_TUNE_PIPE_ON ? true : tu.flags & TCPCSUM_TUNE_PIPE_OFF ? false : kShapePipe[p.shape];
    p.nt = tu.flags & TCPCSUM_TUNE_NT_ON ? true : tu.flags & TCPCSUM_TUNE_NT_OFF ? false : kShapeNt[p.shape];
    p.blocked = (tu.flags & TCPCSUM_TUNE_BLOCKED) ? 1 : 0;
    return p;
}

template <bool PIPE, bool NT>
static void launch_uniform_pn(const UniformPlan& p, const uint8_t* base, uint64_t stride, uint32_t len,
                              const uint32_t* ss, uint32_t ss0, uint16_t* out, uint64_t n, hipStream_t s) {
    if (p.mode == M16)
        launch_uniform_mode<M16, PIPE, NT>(p.shape, p.unroll, base, stride, len, ss, ss0, out, n, s, p.max_blocks,
                                           p.blocked);
    else if (p.mode == M4)
        launch_uniform_mode<M4, PIPE, NT>(p.shape, p.unroll, base, stride, len, ss, ss0, out, n, s, p.max_blocks,
                                          p.blocked);
    else
        launch_uniform_mode<M1, PIPE, NT>(p.shape, p.unroll, base, stride, len, ss, ss0, out, n, s, p.max_blocks,
                                          p.blocked);
}

void launch_uniform(const uint8_t* base, uint64_t stride, uint32_t len, const uint32_t* ss, uint32_t ss0,
                    uint16_t* out, uint64_t n, hipStream_t s, const Tuning& tu) {
    const UniformPlan p = plan_uniform((uintptr_t)base, stride, len, n, tu);
#if TCPCSUM_TUNING_VARIANTS
    // experiment build: software-pipelined tiles and default-policy loads
    // (neither beat the shipped kernel on MI355X)
    if (p.pipe && p.nt) launch_uniform_pn<true, true>(p, base, stride, len, ss, ss0, out, n, s);
    else if (p.pipe) launch_uniform_pn<true, false>(p, base, stride, len, ss, ss0, out, n, s);
    else if (p.nt) launch_uniform_pn<false, true>(p, base, stride, len, ss, ss0, out, n, s);
    else launch_uniform_pn<false, false>(p, base, stride, len, ss, ss0, out, n, s);
#else
    launch_uniform_pn<false, true>(p, base, stride, len, ss, ss0, out, n, s);
#endif
}

template <int G, int C, int U, int MODE>
static void launch_multi_t(const UniformMultiArgs& a, uint32_t k, hipStream_t s, int max_blocks) {
    constexpr int UE = (C * U > 32) ? (32 / C > 0 ? 32 / C : 1) : U;   // VGPR budget, as launch_uniform_t
    constexpr int SPT = (64 / G) * UE;
    uint64_t tiles = 0;
    for (uint32_t i = 0; i < k; ++i) tiles = std::max<uint64_t>(tiles, (a.e[i].n + SPT - 1) / SPT);
    hipLaunchKernelGGL((k_uniform_multi<G, C, UE, MODE>), dim3(grid_for(tiles, max_blocks), k), dim3(256), 0, s, a);
}

template <int MODE>
static void launch_multi_mode(int shape, int unroll, const UniformMultiArgs& a, uint32_t k, hipStream_t s,
                              int max_blocks) {
#define TM(G, C, U) launch_multi_t<G, C, U, MODE>(a, k, s, max_blocks)
#define TM48(G, C)                 \
    do {                           \
        if (unroll <= 4) TM(G, C, 4); \
        else TM(G, C, 8);          \
    } while (0)
    switch (shape) {
        case 0: TM48(4, 1); break;
        case 1: TM48(8, 1); break;
        case 2: TM48(16, 1); break;
        case 3: TM48(32, 1); break;
        case 4: TM48(64, 1); break;
        case 5: TM48(32, 3); break;
        case 6: TM48(64, 2); break;
        case 7: TM48(64, 4); break;
        case 8: TM(64, 8, 4); break;
        case 10: TM(1, 5, 2); break;
        default: TM(2, 4, 2); break;   // 11
    }
#undef TM48
#undef TM
}

// Batches that share a lane-group shape (segments up to 8 KiB) go out as one
// launch, in the most general alignment mode any of them needs and the widest
// shape any of them needs (a shape covers every shorter segment). Anything
// else — long segments, split or flat shapes — is launched batch by batch, where
// a launch's ramp is a small share of its time anyway.
void launch_uniform_multi(const tcpcsum_ubatch_t* b, uint32_t k, hipStream_t s, const Tuning& tu) {
    UniformMultiArgs a;
    uint32_t m = 0;
    int mode = M16, shape = -1, unroll = 8, max_blocks = 0;
    bool one = true;
    for (uint32_t i = 0; i < k; ++i) {
        if (b[i].n == 0) continue;
        const UniformPlan p = plan_uniform((uintptr_t)b[i].d_base, b[i].stride, b[i].len, b[i].n, tu);
        unroll = std::min(unroll, p.unroll);            // the smallest tile any batch's plan takes
        max_blocks = std::max(max_blocks, p.max_blocks);
        const bool lane_group = p.shape <= 8 || p.shape == 10 || p.shape == 11;
        if (!lane_group || (shape >= 0 && (shape > 8 || p.shape > 8) && shape != p.shape)) one = false;
        mode = std::max(mode, p.mode);
        shape = std::max(shape, p.shape);
        a.e[m++] = UniformMultiEntry{(const uint8_t*)b[i].d_base, b[i].d_sum_start, b[i].d_out, b[i].stride,
                                     b[i].n, b[i].len, b[i].sum_start};
    }
    if (m == 0) return;
    if (!one) {
        for (uint32_t i = 0; i < k; ++i)
            if (b[i].n)
                launch_uniform((const uint8_t*)b[i].d_base, b[i].stride, b[i].len, b[i].d_sum_start, b[i].sum_start,
                               b[i].d_out, b[i].n, s, tu);
        return;
    }
    // the single-batch plans' launch shape (plan_uniform: one tile per wave for lane-group
    // shapes); the byte-granular mode any batch forces keeps its own (<= 4 in flight, 16384
    // workgroups)
    if (mode == M1) {
        if (!tu.unroll) unroll = std::min(unroll, 4);
        max_blocks = tu.max_blocks > 0 ? tu.max_blocks : 16384;
    }
    if (mode == M16) launch_multi_mode<M16>(shape, unroll, a, m, s, max_blocks);
    else if (mode == M4) launch_multi_mode<M4>(shape, unroll, a, m, s, max_blocks);
    else launch_multi_mode<M1>(shape, unroll, a, m, s, max_blocks);
}

template <int G, int C, int U>
static void launch_desc_t(const uint8_t* base, const tcpcsum_desc_t* d, uint64_t n, uint16_t* out,
                          hipStream_t s, int max_blocks) {
    constexpr int SPT = (64 / G) * U;
    hipLaunchKernelGGL((k_desc<G, C, U>), dim3(grid_for((n + SPT - 1) / SPT, max_blocks)), dim3(256), 0, s, base, d,
                       n, out);
}

void launch_desc(const uint8_t* base, const tcpcsum_desc_t* d, uint64_t n, uint32_t max_len, uint16_t* out,
                 hipStream_t s, const Tuning& tu) {
    const uint64_t nch = ((uint64_t)max_len + 30u) >> 4;   // worst-case start alignment
    const int max_blocks = tu.max_blocks > 0 ? tu.max_blocks : kDefaultMaxBlocks;
    const int unroll = tu.unroll ? tu.unroll : 2;
#define DS_U(G, C)                                                                 \
    do {                                                                           \
        if (unroll <= 1) launch_desc_t<G, C, 1>(base, d, n, out, s, max_blocks);   \
        else if (unroll == 2) launch_desc_t<G, C, 2>(base, d, n, out, s, max_blocks); \
        else launch_desc_t<G, C, 4>(base, d, n, out, s, max_blocks);               \
    } while (0)
    // lane-group shape: by max_len, or forced (tuning shape 0..6, in this order;
    // 7 / 8: balanced chunk space with 4 / 8 loads per lane in flight)
    int sh = tu.shape;
    if (sh > 8) sh = -1;
    const bool auto_shape = sh < 0;
    // auto: a large ragged batch takes the balanced kernel (a ragged batch has mixed
    // lengths by nature; uniform lengths belong to tcpcsum_batch_uniform_dev); small
    // batches and very long segments the lane groups by max_len
    if (sh < 0 && n >= 65536u && max_len <= 65536u) sh = 7;
    if (sh < 0)
        sh = nch <= 4 ? 0 : nch <= 8 ? 1 : nch <= 16 ? 2 : nch <= 32 ? 3 : nch <= 96 ? 4 : nch <= 256 ? 5 : 6;
    if (sh == 7 || sh == 8) {
        // Segments per wave tile: 64, or for long segments as many as make about
        // 8192 chunks (128 KiB) of work per wave at max_len — a tile of 64 long
        // segments leaves too few waves: 64K x 64 KiB 1.385 ms with 64 per tile
        // against 0.635 for lane groups (tools/desc_sweep.py,
        // profiles/r02_desc_sweep.jsonl)
        // (a forced unroll u divides it: at most 64 / u per tile — tile-size sweeps)
        uint32_t spw = tu.unroll ? 64u / (uint32_t)tu.unroll : 64u;
        while (spw > 1 && (uint64_t)spw * nch > 8192u) spw >>= 1;
        // and, chosen automatically, at least 4096 wave tiles where the batch allows
        // (16 waves per CU: 16K x 1500-B descriptors 0.0361 -> 0.0082 ms; a forced
        // shape keeps the max_len tile, which is what the tile-edge tests exercise)
        if (auto_shape)
            while (spw > 1 && (n + spw - 1) / spw < 4096u) spw >>= 1;
        // one tile per wave by default (4M x 84-B packets: -4 %)
        const dim3 grid(grid_for((n + spw - 1) / spw, tu.max_blocks > 0 ? tu.max_blocks : 1 << 24));
        if (sh == 7) hipLaunchKernelGGL(k_desc_lb<4>, grid, dim3(256), 0, s, base, d, n, out, spw);
        else hipLaunchKernelGGL(k_desc_lb<8>, grid, dim3(256), 0, s, base, d, n, out, spw);
        return;
    }
    switch (sh) {
        case 0: DS_U(4, 1); break;
        case 1: DS_U(8, 1); break;
        case 2: DS_U(16, 1); break;
        case 3: DS_U(32, 1); break;
        case 4: DS_U(32, 3); break;
        case 5: DS_U(64, 4); break;
        default: DS_U(64, 8); break;
    }
#undef DS_U
}

template <int G, int C, int U, bool VER>
static void launch_ipv4_m(uint8_t* pkts, const uint64_t* off, const uint32_t* plen, uint64_t n, uint32_t cap,
                          uint64_t limit, int mode, uint16_t* out, uint8_t* status, uint16_t* ipout, hipStream_t s,
                          const dim3 grid, bool nt, uint32_t amask, int dw) {
    // per-packet bounds only when given: the extra load and register cost the
    // region-bounded MTU batches 4-8 % (tools/wire_ab.py)
    if (plen && nt)
        hipLaunchKernelGGL((k_ipv4<G, C, U, true, true, VER>), grid, dim3(256), 0, s, pkts, off, plen, n, cap, limit,
                           mode, out, status, ipout, amask, dw);
    else if (plen)
        hipLaunchKernelGGL((k_ipv4<G, C, U, false, true, VER>), grid, dim3(256), 0, s, pkts, off, plen, n, cap, limit,
                           mode, out, status, ipout, amask, dw);
    else if (nt)
        hipLaunchKernelGGL((k_ipv4<G, C, U, true, false, VER>), grid, dim3(256), 0, s, pkts, off, plen, n, cap, limit,
                           mode, out, status, ipout, amask, dw);
    else
        hipLaunchKernelGGL((k_ipv4<G, C, U, false, false, VER>), grid, dim3(256), 0, s, pkts, off, plen, n, cap, limit,
                           mode, out, status, ipout, amask, dw);
}

template <int G, int C, int U>
static void launch_ipv4_t(uint8_t* pkts, const uint64_t* off, const uint32_t* plen, uint64_t n, uint32_t cap,
                          uint64_t limit, int mode, uint16_t* out, uint8_t* status, uint16_t* ipout, hipStream_t s,
                          int max_blocks, bool nt, uint32_t amask, int dw) {
    constexpr int SPT = (64 / G) * U;
    const dim3 grid(grid_for((n + SPT - 1) / SPT, max_blocks));
    if (mode & TCPCSUM_IPV4_VERIFY)
        launch_ipv4_m<G, C, U, true>(pkts, off, plen, n, cap, limit, mode, out, status, ipout, s, grid, nt, amask, dw);
    else
        launch_ipv4_m<G, C, U, false>(pkts, off, plen, n, cap, limit, mode, out, status, ipout, s, grid, nt, amask, dw);
}

void launch_ipv4(uint8_t* pkts, const uint64_t* off, const uint32_t* plen, uint64_t n, uint32_t cap, uint64_t limit,
                 uint64_t footprint, int mode, uint16_t* out, uint8_t* status, uint16_t* ipout, hipStream_t s,
                 const Tuning& tu) {
    // caps up to 4 KiB: one tile per wave, so the tiles go XCD by XCD at any batch size
    // (2M MTU packets in 1536-B slots: FILL 0.6345 -> 0.6065 ms, VERIFY 0.4824 -> 0.4674
    // against 32768 looping workgroups; 1M and fewer already covered;
    // profiles/r05_wire_grid_xcd.jsonl). Jumbo caps: 32768 workgroups (at most one or two
    // tiles per wave): 1M x 9000-B packets VERIFY 1.46 -> 1.41 ms, FILL 1.62 -> 1.59 against
    // 8192 (profiles/r02_wire_jumbo_sweep.jsonl)
    const int max_blocks = tu.max_blocks > 0 ? tu.max_blocks : cap <= 4096u ? (1 << 24) : 32768;
    const int unroll = tu.unroll ? tu.unroll : 1;
    const bool nt = (tu.flags & TCPCSUM_TUNE_WIRE_CACHED) == 0;
    const uint32_t amask = (tu.flags & TCPCSUM_TUNE_WIN16) ? 15u : 127u;
    // FILL store: the whole 128-B line written through where it lies inside the
    // packet (default), one native u16 (context.c:208), or the check|urg_ptr dword
    const int dw = (tu.flags & TCPCSUM_TUNE_FILL_DWORD) ? 1 : (tu.flags & TCPCSUM_TUNE_FILL_U16) ? 0
                 : (tu.flags & TCPCSUM_TUNE_FILL_HALF) ? 3 : 2;
    // shape by the cap and by the mean packet footprint (region bytes / n; the
    // summed lengths for scatter-gather batches): packed small packets one
    // chunk per lane, MTU slots one round of 96 chunks per packet
    const uint64_t nch = ((uint64_t)cap + 15u) >> 4;   // an odd start takes one extra round
    const uint64_t mean = n ? footprint / n : 0;
#define IP_U(G, C)                                                                                                   \
    do {                                                                                                             \
        if (unroll <= 1)                                                                                             \
            launch_ipv4_t<G, C, 1>(pkts, off, plen, n, cap, limit, mode, out, status, ipout, s, max_blocks, nt,     \
                                   amask, dw);                                                                           \
        else if (unroll == 2)                                                                                        \
            launch_ipv4_t<G, C, 2>(pkts, off, plen, n, cap, limit, mode, out, status, ipout, s, max_blocks, nt,     \
                                   amask, dw);                                                                           \
        else                                                                                                         \
            launch_ipv4_t<G, C, 4>(pkts, off, plen, n, cap, limit, mode, out, status, ipout, s, max_blocks, nt,     \
                                   amask, dw);                                                                           \
    } while (0)
    // forced: 0 (8,1), 1 (32,3), 2 (64,4), 3 (16,2), 4 (16,6), 5 (8,12), 6 (8,2), 7 (8,4),
    // 8 / 9: balanced chunk space (k_ipv4_lb) with 4 / 8 loads per lane in flight
    int sh = tu.shape;
    const bool auto_shape = sh < 0 || sh > 9;
    // auto: large batches of small or mixed packets (mean footprint < 960 B,
    // e.g. packed IMIX, 576-896-B slots) take the balanced kernel; MTU-size
    // slots, jumbo packets and small batches (a releaseSend batch of <= 1024
    // packets: latency, not throughput — a balanced wave walks 64 packets in
    // turn) the lane-group kernels, one speculative round trip per packet. Large
    // batches of 1-1.5 KiB packets take 4-chunk rounds (fewer registers, more
    // waves: 1024-B slots 0.226 -> 0.173 ms VERIFY, 1536-B 0.250 -> 0.242 than
    // one 12-chunk round; profiles/r02_wire_mtu_sweep.jsonl)
    // Large batches of 1.5-5 KiB packets (the cap, or the mean footprint when
    // smaller, sizes them) keep 4- or 6-chunk rounds: 2 KiB slots VERIFY 0.549 ->
    // 0.314 ms and FILL 0.578 -> 0.402 against one 96-chunk round per lane group
    // (32,3); 3 KiB -19 % / -11 %, 4.5 KiB -7 % / -7 % with (16,6); 9 KiB jumbo
    // slots alike across shapes and keep (32,3) (profiles/r02_wire_big_sweep.jsonl,
    // profiles/r02_wire_big_sweep.jsonl)
    const uint64_t nsz = mean && ((mean + 15u) >> 4) < nch ? (mean + 15u) >> 4 : nch;
    if (sh < 0 || sh > 9) {
        if (n >= 65536u && mean < 960u) {
            sh = 8;
        } else if (nch <= 8 || mean <= 112u) {
            sh = 0;
        } else if (nsz <= 192 && n >= 16384u) {
            // from 16K packets up (32K MTU packets 0.0116 -> 0.0103 ms; up to 8K
            // packets every shape is within launch latency, ~8.5 us;
            // profiles/r02_wire_small_sweep.jsonl)
            sh = 7;
        } else if (nsz <= 320 && n >= 65536u) {
            sh = 4;
        } else {
            sh = nch <= 96 ? 5 : 1;
        }
    }
    if (sh == 8 || sh == 9) {
        // 64 packets per wave tile; chosen automatically, at least 4096 tiles where
        // the batch allows (16 waves per CU; profiles/r02_wire_lb_small_batches.jsonl)
        // 32 packets per wave tile (a forced unroll u: 64 / u — tile-size sweeps): against 64,
        // same process, the flush mix FILL 0.1118 -> 0.0982 ms (VERIFY even), 2M packed 576-B
        // packets FILL -11 %, VERIFY -6 %; 16 loses VERIFY (+6 .. +16 %)
        // (profiles/r06_wire_lb_tile.jsonl)
        uint32_t spw = tu.unroll ? 64u / (uint32_t)tu.unroll : 32u;
        if (auto_shape)
            while (spw > 1 && (n + spw - 1) / spw < 4096u) spw >>= 1;
        // one tile per wave by default (4M packed 84-B packets 0.116 -> 0.112 ms
        // against 8192 blocks; profiles/r02_lb_grid_sweep.jsonl); the prefetching loop of
        // measurement variant 4 wants several tiles per wave: 1536 workgroups
        const int lb_blocks = (TCPCSUM_LB_VARIANT & 4) ? 1536 : 1 << 24;
        const dim3 grid(grid_for((n + spw - 1) / spw, tu.max_blocks > 0 ? tu.max_blocks : lb_blocks));
        // the head-in-registers path (k_ipv4_lb) is its own instantiation, for FILL without
        // IPHDR: it needs 86 VGPRs against 78 (5 waves per SIMD, not 6; asked for 6 the
        // compiler spills) and VERIFY ran slower with it (flush mix VERIFY 0.0851 vs 0.078 ms),
        // FILL faster (flush mix 0.0928 vs 0.0962, 2M packed 576-B 0.254 vs 0.290;
        // profiles/r06_lb_head_ab.jsonl)
        const bool hd = !(mode & TCPCSUM_IPV4_IPHDR) &&
                        (TCPCSUM_LB_HEAD == 2 || (TCPCSUM_LB_HEAD == 1 && !(mode & TCPCSUM_IPV4_VERIFY)));
#define TCPCSUM_LB_WIRE(C_, PL_, HD_)                                                                          \
    hipLaunchKernelGGL((k_ipv4_lb<C_, PL_, HD_>), grid, dim3(256), 0, s, pkts, off, plen, n, cap, limit, mode, out, \
                       status, ipout, spw)
        if (sh == 8) {
            if (plen) { if (hd) TCPCSUM_LB_WIRE(4, true, true); else TCPCSUM_LB_WIRE(4, true, false); }
            else { if (hd) TCPCSUM_LB_WIRE(4, false, true); else TCPCSUM_LB_WIRE(4, false, false); }
        } else {
            if (plen) { if (hd) TCPCSUM_LB_WIRE(8, true, true); else TCPCSUM_LB_WIRE(8, true, false); }
            else { if (hd) TCPCSUM_LB_WIRE(8, false, true); else TCPCSUM_LB_WIRE(8, false, false); }
        }
#undef TCPCSUM_LB_WIRE
        return;
    }
    switch (sh) {
        case 0: IP_U(8, 1); break;
        case 1: IP_U(32, 3); break;
        case 2: IP_U(64, 4); break;
        case 3: IP_U(16, 2); break;
        case 4: IP_U(16, 6); break;
        case 5: IP_U(8, 12); break;
        case 6: IP_U(8, 2); break;
        default: IP_U(8, 4); break;
    }
#undef IP_U
}

template <int G, int C, int U>
static void launch_tx_t(const uint8_t* payload, const tcpcsum_txseg_t* segs, uint64_t n, uint8_t* outp, int mode,
                        uint16_t* checks, hipStream_t s, int max_blocks, int sp) {
    constexpr int SPT = (64 / G) * U;
    const dim3 grid(grid_for((n + SPT - 1) / SPT, max_blocks));
    if (sp == 1)
        hipLaunchKernelGGL((k_tx_build<G, C, U, 1>), grid, dim3(256), 0, s, payload, segs, n, outp, mode, checks);
    else if (sp == 2)
        hipLaunchKernelGGL((k_tx_build<G, C, U, 2>), grid, dim3(256), 0, s, payload, segs, n, outp, mode, checks);
    else
        hipLaunchKernelGGL((k_tx_build<G, C, U, 0>), grid, dim3(256), 0, s, payload, segs, n, outp, mode, checks);
}

void launch_tx_build(const uint8_t* payload, const tcpcsum_txseg_t* segs, uint64_t n, uint32_t max_len,
                     uint8_t* outp, int mode, uint16_t* checks, hipStream_t s, const Tuning& tu) {
    // 32768 blocks: 1M x 1456-B payloads 0.777 -> 0.746 ms against 4096 (tools/txbench.py --sweep)
    const int max_blocks = tu.max_blocks > 0 ? tu.max_blocks : 32768;
    const int unroll = tu.unroll ? tu.unroll : 1;
    const uint64_t nfull = ((uint64_t)max_len + 15u) >> 4;   // full chunks a payload can have
    const int sp = (tu.flags & TCPCSUM_TUNE_TX_WT_STORE) ? 2 : (tu.flags & TCPCSUM_TUNE_TX_NT_STORE) ? 1 : 0;
#define TX_U(G, C)                                                                         \
    do {                                                                                   \
        if (unroll <= 1) launch_tx_t<G, C, 1>(payload, segs, n, outp, mode, checks, s, max_blocks, sp); \
        else if (unroll == 2) launch_tx_t<G, C, 2>(payload, segs, n, outp, mode, checks, s, max_blocks, sp); \
        else launch_tx_t<G, C, 4>(payload, segs, n, outp, mode, checks, s, max_blocks, sp);    \
    } while (0)
    // payloads of 129 B .. 768 B: 16-lane groups, two chunks per lane per round
    // (round 2: 256 B 1.76 -> 1.05 ms, 536 B 1.40 -> 1.07; profiles/r02_tx_size_sweep.jsonl);
    // 769 B .. 1.5 KiB: 16-lane groups, six chunks per lane, one round (round 3, after
    // the lane-exchange change, 1.5 GB of payload per launch: 896 B 0.734 -> 0.698 ms,
    // 1024 B 0.719 -> 0.638, 1200 B 0.795 -> 0.644, 1456 B 0.624 -> 0.611 against the
    // previous (16,2) / (32,3); profiles/r03_tx_size_ab.jsonl); longer: (64,4)
    int shape = nfull <= 8 ? 0 : nfull <= 48 ? 1 : nfull <= 96 ? 5 : 4;
    if (tu.shape >= 0 && tu.shape <= 6) shape = tu.shape;   // any shape is correct (extra rounds)
    switch (shape) {
        case 0: TX_U(8, 1); break;
        case 1: TX_U(16, 2); break;
        case 2: TX_U(32, 3); break;
        case 3: TX_U(64, 2); break;
        case 5: TX_U(16, 6); break;
        case 6: TX_U(8, 12); break;
        default: TX_U(64, 4);
    }
#undef TX_U
}

void launch_synth_fill(uint8_t* dst, uint64_t off, uint64_t nbytes, hipStream_t s) {
    const uint64_t words = ((off + nbytes + 7) >> 3) - (off >> 3);
    uint64_t blocks = (words + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_synth_fill, dim3((unsigned)blocks), dim3(256), 0, s, dst, off, nbytes);
}

void launch_synth_pseudo(uint32_t* ss, uint64_t seg0, uint64_t n, uint32_t seg_len, hipStream_t s) {
    const uint32_t l16 = seg_len & 0xffffu;
    const uint32_t len_be = ((l16 & 0xffu) << 8) | (l16 >> 8);
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_synth_pseudo, dim3((unsigned)blocks), dim3(256), 0, s, ss, seg0, n, len_be);
}

int launch_probe(const uint8_t* src, uint64_t nbytes, uint64_t* partials, hipStream_t s, const Tuning& tu) {
    // chunks per lane per wave tile, C: by unroll 0 / 1 / 2 / >= 4 -> 4 (the default: one 4 KiB
    // tile per wave, the uniform plan's tile) / 8 / 16 / 32; a read-only probe also takes
    // shape 2 or 3 as C, and shape 10 / 11 / 12 as 32-lane groups with C = 2 / 3 / 4 (sweeps)
    const bool wr = (tu.flags & TCPCSUM_TUNE_PROBE_WRITE) != 0;
    int C = tu.unroll == 0 ? 4 : tu.unroll == 1 ? 8 : tu.unroll == 2 ? 16 : 32;
    if (!wr && (tu.shape == 2 || tu.shape == 3)) C = tu.shape;
    const int max_blocks = tu.max_blocks > 0 ? tu.max_blocks : (1 << 24);
    const uint64_t nchunks = nbytes / 16;
    const unsigned g = grid_for((nchunks + 64u * C - 1) / (64u * C), max_blocks);
    const int used = (int)(4ull * g < (uint64_t)kProbeSlots ? 4ull * g : (uint64_t)kProbeSlots);
    // write-back probe: the wire FILL's traffic, shape = line period
    const uint32_t period = wr ? (tu.shape > 0 ? (uint32_t)tu.shape : 12u) : 1u;
#define TC_P(CC)                                                                                              \
    do {                                                                                                      \
        if (wr) hipLaunchKernelGGL((k_probe<CC, true>), dim3(g), dim3(256), 0, s, src, nchunks, partials, period); \
        else hipLaunchKernelGGL((k_probe<CC, false>), dim3(g), dim3(256), 0, s, src, nchunks, partials, period);   \
    } while (0)
    if (!wr && tu.shape >= 10 && tu.shape <= 12) {   // 32-lane groups (two 512-B pieces per instruction), C = 2..4
        const unsigned C2 = (unsigned)tu.shape - 8u;
        const unsigned g2 = grid_for((nchunks + 64u * C2 - 1) / (64u * C2), max_blocks);
        if (C2 == 2) hipLaunchKernelGGL((k_probe<2, false, 32>), dim3(g2), dim3(256), 0, s, src, nchunks, partials, 1u);
        else if (C2 == 3) hipLaunchKernelGGL((k_probe<3, false, 32>), dim3(g2), dim3(256), 0, s, src, nchunks, partials, 1u);
        else hipLaunchKernelGGL((k_probe<4, false, 32>), dim3(g2), dim3(256), 0, s, src, nchunks, partials, 1u);
        return (int)(4ull * g2 < (uint64_t)kProbeSlots ? 4ull * g2 : (uint64_t)kProbeSlots);
    }
    switch (C) {
        case 2: hipLaunchKernelGGL((k_probe<2, false>), dim3(g), dim3(256), 0, s, src, nchunks, partials, 1u); break;
        case 3: hipLaunchKernelGGL((k_probe<3, false>), dim3(g), dim3(256), 0, s, src, nchunks, partials, 1u); break;
        case 4: TC_P(4); break;
        case 8: TC_P(8); break;
        case 16: TC_P(16); break;
        default: TC_P(32); break;
    }
#undef TC_P
    return used;
}

}  // namespace tcpcsum
