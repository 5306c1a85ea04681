// tcpcsum_internal.h — launchers shared between the kernel TU and the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tcpcsum.h"

// ---------------------------------------------------------------- build knobs
// Compile-time knobs. A product library leaves every one at its default; only a
// measurement build (tools/*_ab.py, -DTCPCSUM_MEASUREMENT_BUILD=1) may set them,
// and tcpcsum_build_info() reports them either way ("product": false there).
//   TCPCSUM_TUNING_VARIANTS  1: also compile the pipelined / default-load kernel
//                            variants the TCPCSUM_TUNE_PIPE_* / NT_* flags select
//   TCPCSUM_TX_KNOCKOUT      parts of the segment builder switched off to see what
//                            its time is made of — the output is then WRONG. 1:
//                            ragged-end stores, 2: header stores, 4: second source
//                            loads, 8: full-chunk stores
//   TCPCSUM_WIRE_WAVES       minimum waves per SIMD asked of the lane-group wire
//   TCPCSUM_TX_WAVES         kernel / the segment builder (1 = the compiler's choice)
#ifndef TCPCSUM_MEASUREMENT_BUILD
#define TCPCSUM_MEASUREMENT_BUILD 0
#endif
#ifndef TCPCSUM_TUNING_VARIANTS
#define TCPCSUM_TUNING_VARIANTS 0
#endif
#ifndef TCPCSUM_TX_KNOCKOUT
#define TCPCSUM_TX_KNOCKOUT 0
#endif
#ifndef TCPCSUM_WIRE_WAVES
#define TCPCSUM_WIRE_WAVES 1
#endif
#ifndef TCPCSUM_TX_WAVES
#define TCPCSUM_TX_WAVES 1
#endif
//   TCPCSUM_LINE_CPOL        cache-policy bits of the 16-B line stores (wire FILL, write-back
//                            probe): 17 = sc0|sc1, written through (the product's)
#ifndef TCPCSUM_LINE_CPOL
#define TCPCSUM_LINE_CPOL 17
#endif
//   TCPCSUM_LOAD_CPOL        >= 0: the uniform kernel's segment loads become buffer loads with
//                            these cache-policy bits (batches under 4 GiB only); -1: global
//                            loads, non-temporal (the product's)
#ifndef TCPCSUM_LOAD_CPOL
#define TCPCSUM_LOAD_CPOL -1
#endif
//   TCPCSUM_XCD_REMAP        1 (the product's): a wave-tile launch whose grid covers its batch in
//                            whole XCD rounds takes its tiles XCD by XCD (xcd_block: block b, on
//                            XCD b % 8 under round-robin dispatch, takes tile run (b % 8) * B/8 +
//                            b / 8), so each XCD sweeps one contiguous eighth of the batch;
//                            0: block b takes tile run b
#ifndef TCPCSUM_XCD_REMAP
#define TCPCSUM_XCD_REMAP 1
#endif
//   TCPCSUM_XCD_CHUNK        > 0: with the XCD order, the XCDs take runs of this many workgroups
//                            in turn instead of one contiguous eighth each; 0 (the product's)
#ifndef TCPCSUM_XCD_CHUNK
#define TCPCSUM_XCD_CHUNK 0
#endif
//   TCPCSUM_UNIFORM_WPB      waves per workgroup of the uniform kernel: 4 (the product's), 1 or 2
#ifndef TCPCSUM_UNIFORM_WPB
#define TCPCSUM_UNIFORM_WPB 4
#endif
//   TCPCSUM_DESC_LB_WAVES    minimum waves per SIMD asked of the balanced kernels (ragged and
//                            wire; amdgpu_waves_per_eu): 1 = the compiler's choice (the product's)
#ifndef TCPCSUM_DESC_LB_WAVES
#define TCPCSUM_DESC_LB_WAVES 1
#endif
//   TCPCSUM_SS_LOAD          how the uniform kernel's lane-group tiles read the start values:
//                            0 one dword per group (lane 0), 1 the same non-temporal, 2 one
//                            coalesced dword per lane for the tile (ds_bpermute to the groups),
//                            3 the same non-temporal. 2 is the product's: 1M x 576 B -4.5 %, the
//                            rest within +-1 % (profiles/r06_ss_ab.jsonl)
#ifndef TCPCSUM_SS_LOAD
#define TCPCSUM_SS_LOAD 2
#endif
//   TCPCSUM_LB_VARIANT       the balanced kernels' sweep (lb_sums_t): bit 0 the LDS-mark owner
//                            search, bit 1 software-pipelined rounds
#ifndef TCPCSUM_LB_VARIANT
#define TCPCSUM_LB_VARIANT 0
#endif
//   TCPCSUM_LB_HEAD          1: the balanced wire kernel's FILL (without IPHDR) takes 4-B aligned
//                            packets' first 64 bytes in registers and sweeps only the rest (the
//                            product's); 2: VERIFY too; 0: neither (header read apart, every TCP
//                            byte swept)
#ifndef TCPCSUM_LB_HEAD
#define TCPCSUM_LB_HEAD 1
#endif
//   TCPCSUM_LB_HDR_X4        1: the balanced wire kernel reads 4-B aligned tiles' headers with one
//                            dwordx4 and one dword load per packet; 0: five dword loads
#ifndef TCPCSUM_LB_HDR_X4
#define TCPCSUM_LB_HDR_X4 1
#endif
#if !TCPCSUM_MEASUREMENT_BUILD && \
    (TCPCSUM_TUNING_VARIANTS != 0 || TCPCSUM_TX_KNOCKOUT != 0 || TCPCSUM_WIRE_WAVES != 1 || TCPCSUM_TX_WAVES != 1 || \
     TCPCSUM_LINE_CPOL != 17 || TCPCSUM_LOAD_CPOL != -1 || TCPCSUM_XCD_REMAP != 1 || TCPCSUM_XCD_CHUNK != 0 || \
     TCPCSUM_UNIFORM_WPB != 4 || TCPCSUM_DESC_LB_WAVES != 1 || TCPCSUM_SS_LOAD != 2 || TCPCSUM_LB_VARIANT != 0 || \
     TCPCSUM_LB_HEAD != 1 || TCPCSUM_LB_HDR_X4 != 1)
#error "tuning / knock-out / waves knobs are for measurement builds only (-DTCPCSUM_MEASUREMENT_BUILD=1), never a product library"
#endif
// Environment variables a context reads at creation (tcpcsum_build_info "runtime_knobs"):
// a product library reads the deployment ones only — copy threads, their NUMA pinning
// and spin, and the launcher's rank count on the node (copy_pool.h); a measurement build
// also reads the switches of the host pipeline's A/B variants (tcpcsum_host.hip,
// TCPCSUM_MEAS_KNOB), which a product library never sees.
#define TCPCSUM_PRODUCT_RUNTIME_KNOBS \
    "\"TCPCSUM_HOST_THREADS\", \"TCPCSUM_HOST_NUMA\", \"TCPCSUM_HOST_SPIN_US\", \"LOCAL_WORLD_SIZE\""
#if TCPCSUM_MEASUREMENT_BUILD
#define TCPCSUM_RUNTIME_KNOBS_JSON TCPCSUM_PRODUCT_RUNTIME_KNOBS \
    ", \"TCPCSUM_HOST_WIRE_THREADS\", \"TCPCSUM_HOST_BULK_THREADS\", \"TCPCSUM_HOST_NT\", " \
    "\"TCPCSUM_HOST_POLL_US\", \"TCPCSUM_HOST_STAGE_PASSES\", \"TCPCSUM_HOST_DMA\", " \
    "\"TCPCSUM_HOST_PINNED_DMA\", \"TCPCSUM_HOST_SLOT_SLEEP\", \"TCPCSUM_HOST_WIRE_NT\", " \
    "\"TCPCSUM_HOST_SLOTS\", \"TCPCSUM_HOST_CHUNK_MB\", \"TCPCSUM_HOST_DMA_CHUNK_MB\""
#else
#define TCPCSUM_RUNTIME_KNOBS_JSON TCPCSUM_PRODUCT_RUNTIME_KNOBS
#endif
// Hash of the sources the library was compiled from (the Makefile passes it).
#ifndef TCPCSUM_SRC_HASH
#define TCPCSUM_SRC_HASH "unknown"
#endif

namespace tcpcsum {

// 256 CUs x 8 workgroups of 256 threads = 32 waves per CU: the whole grid is
// resident at once and grid-strides over the batch.
constexpr int kDefaultMaxBlocks = 2048;

// Slots of tcpcsum_stream_probe_dev's partials array (= its maximum grid).
constexpr int kProbeSlots = TCPCSUM_PROBE_SLOTS;

struct Tuning {
    int max_blocks = 0;   // 0 = per-shape default
    int unroll = 0;       // 0 = per-shape default; else 1, 2, 4 or 8
    int shape = -1;       // -1 = auto; else a forced lane-group shape (per launcher)
    int flags = 0;        // TCPCSUM_TUNE_* bits
};

struct UniformPlan {
    int mode;        // 0: 16-B aligned starts/len, 1: 4-B aligned, 2: byte granular
    int shape;       // 0..8 segment-group shapes, 9 = one wave per long segment
    int unroll;      // segments in flight per lane group (shape 9: 8*unroll chunks per lane per round)
    int max_blocks;  // resident grid (workgroups of 256 threads)
    bool pipe;       // software-pipelined tiles
    bool nt;         // non-temporal loads
    int blocked;     // contiguous tile runs per wave instead of a grid stride
};
UniformPlan plan_uniform(uintptr_t base, uint64_t stride, uint32_t len, uint64_t n, const Tuning& tu);

// One batch of a multi-batch uniform launch (kernel-argument layout).
struct UniformMultiEntry {
    const uint8_t* base;
    const uint32_t* ss;   // nullable: ss0 for every segment
    uint16_t* out;
    uint64_t stride;
    uint64_t n;
    uint32_t len;
    uint32_t ss0;
};
struct UniformMultiArgs {
    UniformMultiEntry e[TCPCSUM_MULTI_MAX];
};
// k <= TCPCSUM_MULTI_MAX batches: one launch when they share a lane-group
// shape, else one launch per batch.
void launch_uniform_multi(const tcpcsum_ubatch_t* b, uint32_t k, hipStream_t s, const Tuning& tu);

void launch_uniform(const uint8_t* base, uint64_t stride, uint32_t len, const uint32_t* ss, uint32_t ss0,
                    uint16_t* out, uint64_t n, hipStream_t s, const Tuning& tu);
void launch_desc(const uint8_t* base, const tcpcsum_desc_t* d, uint64_t n, uint32_t max_len, uint16_t* out,
                 hipStream_t s, const Tuning& tu);
// Wire batch: packet i at pkts + off[i], readable up to min(limit - off[i], plen[i])
// (plen nullable). footprint: bytes the batch spans (region size, or summed
// lengths), for the shape choice. ipout (nullable): per-packet IPv4 header
// checksum when mode has TCPCSUM_IPV4_IPHDR.
void launch_ipv4(uint8_t* pkts, const uint64_t* off, const uint32_t* plen, uint64_t n, uint32_t cap, uint64_t limit,
                 uint64_t footprint, int mode, uint16_t* out, uint8_t* status, uint16_t* ipout, hipStream_t s,
                 const Tuning& tu);
void launch_tx_build(const uint8_t* payload, const tcpcsum_txseg_t* segs, uint64_t n, uint32_t max_len,
                     uint8_t* outp, int mode, uint16_t* checks, hipStream_t s, const Tuning& tu);
void launch_synth_fill(uint8_t* dst, uint64_t off, uint64_t nbytes, hipStream_t s);
void launch_synth_pseudo(uint32_t* ss, uint64_t seg0, uint64_t n, uint32_t seg_len, hipStream_t s);
// returns the grid size (= partials written)
int launch_probe(const uint8_t* src, uint64_t nbytes, uint64_t* partials, hipStream_t s, const Tuning& tu);

// Shared by the two C-ABI translation units (tcpcsum_api.hip, tcpcsum_host.hip).
void note_hip_error(int e);                              // diagnostics: tcpcsum_last_hip_error
int hip_fail(hipError_t e);                              // note e, return TCPCSUM_EHIP
int get_tuning(const tcpcsum_tuning_t* t, Tuning* out);  // validate; NULL = defaults
int require_device(char* arch, size_t arch_len);         // current device is a gfx950
int check_launch();                                      // hipGetLastError -> status

}  // namespace tcpcsum
