// tcpcsum_internal.h — launchers shared between the kernel TU and the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tcpcsum.h"

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
