/*
 * tcpcsum.h — C ABI of the MI355X (gfx950) TCP checksum engine.
 *
 * Drop-in boundary for the one per-byte hot path of uNetworking/tcp: the
 * 16-bit one's-complement TCP checksum that the reference computes per
 * outgoing segment in
 *     /root/reference/context.c:104-119  getPseudoHeaderSum
 *     /root/reference/context.c:121-145  csum_continue
 *     /root/reference/context.c:208-209  the single call site (send_packet)
 * and flushes in batches of <= 1024 IP packets at
 *     /root/reference/loop.c:27-94       releaseSend -> sendmmsg (loop.c:75)
 *
 * Every batch entry point computes, per segment, exactly
 *     csum_continue(sum_start, segment, nbytes)
 * bit for bit (exact 64-bit sum, the reference's two folds, 16-bit
 * complement, odd trailing byte as the low byte of a zeroed word).
 *
 * Conventions
 *   - Plain C: pointers, sizes, integer status codes; no C++ or torch types.
 *   - "stream" is a hipStream_t passed as void* (NULL = the default stream).
 *     Batch calls are asynchronous on that stream; the caller synchronises.
 *   - d_* pointers are device (or device-accessible) memory; h_* are host.
 *   - Return 0 on success or a negative TCPCSUM_E* code. No mutable global
 *     state: launch shapes come from an explicit per-call tcpcsum_tuning_t
 *     (NULL = built-in defaults) or from the tcpcsum_ctx_t they run in; no
 *     call keeps a pointer after it returns (async calls: until the stream
 *     reaches that point).
 *   - The library page-locks only memory it allocates itself (pinned staging,
 *     tcpcsum_host_alloc); it never registers, locks or unlocks memory it was
 *     handed (ABI v4; DESIGN.md §7 says why). Pageable host memory is copied
 *     by CPU threads into the context's pinned staging instead.
 *   - The caller owns every buffer.
 *   - The batch API covers sum_start < 2^32 (getPseudoHeaderSum returns at
 *     most 6 * 0xFFFF) and segment lengths <= INT32_MAX (csum_continue's
 *     nbytes is an int).
 */
#ifndef TCPCSUM_H
#define TCPCSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCPCSUM_OK 0
#define TCPCSUM_EINVAL (-1)   /* bad argument */
#define TCPCSUM_ENODEV (-2)   /* no usable gfx950 device / HIP runtime */
#define TCPCSUM_EHIP (-3)     /* a HIP call failed (tcpcsum_last_hip_error) */
#define TCPCSUM_ENOMEM (-4)   /* allocation failed */

#define TCPCSUM_ABI_VERSION 5

/* Launch-shape override, passed per call (NULL = the built-in shapes measured
 * on MI355X). Fields: max_blocks (0 = per-shape default, else
 * the resident grid), unroll in {0,1,2,4,8} (0 = default; segments in flight
 * per lane group), shape in {-1, 0..14} (-1 = auto; meaning per entry point,
 * see TCPCSUM_TUNE_* below), flags = TCPCSUM_TUNE_* bits (0 = defaults).
 * Every entry point taking one returns TCPCSUM_EINVAL for an invalid value. */
typedef struct tcpcsum_tuning {
    int32_t max_blocks;
    int32_t unroll;
    int32_t shape;
    int32_t flags;
} tcpcsum_tuning_t;

/* Ragged-batch descriptor: segment = d_base[offset .. offset+len). 16 bytes. */
typedef struct tcpcsum_desc {
    uint64_t offset;
    uint32_t len;
    uint32_t sum_start; /* pseudo-header sum (tcpcsum_pseudo) or any start value */
} tcpcsum_desc_t;

/* Wire-batch modes (tcpcsum_ipv4_batch_dev). */
#define TCPCSUM_IPV4_FILL 0   /* tx: checksum with check=0, store it at TCP+16 */
#define TCPCSUM_IPV4_VERIFY 1 /* rx: checksum incl. check; 0 means the segment verifies */
/* OR-able: also the IPv4 header checksum over ihl*4 bytes (the reference's
 * commented-out context.c:179; the kernel fills it for IPPROTO_RAW sockets).
 * FILL stores it at IP+10; VERIFY reports TCPCSUM_PKT_IPHDR_BAD. */
#define TCPCSUM_IPV4_IPHDR 2

/* Wire-batch per-packet status. */
#define TCPCSUM_PKT_OK 0
#define TCPCSUM_PKT_SKIPPED 1    /* not IPv4/TCP, ihl < 5, or tot_len outside [ihl*4+20, cap] */
#define TCPCSUM_PKT_IPHDR_BAD 2  /* VERIFY|IPHDR: the IPv4 header checksum does not verify */
/* VERIFY: the TCP check does not verify but holds the un-complemented folded
 * pseudo-header sum — a CHECKSUM_PARTIAL segment whose checksum was left for
 * NIC offload (Linux loopback does this). OR-ed with the above. */
#define TCPCSUM_PKT_CSUM_PARTIAL 4

/* ---------------------------------------------------------------- library */
int tcpcsum_abi_version(void);
const char *tcpcsum_strerror(int code);
int tcpcsum_last_hip_error(void);      /* hipError_t of the last failing HIP call */
/* 0 if a gfx950 device is usable; TCPCSUM_ENODEV otherwise. Fills the name
 * of the current device's gfx arch into arch (may be NULL). */
int tcpcsum_device_check(char *arch, size_t arch_len);
/* Build provenance: a NUL-terminated one-line JSON object naming the source
 * hash the library was compiled from (sha256 over the product sources and the
 * Makefile, computed by the Makefile), the compile-time knobs, the offload arch
 * and whether it is a product build ("product": true) or a measurement build
 * (knock-outs / register-budget knobs set; never shipped). Static storage. */
const char *tcpcsum_build_info(void);

/* ------------------------------------------------------ scalar drop-ins
 * Synchronous, reference-identical per-segment helpers for code that needs a
 * single result immediately (e.g. the SYN-ACK retransmit at context.c:94).
 * They run on the calling CPU thread; they are NOT used by any batch entry
 * point below, which always run on the GPU. */

/* == getPseudoHeaderSum, context.c:104-119. saddr/daddr in network order as
 * stored in struct iphdr; len_be = htons(tcp header + payload length). */
unsigned long tcpcsum_pseudo(uint32_t saddr_be, uint32_t daddr_be, uint16_t len_be);

/* == csum_continue, context.c:121-145. */
unsigned short tcpcsum_continue(unsigned long sum_start, const char *p, int nbytes);

/* ------------------------------------------------------ device batches (GPU) */

/* Uniform layout: segment i = d_base[i*stride .. i*stride+len), i < n.
 * Start value: d_sum_start[i] if d_sum_start != NULL, else sum_start.
 * Result:      d_out[i] = csum_continue(start_i, segment_i, len).
 * Replaces the per-packet call at context.c:208-209 for a whole batch. */
int tcpcsum_batch_uniform_dev(const void *d_base, uint64_t stride, uint32_t len,
                              const uint32_t *d_sum_start, uint32_t sum_start,
                              uint16_t *d_out, uint64_t n, void *stream, const tcpcsum_tuning_t *tune);

/* Several independent uniform batches in ONE launch — e.g. the small-segment
 * batches a loop flushes one after another (releaseSend, loop.c:27-94): the
 * launch's ramp and drain, which dominate a single batch of 64-B segments, are
 * paid once. Batch j is exactly tcpcsum_batch_uniform_dev(b[j].d_base,
 * b[j].stride, b[j].len, b[j].d_sum_start, b[j].sum_start, b[j].d_out, b[j].n).
 * batches is a HOST array of k entries (passed to the kernel by value,
 * TCPCSUM_MULTI_MAX per launch). Batches whose segments fit one lane-group
 * shape (up to 8 KiB) share a launch; longer ones are launched one by one. */
#define TCPCSUM_MULTI_MAX 16
typedef struct tcpcsum_ubatch {
    const void *d_base;
    uint64_t stride;
    const uint32_t *d_sum_start;   /* NULL: sum_start for every segment */
    uint16_t *d_out;
    uint64_t n;
    uint32_t len;
    uint32_t sum_start;
} tcpcsum_ubatch_t;
int tcpcsum_batch_uniform_multi_dev(const tcpcsum_ubatch_t *batches, uint32_t k, void *stream,
                                    const tcpcsum_tuning_t *tune);

/* Ragged layout: segment i = d_base[d_desc[i].offset .. +d_desc[i].len).
 * max_len: an upper bound on every d_desc[i].len (picks the kernel shape;
 * segments longer than max_len are still summed correctly, only slower).
 * d_out[i] = csum_continue(d_desc[i].sum_start, segment_i, d_desc[i].len). */
int tcpcsum_batch_desc_dev(const void *d_base, const tcpcsum_desc_t *d_desc, uint64_t n,
                           uint32_t max_len, uint16_t *d_out, void *stream, const tcpcsum_tuning_t *tune);

/* Wire layout (the loop's out-buffers, loop.c:107-116 / releaseSend
 * loop.c:27-94): packet i is a raw IPv4 packet at d_pkts + d_pkt_off[i], of
 * at most cap bytes, inside a device region of region_bytes bytes (the kernel
 * reads at most min(cap, region_bytes - off) bytes of each packet, never
 * outside the region). The pseudo header comes from the IP header (saddr @12,
 * daddr @16, tcp length = tot_len - ihl*4), the TCP segment starts at ihl*4.
 *   FILL:   the sum is taken with the check field (TCP+16) as zero, as
 *           context.c:182 leaves it; the result is stored at TCP+16 in place
 *           (and in d_out[i] when d_out != NULL).
 *   VERIFY: d_out[i] = csum over the segment including check (0 == valid).
 * d_status[i] (may be NULL) = TCPCSUM_PKT_OK or TCPCSUM_PKT_SKIPPED (also when
 * off + tot_len > region_bytes); skipped packets are left untouched and
 * d_out[i] = 0. */
int tcpcsum_ipv4_batch_dev(void *d_pkts, uint64_t region_bytes, const uint64_t *d_pkt_off, uint64_t n,
                           uint32_t cap, int mode, uint16_t *d_out, uint8_t *d_status, void *stream,
                           const tcpcsum_tuning_t *tune);

/* Scatter-gather wire batch: packet i is a raw IPv4 packet at the
 * device-accessible address d_pkt_ptrs[i] (HBM, or page-locked / registered
 * host memory read over PCIe), with d_lens[i] readable bytes there (the
 * iov_len / msg_len of its message; the kernel never reads past it, and a
 * packet with tot_len > d_lens[i] or d_lens[i] < 20 is SKIPPED). cap, modes,
 * results and status exactly as tcpcsum_ipv4_batch_dev. This is the
 * loop's own layout — one separate out-buffer per packet (loop.c:180-183,
 * iov_base per message at loop.c:53-54) — with no gather copy.
 * bytes_hint: the sum of d_lens[i] if the caller knows it (0 = unknown, taken
 * as n * cap). Only the kernel shape depends on it — as the region's size
 * does for tcpcsum_ipv4_batch_dev: large batches of small or mixed packets go
 * to the balanced kernel, MTU-size packets to the lane groups. */
int tcpcsum_ipv4_batch_ptrs_dev(void *const *d_pkt_ptrs, const uint32_t *d_lens, uint64_t n, uint32_t cap,
                                uint64_t bytes_hint, int mode, uint16_t *d_out, uint8_t *d_status, void *stream,
                                const tcpcsum_tuning_t *tune);

/* Segment assembly + checksum in one pass (device-side
 * us_internal_socket_context_send_packet, context.c:150-213, minus its 10 %
 * drop and printf trace). For each descriptor the kernel writes a complete
 * IPv4/TCP packet at d_out_pkts + out_off, laid out exactly as context.c:169-206
 * builds it (ihl 5, tot_len, id = (u16)htonl(54321), ttl 255, TCP, window-scale
 * option 03 03 05 00, doff 6, window 8192), copies the payload (the memcpy at
 * context.c:190) and stores the TCP check (context.c:208) — the payload is
 * read once and written once. 48-byte descriptor: */
#define TCPCSUM_TXF_ACK 1
#define TCPCSUM_TXF_SYN 2
#define TCPCSUM_TXF_FIN 4
#define TCPCSUM_TXF_RST 8
#define TCPCSUM_TXF_DATA 16   /* payload present: PSH set and len bytes copied (context.c:188-191) */
typedef struct tcpcsum_txseg {
    uint64_t payload_off;   /* payload at d_payload + payload_off */
    uint64_t out_off;       /* packet (44 + len bytes) written at d_out_pkts + out_off */
    uint32_t saddr_be;      /* networkSourceIp, as stored (context.c:177) */
    uint32_t daddr_be;      /* networkDestIp (context.c:178) */
    uint32_t seq;           /* hostSeq, host order (stored htonl, context.c:194) */
    uint32_t ack;           /* hostAck, host order (context.c:193) */
    uint16_t sport;         /* hostSourcePort, host order (context.c:195) */
    uint16_t dport;         /* hostDestPort, host order (context.c:196) */
    uint16_t len;           /* payload bytes, <= 65491; forced to 0 without TCPCSUM_TXF_DATA */
    uint8_t flags;          /* TCPCSUM_TXF_* */
    uint8_t reserved0;
    uint64_t reserved1;
} tcpcsum_txseg_t;

/* mode: 0, or TCPCSUM_IPV4_IPHDR to also fill the IPv4 header checksum (the
 * reference leaves it 0 for the kernel, context.c:179). max_len: an upper
 * bound on the payload lengths (kernel shape only). d_check (nullable): the
 * TCP checks, also stored in the packets. Segments with len > 65491 are not
 * written (d_check = 0). Packets must not overlap; d_segs 16-B aligned. */
int tcpcsum_tx_build_dev(const void *d_payload, const tcpcsum_txseg_t *d_segs, uint64_t n, uint32_t max_len,
                         void *d_out_pkts, int mode, uint16_t *d_check, void *stream,
                         const tcpcsum_tuning_t *tune);

/* ------------------------------------------------------ host-memory batches
 * The path as the reference sees it: segments start and end in host memory
 * (raw-socket buffers). A context owns one device, one stream, pinned
 * staging and a few host copy threads (TCPCSUM_HOST_THREADS, default half the
 * CPUs the process may use, at most 8 — or, with LOCAL_WORLD_SIZE = k > 1 ranks
 * sharing the node's CPU quota, the rank's 1/k share; a staged wire batch of up
 * to 8 MiB copies on the calling thread alone, a bulk uniform copy on at most 4).
 * tcpcsum_ctx_destroy drains the stream and joins the copy threads before it
 * frees the context's HIP objects: call it while the HIP runtime is up (before
 * exit), as the Python front end's atexit hook does for contexts left open.
 * Host memory is used one of two ways:
 *   - memory its owner page-locked (tcpcsum_host_alloc / hipHostMalloc, or the
 *     application's own hipHostRegister) is read — FILL: written — in place by
 *     the kernel over PCIe (a uniform batch of 32 MiB or more goes to HBM by
 *     DMA from those pages first, 256 MiB at a time);
 *   - pageable memory is copied by the CPU threads into the context's pinned
 *     staging (uniform batches chunk by chunk — 16, 32, 64, then 128 MiB —
 *     each chunk's DMA to HBM and kernel overlapped with the copy of the
 *     next; wire batches only the packets' bytes), the kernel reads the
 *     staging, and FILL's checks are stored back into the caller's
 *     packets by the CPU. It is never page-locked.
 * All host calls are synchronous: they return when every result is in place. */
typedef struct tcpcsum_ctx tcpcsum_ctx_t;

/* scratch_bytes: pinned staging per pipeline slot for pageable uniform
 * batches, and the DMA piece for page-locked ones (0 = 128 MiB staging,
 * 256 MiB DMA pieces; page-locked batches under 32 MiB — two scratch_bytes
 * when given — are read in place). */
int tcpcsum_ctx_create(int device, size_t scratch_bytes, tcpcsum_ctx_t **out);
void tcpcsum_ctx_destroy(tcpcsum_ctx_t *ctx);

/* Launch shapes for this context's batches (NULL = built-in defaults). Only
 * this context is affected; other contexts and the device calls are not. */
int tcpcsum_ctx_set_tuning(tcpcsum_ctx_t *ctx, const tcpcsum_tuning_t *tune);

/* Context flags (0 = default). (ABI v3's TCPCSUM_CTX_AUTO_REGISTER = 1 is gone
 * with the registration calls: the value is refused.) */
/* Wait for the device by polling its completion between short sleeps instead
 * of HIP's spin in hipStreamSynchronize: the calling thread leaves its core
 * while the kernel runs, for a few microseconds more latency. */
#define TCPCSUM_CTX_BLOCKING_WAIT 2u
int tcpcsum_ctx_set_flags(tcpcsum_ctx_t *ctx, uint32_t flags);

/* Counters of what the context did (cumulative since creation). */
typedef struct tcpcsum_ctx_stats {
    uint64_t batches;            /* host batch calls */
    uint64_t pkts_in_place;      /* wire packets read / written in page-locked memory */
    uint64_t pkts_staged;        /* wire packets copied through pinned staging */
    uint64_t bytes_staged;       /* bytes copied into pinned staging (all host paths) */
    uint64_t copy_threads;       /* threads a staged wire batch (<= 8 MiB) copies on, caller included */
    uint64_t bulk_threads;       /* threads a staged uniform or large wire batch copies on */
    uint64_t ns_copy;            /* wall time spent copying into / out of staging (CPU) */
    uint64_t ns_wait;            /* wall time spent waiting for the device after the last launch */
    uint64_t ns_cpu_caller;      /* CPU time of the calling threads inside this context's host calls */
    uint64_t ns_cpu_workers;     /* CPU time of its copy threads since creation (copies, spin, wake-ups) */
    uint64_t gpu_numa_node;      /* the device's NUMA node (UINT64_MAX: unknown); staging and copy threads go there */
    uint64_t staging_numa_node;  /* where the pinned staging's first page lives (UINT64_MAX: none yet / unknown) */
} tcpcsum_ctx_stats_t;
int tcpcsum_ctx_get_stats(tcpcsum_ctx_t *ctx, tcpcsum_ctx_stats_t *out);

/* Page-locked host memory for packet pools — e.g. the loop's 1024 out-buffers
 * (loop.c:180-183) carved from one allocation: the host calls read and FILL it
 * in place over PCIe, with no copy. NULL on failure. */
void *tcpcsum_host_alloc(size_t bytes);
void tcpcsum_host_free(void *p);
/* The same, allocated for GPU `device` (its NUMA node; the calling thread's current
 * device is restored): one loop process per GPU (ABI v5). NULL on failure. */
void *tcpcsum_host_alloc_on(int device, size_t bytes);

/* 1 on a thread the library started (its copy threads), else 0 (ABI v5): an
 * allocator in front of the library (the interposer's arena) serves the
 * application's threads only. */
int tcpcsum_on_library_thread(void);

/* Uniform layout in host memory; h_out[i] as tcpcsum_batch_uniform_dev.
 * h_sum_start may be NULL (then sum_start is used for every segment).
 * Page-locked input is read in place; pageable input is staged (above). */
int tcpcsum_batch_uniform_host(tcpcsum_ctx_t *ctx, const void *h_base, uint64_t stride,
                               uint32_t len, const uint32_t *h_sum_start, uint32_t sum_start,
                               uint16_t *h_out, uint64_t n);

/* Wire layout in host memory: n packets at h_pkts + h_pkt_off[i] (offsets
 * within one host region of region_bytes; each header must lie inside it).
 * FILL patches check in place in host memory. A region that one page-locked
 * allocation covers (tcpcsum_host_alloc, or the application's own
 * hipHostRegister) is read in place; otherwise only the packets are copied
 * into staging. Results exactly as tcpcsum_ipv4_batch_dev. */
int tcpcsum_ipv4_batch_host(tcpcsum_ctx_t *ctx, void *h_pkts, size_t region_bytes,
                            const uint64_t *h_pkt_off, uint64_t n, uint32_t cap, int mode,
                            uint16_t *h_out, uint8_t *h_status);

/* Wire batch over the caller's own per-packet buffers (the reference's
 * layout: 1024 separately malloc'd 32 KiB out-buffers, loop.c:180-183, one
 * iov_base per message, loop.c:53-54): packet i at h_pkts[i] with h_lens[i]
 * readable bytes (results and status as tcpcsum_ipv4_batch_ptrs_dev). A
 * packet inside one page-locked allocation (tcpcsum_host_alloc, the
 * application's own hipHostRegister) is read and FILLed in place; any other is
 * copied into staging and its check stored back. Host batches store exactly the
 * 2-byte check (and, with IPHDR, the 2-byte IP header checksum) into the caller's
 * packets, as context.c:208 does; device batches may write the check's whole 128-B
 * line back (the bytes they read, check patched in), see TCPCSUM_TUNE_FILL_U16. */
int tcpcsum_ipv4_batch_ptrs_host(tcpcsum_ctx_t *ctx, void *const *h_pkts, const uint32_t *h_lens, uint64_t n,
                                 int mode, uint16_t *h_out, uint8_t *h_status);

/* ------------------------------------------------------ synthetic workload
 * Device-side generation of the SURVEY.md Appendix B batches, so benchmarks
 * start with inputs already resident in HBM (no H2D in the timed region). */

/* d_dst[k] = byte (off+k) of the Appendix B stream, k < nbytes. */
int tcpcsum_synth_fill_dev(void *d_dst, uint64_t stream_off, uint64_t nbytes, void *stream);

/* d_sum_start[k] = getPseudoHeaderSum(saddr(seg0+k), daddr(seg0+k), htons((u16)seg_len)). */
int tcpcsum_synth_pseudo_dev(uint32_t *d_sum_start, uint64_t seg0, uint64_t n, uint32_t seg_len,
                             void *stream);

/* ------------------------------------------------------ measurement helpers */

/* Read-only streaming probe: the chip's practical HBM read ceiling for the
 * checksum kernels' access pattern (16-B non-temporal loads, each wave
 * reading contiguous 1 KiB per instruction; by default one 4 KiB tile per
 * wave, tiles in XCD order, as the uniform kernel's plan), reported beside
 * them. With TCPCSUM_TUNE_PROBE_WRITE it also writes lines back (the wire
 * FILL's ceiling); d_src is then written (its bytes unchanged) and must be
 * writable. d_partials: TCPCSUM_PROBE_SLOTS u64 entries; the launch ADDS into
 * (since ABI v5; v4 overwrote per-block slots — zero them before reuse) the first *n_partials of them (wave w into slot w % TCPCSUM_PROBE_SLOTS),
 * so when they were zero, their sum on completion is the sum of the lo16+hi16
 * halves of every u32 word of d_src. nbytes multiple of 16, d_src 16-B aligned.
 * Tuning: unroll 0 / 1 / 2 / 4 = 4 / 8 / 16 / 32 chunks per lane per tile; for the
 * read-only probe, shape 2 or 3 = that many chunks, 10 / 11 / 12 = 32-lane groups
 * with 2 / 3 / 4 (tile-shape sweeps); max_blocks caps the grid. */
#define TCPCSUM_PROBE_SLOTS 8192
int tcpcsum_stream_probe_dev(const void *d_src, uint64_t nbytes, uint64_t *d_partials,
                             int *n_partials, void *stream, const tcpcsum_tuning_t *tune);

/* Host-side planning only (no device work): the kernel the library would use
 * for a uniform batch at device address base. mode: 0 = 16-B aligned, 1 =
 * 4-B aligned, 2 = byte-granular; shape: 0..8 = lane-group shapes covering
 * 4,8,16,32,64,96,128,256,512 chunks, 9 = one wave per long segment,
 * 10 / 11 = one / two lanes per segment (up to 5 / 8 chunks), 12 = flat
 * tiles (contiguous 1 KiB per load instruction; 1-32 KiB segments, 4-B
 * aligned, stride >= len), 13 = split segments (a workgroup of four waves
 * per segment, 4*unroll chunk loads per thread per round), 14 = a workgroup
 * per segment, segments taken XCD by XCD (unroll 1 / 2 / 4 / 8 = 16 waves x 4
 * loads, 8 x 8, 16 x 2, 4 x 16 per lane per round; 4- or 16-B aligned only);
 * unroll: segments in flight per lane group; max_blocks: resident grid
 * (1 << 24: one wave tile per wave, the grid rounded to whole XCD rounds and
 * the tiles taken XCD by XCD — the default for lane-group shapes, with a tile
 * of at most ~4.5 KiB). */
int tcpcsum_plan_uniform(uint64_t base, uint64_t stride, uint32_t len, uint64_t n,
                         const tcpcsum_tuning_t *tune, int *mode, int *shape, int *unroll, int *max_blocks);

/* tcpcsum_tuning_t.shape, read per entry point: uniform 0..14 (a forced shape
 * that cannot cover the segments is ignored), ragged 0..6 = (G,C) (4,1) (8,1) (16,1) (32,1) (32,3) (64,4) (64,8)
 * and 7..8 = balanced chunk space (4 / 8 loads per lane in flight; a nonzero
 * unroll u caps its tile at 64 / u segments),
 * wire 0..7 = (8,1) (32,3) (64,4) (16,2) (16,6) (8,12) (8,2) (8,4) and 8..9 =
 * balanced (4 / 8 loads per lane), builder 0..4. tcpcsum_tuning_t.flags: */
/* PIPE_* and NT_* take effect only in a library built with TUNING_VARIANTS=1 */
#define TCPCSUM_TUNE_PIPE_ON 1   /* software-pipelined tiles */
#define TCPCSUM_TUNE_PIPE_OFF 2
#define TCPCSUM_TUNE_NT_ON 4     /* non-temporal loads */
#define TCPCSUM_TUNE_NT_OFF 8
#define TCPCSUM_TUNE_BLOCKED 16  /* contiguous tile runs per wave (non-pipelined lane-group kernels) */
#define TCPCSUM_TUNE_WIRE_CACHED 32  /* wire: default-policy (not non-temporal) packet loads */
#define TCPCSUM_TUNE_WIN16 64    /* wire: 16-B (not 128-B) aligned packet windows */
#define TCPCSUM_TUNE_TX_NT_STORE 128  /* builder: non-temporal payload stores */
#define TCPCSUM_TUNE_FILL_DWORD 256   /* wire FILL: store check|urg_ptr as one dword when TCP+16 is 4-B aligned */
/* wire FILL: always the 2-byte store (default: where the 128-B line holding the check lies
 * inside the packet, the whole line is written back through, the check patched in) */
#define TCPCSUM_TUNE_FILL_U16 512
#define TCPCSUM_TUNE_TX_WT_STORE 1024  /* builder: payload stores written through (sc0 sc1 buffer stores) */
/* wire FILL: the 64-B block holding the checks written through instead of the 128-B line */
#define TCPCSUM_TUNE_FILL_HALF 2048
/* stream probe: also write back through (sc0 sc1) every shape-th 128-B line it reads, bytes
 * unchanged (shape 0: every 12th) — the wire FILL's traffic on 1536-B slots, without its work */
#define TCPCSUM_TUNE_PROBE_WRITE 4096
/* 0 if *tune is a valid tuning (NULL counts as valid), else TCPCSUM_EINVAL. */
int tcpcsum_tuning_check(const tcpcsum_tuning_t *tune);

#ifdef __cplusplus
}
#endif
#endif /* TCPCSUM_H */
