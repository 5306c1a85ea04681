/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the uNetworking/tcp checksum hot path, used as the parity
 * checker for the HIP path (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg). Nothing in tcp_amd/ links, loads or calls this code.
 *
 * Pinned against:
 *   - SURVEY.md Appendix A known-answer tests (computed by the reference),
 *   - SURVEY.md Appendix B digests (computed by the reference's own
 *     csum_continue over the synthetic configs in the survey session).
 * A build of the reference itself (oracle/_ref) is not available: see
 * DESIGN.md "Oracle and parity pin".
 */
#ifndef TCPCSUM_ORACLE_H
#define TCPCSUM_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* context.c:104-119 getPseudoHeaderSum(saddr, daddr, tcpLength). */
unsigned long oracle_pseudo(uint32_t saddr_be, uint32_t daddr_be, uint16_t len_be);

/* context.c:121-145 csum_continue(sumStart, p, nbytes). */
unsigned short oracle_csum_continue(unsigned long sum_start, const char *p, int nbytes);

/* SURVEY.md Appendix B synthetic generator. */
uint64_t oracle_mix64(uint64_t z);
void oracle_gen_stream(uint8_t *dst, uint64_t stream_off, uint64_t nbytes);
uint32_t oracle_saddr(uint64_t seg);   /* htonl(0x0A000000 | (i & 0xFFFFFF)) */
uint32_t oracle_daddr(uint64_t seg);   /* htonl(0xC0A80000 | ((i*7) & 0xFFFF)) */

/* out[k] for segments seg0..seg0+n-1 of length L of the Appendix B stream,
 * generated on the fly (never materialised), nthreads pthreads. */
int oracle_synth_batch(uint64_t seg0, uint64_t n, uint32_t seg_len,
                       uint16_t *out, int nthreads);

/* Ragged batch: segment k = base[off[k] .. off[k]+len[k]), sum_start[k]. */
void oracle_batch_desc(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                       const uint32_t *sum_start, uint64_t n, uint16_t *out);

/* Wire batch: IPv4 packets at base + off[k]. mode 0 = fill (check treated as
 * 0, result written to check and out), mode 1 = verify (out = csum incl.
 * check; 0 == valid); | 2 = also the IPv4 header checksum (fill at IP+10 /
 * verify). status[k]: 0 ok, 1 not IPv4/TCP or malformed, |2 IP header bad,
 * |4 verify found a CHECKSUM_PARTIAL check (un-complemented pseudo sum). */
void oracle_ipv4_batch(uint8_t *base, const uint64_t *off, uint64_t n, uint32_t cap,
                       int mode, uint16_t *out, uint8_t *status);

/* context.c:150-213 segment builder (minus the drop and the trace) for a
 * batch: layout-identical to tcpcsum_txseg_t (48 bytes). iphdr: also fill the
 * IPv4 header checksum. checks (nullable) receives the TCP checks. */
typedef struct oracle_txseg {
    uint64_t payload_off, out_off;
    uint32_t saddr_be, daddr_be, seq, ack;
    uint16_t sport, dport, len;
    uint8_t flags, reserved0;
    uint64_t reserved1;
} oracle_txseg_t;
void oracle_tx_build(const uint8_t *payload, const oracle_txseg_t *segs, uint64_t n, uint8_t *out, int iphdr,
                     uint16_t *checks);

/* Digests of SURVEY.md Appendix B: fnv1a64 over out[] as LE u16 bytes. */
void oracle_digest(const uint16_t *out, uint64_t n, uint64_t *fnv, uint64_t *sum,
                   uint16_t *xr);

/* CPU throughput harness (CLOCK_MONOTONIC, pthreads, contiguous shards).
 * Times the checksum of nseg synthetic segments of seg_len bytes held in
 * host memory, pseudo-header sum computed per segment as context.c:208 does.
 * Repeats passes until min_seconds elapsed (>= 5 passes, persistent threads,
 * each pass timed from before the start barrier releases the workers to
 * after the last one finishes); returns the best pass in GiB/s, the fnv1a64
 * digest of the outputs, the summed duration of all passes (mean rate =
 * passes * bytes / total) and the median pass in GiB/s. */
double oracle_cpu_bench(int nthreads, uint32_t seg_len, uint64_t nseg, double min_seconds,
                        uint64_t *digest_out, int *passes_out, double *total_out, double *median_out);

#ifdef __cplusplus
}
#endif
#endif
