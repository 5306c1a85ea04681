/*
 * scalar_dropin.c — the synchronous single-segment entry points of
 * include/tcpcsum.h (tcpcsum_pseudo, tcpcsum_continue).
 *
 * These exist so a caller can replace the reference's two file-static helpers
 * one for one where it needs a result immediately (context.c:208-209 for a
 * lone SYN-ACK or retransmit, context.c:94). They run on the calling thread.
 * No batch entry point calls them: every batch is checksummed by the gfx950
 * kernels in tcpcsum_kernels.hip.
 *
 *   tcpcsum_pseudo   == getPseudoHeaderSum  /root/reference/context.c:104-119
 *   tcpcsum_continue == csum_continue       /root/reference/context.c:121-145
 */
#include <stdint.h>
#include <string.h>

#include "tcpcsum.h"

/* Six native-order u16 words of {saddr, daddr, 0, IPPROTO_TCP, len_be}; on a
 * little-endian host the zero/protocol word reads as 0x0600. */
unsigned long tcpcsum_pseudo(uint32_t saddr_be, uint32_t daddr_be, uint16_t len_be) {
    return (unsigned long) (saddr_be & 0xffffu) + (saddr_be >> 16) + (daddr_be & 0xffffu) +
           (daddr_be >> 16) + 0x0600u + len_be;
}

/* Exact 64-bit word sum; odd trailing byte as a low byte; two folds; ~. */
unsigned short tcpcsum_continue(unsigned long sum_start, const char *p, int nbytes) {
    int64_t sum = (int64_t) sum_start;
    const unsigned char *q = (const unsigned char *) p;
    for (; nbytes > 1; nbytes -= 2, q += 2) sum += (int64_t) (q[0] | ((unsigned) q[1] << 8));
    if (nbytes == 1) sum += q[0];
    sum = (sum >> 16) + (sum & 0xffff);
    sum = sum + (sum >> 16);
    return (unsigned short) ~sum;
}
