/* rx_compact_test.c — the interposer's rx drop (tcp_amd/csrc/rx_compact.h) on
 * the CPU, under ASan/UBSan (tests/test_sanitize.py). A receive of N messages,
 * laid out as the reference lays them out: one iovec per message in the loop's
 * own array (loop.c:190-194), read back by index (getIpPacket, loop.c:96-100).
 * After the drop, position i of that array holds the i-th passing message —
 * its bytes, its msg_len and its sender — every buffer is still referenced
 * exactly once, and the vector's msg_iov pointers are where the caller put them.
 * A receive holding a message with two iovecs is reordered by whole vector
 * entries instead (read through the vector). Chunks of 7 messages at a time, as
 * the interposer verifies batches of <= 1024.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../tcp_amd/csrc/rx_compact.h"

#define N 61
#define CHUNK 7

static int fail(const char *what, int i) {
    printf("rx_compact_test: FAIL %s at %d\n", what, i);
    return 1;
}

static int run(int pattern, int multi) {
    static unsigned char buf[N][64];
    static struct sockaddr_storage name[N];
    struct iovec iov[N], iov2[2];
    struct mmsghdr vec[N];
    unsigned char keep_all[N];
    memset(vec, 0, sizeof vec);
    for (int k = 0; k < N; ++k) {
        memset(buf[k], k, sizeof buf[k]);
        iov[k].iov_base = buf[k];
        iov[k].iov_len = sizeof buf[k];
        vec[k].msg_hdr.msg_iov = &iov[k];
        vec[k].msg_hdr.msg_iovlen = 1;
        vec[k].msg_hdr.msg_name = &name[k];
        vec[k].msg_hdr.msg_namelen = (socklen_t) (16 + k % 3);
        memset(&name[k], 0, sizeof name[k]);
        ((unsigned char *) &name[k])[0] = (unsigned char) k;
        vec[k].msg_len = 100u + (unsigned) k;
        vec[k].msg_hdr.msg_flags = k;
        keep_all[k] = pattern == 0 ? (k % 3 != 1) : pattern == 1 ? 0 : pattern == 2 ? 1 : (k >= N / 2);
    }
    if (multi) {   /* a message with two iovecs (SKIPPED by the GPU pass, so kept) */
        iov2[0].iov_base = buf[5];
        iov2[0].iov_len = 32;
        iov2[1].iov_base = buf[5] + 32;
        iov2[1].iov_len = 32;
        vec[5].msg_hdr.msg_iov = iov2;
        vec[5].msg_hdr.msg_iovlen = 2;
        keep_all[5] = 1;
    }
    const int by_entry = rx_by_entry(vec, N);
    if (by_entry != multi) return fail("by_entry", by_entry);
    unsigned int kept = 0;
    for (unsigned int done = 0; done < N; done += CHUNK) {
        const unsigned int cnt = N - done < CHUNK ? N - done : CHUNK;
        kept = rx_keep_passing(vec, kept, done, cnt, keep_all + done, by_entry);
    }
    int want[N], nw = 0;
    for (int k = 0; k < N; ++k)
        if (keep_all[k]) want[nw++] = k;
    if ((int) kept != nw) return fail("count", (int) kept);
    int seen[N];
    memset(seen, 0, sizeof seen);
    for (int i = 0; i < N; ++i) {
        const struct msghdr *h = &vec[i].msg_hdr;
        /* the reference's by-index read; a receive with a scatter-gather message is
         * reordered by vector entries, and its caller reads through the vector */
        const unsigned char *b = multi ? (const unsigned char *) h->msg_iov[0].iov_base
                                       : (const unsigned char *) iov[i].iov_base;
        const int id = b[0];
        if (id < 0 || id >= N || seen[id]++) return fail("buffer referenced twice or lost", i);
        if (!multi && h->msg_iov != &iov[i]) return fail("msg_iov pointer moved", i);
        if (vec[i].msg_len != 100u + (unsigned) id) return fail("msg_len did not travel", i);
        if (h->msg_flags != id) return fail("msg_flags did not travel", i);
        if (((const unsigned char *) h->msg_name)[0] != id || h->msg_namelen != (socklen_t) (16 + id % 3))
            return fail("sender did not travel", i);
        if (i < nw && id != want[i]) return fail("passing message out of order", i);
        if (i >= nw && keep_all[id]) return fail("passing message behind the count", i);
    }
    return 0;
}

int main(void) {
    for (int pattern = 0; pattern < 4; ++pattern)
        for (int multi = 0; multi < 2; ++multi)
            if (run(pattern, multi)) return 1;
    printf("rx_compact_test: OK\n");
    return 0;
}
