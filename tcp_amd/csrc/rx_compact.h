/* rx_compact.h — rx drop for the recvmmsg interposer (preload_mmsg.c): the
 * messages that passed GPU verification move to the front of the received
 * batch. Plain C, no GPU: tests/c/rx_compact_test.c runs it under ASan/UBSan.
 * struct mmsghdr needs _GNU_SOURCE before the first system header.
 */
#pragma once

#include <stddef.h>
#include <sys/socket.h>
#include <sys/uio.h>

/* Exchange two received messages for rx drop. The reference reads packet i of a
 * receive through its own iovec array, by index (getIpPacket, loop.c:96-100:
 * loop->iovecs[index].iov_base), not through the mmsghdr vector, so the data
 * must move with the iovec CONTENTS (buffer and length) — the vector's msg_iov
 * pointers stay where the caller put them. Length, flags, and the name and
 * control buffers (by pointer) travel with the data. by_entry: swap whole
 * vector entries instead — for a receive holding any message with several
 * iovecs, whose caller reads through the vector (one iovec cannot hold two). */
static inline void swap_msgs(struct mmsghdr *a, struct mmsghdr *b, int by_entry) {
    struct msghdr *x = &a->msg_hdr, *y = &b->msg_hdr;
    if (by_entry || x->msg_iov == y->msg_iov) {
        struct mmsghdr t = *a;
        *a = *b;
        *b = t;
        return;
    }
    struct iovec tv = x->msg_iov[0];
    x->msg_iov[0] = y->msg_iov[0];
    y->msg_iov[0] = tv;
    unsigned int tl = a->msg_len;
    a->msg_len = b->msg_len;
    b->msg_len = tl;
    int tf = x->msg_flags;
    x->msg_flags = y->msg_flags;
    y->msg_flags = tf;
    void *tn = x->msg_name;
    socklen_t tnl = x->msg_namelen;
    x->msg_name = y->msg_name;
    x->msg_namelen = y->msg_namelen;
    y->msg_name = tn;
    y->msg_namelen = tnl;
    void *tc = x->msg_control;
    size_t tcl = x->msg_controllen;
    x->msg_control = y->msg_control;
    x->msg_controllen = y->msg_controllen;
    y->msg_control = tc;
    y->msg_controllen = tcl;
}

/* Whether a receive of n messages must be reordered by whole vector entries:
 * some message has other than exactly one iovec. */
static inline int rx_by_entry(const struct mmsghdr *vec, unsigned int n) {
    for (unsigned int i = 0; i < n; ++i)
        if (vec[i].msg_hdr.msg_iovlen != 1) return 1;
    return 0;
}

/* Messages [done, done + cnt) of vec were verified; keep[i] says whether message
 * done + i passed. The passing ones move, in arrival order, to positions
 * kept, kept + 1, ... (kept <= done: the passing messages of earlier chunks
 * already sit below it); the failing ones end up behind them. by_entry: from
 * rx_by_entry over the whole receive. Returns the new count of passing messages. */
static inline unsigned int rx_keep_passing(struct mmsghdr *vec, unsigned int kept, unsigned int done,
                                           unsigned int cnt, const unsigned char *keep, int by_entry) {
    for (unsigned int i = 0; i < cnt; ++i) {
        if (!keep[i]) continue;
        if (kept != done + i) swap_msgs(&vec[kept], &vec[done + i], by_entry);
        ++kept;
    }
    return kept;
}
