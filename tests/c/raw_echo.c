/*
 * raw_echo.c — the plumbing configuration (BASELINE configs[0]: the reference's
 * stress server echoing 1500-byte-MTU segments over loopback) rebuilt from the
 * reference's own socket layer, without the reference:
 *
 *   server  rx: socket(AF_INET, SOCK_RAW, IPPROTO_TCP), recvmmsg of up to 1024
 *               IP packets per call into 32 KiB buffers (loop.c:22-25, :155-200)
 *           tx: socket(AF_INET, SOCK_RAW, IPPROTO_RAW); every echo is framed as
 *               us_internal_socket_context_send_packet frames it
 *               (context.c:169-206: ihl 5, id = (u16)htonl(54321), ttl 255, doff 6,
 *               window-scale option 03 03 05 00, window 8192, ACK|PSH, payload
 *               copied at :190) with check = 0 (:182), queued in separately
 *               malloc'd 32 KiB out-buffers (loop.c:180-183) and flushed with ONE
 *               sendmmsg per round (releaseSend, loop.c:27-94) — stress.c's on_data
 *               echo (stress.c:20-24 -> us_socket_write -> send_packet).
 *   client  1456-byte data segments 45001 -> 4000 (1500-byte IP packets) sent with
 *           sendto on its own IPPROTO_RAW socket, checks by the CPU path
 *           (tcpcsum_continue == csum_continue) — not interposed.
 *
 * Run under LD_PRELOAD=libtcpcsum_preload.so in its DEFAULT mode (SOCK_RAW
 * sockets only): the GPU fills the echo checks at the server's sendmmsg and,
 * with TCPCSUM_PRELOAD_RX=verify, verifies every batch the server's recvmmsg
 * returns — client segments, the echoes themselves (the rx socket sniffs lo)
 * and the kernel's own RSTs (no listener owns these ports), which loopback
 * leaves CHECKSUM_PARTIAL (counted apart).
 *
 *   raw_echo <nsegs> <out-file> [cpu]
 * cpu: the server fills each check on the CPU as the reference does (the
 * plumbing config exactly, no GPU); otherwise checks are left 0 for the
 * interposer to fill. Needs CAP_NET_RAW: it first moves itself into a fresh user + network
 * namespace (unshare(2) in-process, so the dynamic loader and LD_PRELOAD are
 * untouched; an ordinary user is root there), brings that namespace's lo up,
 * and runs there — nothing else on the host sees the traffic. Exit 0 ok; 77
 * no way to raw sockets (no user namespaces, not root); 3 send failed; 4 recv failed;
 * 5 echoes missing. Writes, per echo: u32 length + the packet as built (check
 * 0), u32 length + the packet as sniffed. Prints one JSON summary line.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <net/if.h>
#include <sched.h>
#include <netinet/in.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "tcpcsum.h"

enum { SLOT = 32768, VLEN = 1024, PAYLOAD = 1456, ROUND = 256 };
enum { CLIENT_PORT = 45001, SERVER_PORT = 4000 };

static uint64_t rng = 0x452821E638D01377ull;
static uint32_t next32(void) {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (uint32_t) (rng >> 16);
}

static int write_file(const char *path, const char *text) {
    int fd = open(path, O_WRONLY);
    if (fd < 0) return -1;
    ssize_t n = write(fd, text, strlen(text));
    close(fd);
    return n == (ssize_t) strlen(text) ? 0 : -1;
}

/* A private network namespace: as an ordinary user through a new user
 * namespace (mapping us to its root), else directly when already root. */
static const char *enter_netns(void) {
    const unsigned uid = (unsigned) getuid(), gid = (unsigned) getgid();
    if (unshare(CLONE_NEWUSER | CLONE_NEWNET) == 0) {
        char m[64];
        (void) write_file("/proc/self/setgroups", "deny");
        snprintf(m, sizeof m, "0 %u 1", uid);
        if (write_file("/proc/self/uid_map", m)) return "user+net (uid_map failed)";
        snprintf(m, sizeof m, "0 %u 1", gid);
        (void) write_file("/proc/self/gid_map", m);
        return "user+net";
    }
    if (unshare(CLONE_NEWNET) == 0) return "net";
    return "none";
}

static void lo_up(void) {
    int s = socket(AF_INET, SOCK_DGRAM, 0);
    struct ifreq ifr;
    memset(&ifr, 0, sizeof ifr);
    strcpy(ifr.ifr_name, "lo");
    if (ioctl(s, SIOCGIFFLAGS, &ifr) == 0 && !(ifr.ifr_flags & IFF_UP)) {
        ifr.ifr_flags |= IFF_UP | IFF_RUNNING;
        (void) ioctl(s, SIOCSIFFLAGS, &ifr);
    }
    close(s);
}

/* IPv4 + TCP header as context.c:169-206 writes them; check left 0 (:182). */
static size_t frame(uint8_t *b, uint32_t saddr, uint32_t daddr, uint16_t sport, uint16_t dport, uint32_t seq,
                    uint32_t ack, const uint8_t *data, size_t len) {
    const size_t tot = 20 + 24 + len;
    memset(b, 0, 44);
    b[0] = 0x45;
    b[2] = (uint8_t) (tot >> 8); b[3] = (uint8_t) tot;
    const uint32_t id = htonl(54321);
    memcpy(b + 4, &id, 2);                      /* the u16 field keeps the low half */
    b[8] = 255; b[9] = IPPROTO_TCP;
    memcpy(b + 12, &saddr, 4); memcpy(b + 16, &daddr, 4);
    uint8_t *t = b + 20;
    t[0] = (uint8_t) (sport >> 8); t[1] = (uint8_t) sport;
    t[2] = (uint8_t) (dport >> 8); t[3] = (uint8_t) dport;
    const uint32_t s = htonl(seq), a = htonl(ack);
    memcpy(t + 4, &s, 4); memcpy(t + 8, &a, 4);
    t[12] = 6 << 4;                             /* doff 6 */
    t[13] = 0x10 | (data ? 0x08 : 0);           /* ACK, PSH with data */
    t[14] = 8192 >> 8;                          /* window */
    t[20] = 3; t[21] = 3; t[22] = 5; t[23] = 0; /* window scale */
    if (data) memcpy(t + 24, data, len);
    return tot;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s nsegs out-file [cpu]\n", argv[0]); return 2; }
    const int nsegs = atoi(argv[1]);
    /* cpu: the server computes each echo's check itself, as the reference does
     * (context.c:208-209, csum_continue on the CPU) — BASELINE configs[0] as is */
    const int cpu_checks = argc > 3 && !strcmp(argv[3], "cpu");
    FILE *f = fopen(argv[2], "wb");
    if (!f || nsegs <= 0) return 2;
    const char *ns = enter_netns();
    lo_up();
    const int rx = socket(AF_INET, SOCK_RAW | SOCK_NONBLOCK, IPPROTO_TCP);
    const int tx = socket(AF_INET, SOCK_RAW, IPPROTO_RAW);
    const int cl = socket(AF_INET, SOCK_RAW, IPPROTO_RAW);
    if (rx < 0 || tx < 0 || cl < 0) {
        printf("{\"error\": \"raw sockets: %s\", \"namespace\": \"%s\"}\n", strerror(errno), ns);
        return 77;
    }
    int big = 64 << 20;
    setsockopt(rx, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    /* loop.c:180-183: in and out buffers, 32 KiB each, malloc'd alternately */
    static uint8_t *inbuf[VLEN], *outbuf[VLEN];
    for (int i = 0; i < VLEN; ++i) {
        inbuf[i] = malloc(SLOT);
        outbuf[i] = malloc(SLOT);
    }
    static struct iovec riov[VLEN], tiov[VLEN];
    static struct mmsghdr rmsg[VLEN], tmsg[VLEN];
    static struct sockaddr_in tsin[VLEN];
    for (int i = 0; i < VLEN; ++i) {
        riov[i].iov_base = inbuf[i];
        riov[i].iov_len = SLOT;
        rmsg[i].msg_hdr.msg_iov = &riov[i];
        rmsg[i].msg_hdr.msg_iovlen = 1;
    }
    const uint32_t lo_addr = htonl(0x7F000001u);
    uint8_t *cpkt = malloc(SLOT), *payload = malloc(PAYLOAD);
    uint8_t **built = calloc((size_t) nsegs, sizeof *built);
    size_t *blen = calloc((size_t) nsegs, sizeof *blen);
    long echoes = 0, client_seen = 0, kernel_rst = 0, other = 0, send_calls = 0, batches_rx = 0;
    uint32_t cseq = 1000, sseq = 846930886;   /* the reference's first ISN (unseeded rand) */
    int sent = 0, queued_total = 0;
    const double t_start = now_s();
    double deadline = now_s() + 60.0;
    while (echoes < nsegs && now_s() < deadline) {
        /* client: a round of data segments 45001 -> 4000, CPU checks */
        int burst = 0;
        for (; burst < ROUND && sent < nsegs; ++burst, ++sent) {
            for (int k = 0; k < PAYLOAD; ++k) payload[k] = (uint8_t) next32();
            const size_t tot = frame(cpkt, lo_addr, lo_addr, CLIENT_PORT, SERVER_PORT, cseq, sseq, payload, PAYLOAD);
            cseq += PAYLOAD;
            const uint16_t c = tcpcsum_continue(tcpcsum_pseudo(lo_addr, lo_addr, htons(24 + PAYLOAD)),
                                                (const char *) cpkt + 20, 24 + PAYLOAD);
            memcpy(cpkt + 36, &c, 2);
            struct sockaddr_in d = {0};
            d.sin_family = AF_INET;
            d.sin_addr.s_addr = lo_addr;
            if (sendto(cl, cpkt, tot, 0, (struct sockaddr *) &d, sizeof d) != (ssize_t) tot) {
                printf("{\"error\": \"client sendto: %s\"}\n", strerror(errno));
                return 3;
            }
        }
        /* server: read batches, echo every client data segment of this round in one flush */
        int queued = 0;
        const double round_deadline = now_s() + 5.0;
        while ((queued < burst || burst == 0) && now_s() < round_deadline) {
            int r = recvmmsg(rx, rmsg, VLEN, 0, NULL);
            if (r < 0) {
                if (errno == EAGAIN || errno == EWOULDBLOCK) {
                    if (burst == 0) break;
                    usleep(100);
                    continue;
                }
                printf("{\"error\": \"recvmmsg: %s\"}\n", strerror(errno));
                return 4;
            }
            ++batches_rx;
            for (int i = 0; i < r; ++i) {
                const uint8_t *ip = inbuf[i];
                const unsigned int n = rmsg[i].msg_len;
                if (n < 40) { ++other; continue; }
                const unsigned int ihl = (ip[0] & 15u) * 4u;
                const uint8_t *t = ip + ihl;
                const unsigned int sport = (t[0] << 8) | t[1], dport = (t[2] << 8) | t[3];
                const unsigned int tot = (ip[2] << 8) | ip[3];
                const unsigned int doff = (t[12] >> 4) * 4u;
                const unsigned int dlen = tot - ihl - doff;
                if (t[13] & 0x04) { ++kernel_rst; continue; }
                if (sport == CLIENT_PORT && dport == SERVER_PORT && dlen > 0) {
                    ++client_seen;
                    /* stress.c on_data: echo it back -> send_packet framing, check 0 */
                    uint32_t cs;
                    memcpy(&cs, t + 4, 4);
                    uint8_t *o = outbuf[queued];
                    const size_t ot = frame(o, lo_addr, lo_addr, SERVER_PORT, CLIENT_PORT, sseq,
                                            ntohl(cs) + dlen, t + doff, dlen);
                    sseq += dlen;
                    if (cpu_checks) {
                        const uint16_t c = tcpcsum_continue(
                            tcpcsum_pseudo(lo_addr, lo_addr, htons((uint16_t) (24 + dlen))),
                            (const char *) o + 20, (int) (24 + dlen));
                        memcpy(o + 36, &c, 2);
                    }
                    const int k = queued_total + queued;
                    if (k < nsegs) {
                        built[k] = malloc(ot);
                        memcpy(built[k], o, ot);
                        blen[k] = ot;
                    }
                    tiov[queued].iov_base = o;
                    tiov[queued].iov_len = ot;          /* = tot_len, loop.c:47,54 */
                    tsin[queued].sin_family = AF_INET;
                    tsin[queued].sin_addr.s_addr = lo_addr;
                    tmsg[queued].msg_hdr.msg_iov = &tiov[queued];
                    tmsg[queued].msg_hdr.msg_iovlen = 1;
                    tmsg[queued].msg_hdr.msg_name = &tsin[queued];
                    tmsg[queued].msg_hdr.msg_namelen = sizeof tsin[queued];
                    ++queued;
                } else if (sport == SERVER_PORT && dport == CLIENT_PORT && dlen > 0) {
                    /* an echo sniffed on lo: record it against what was built */
                    if (echoes < nsegs && blen[echoes]) {
                        uint32_t a = (uint32_t) blen[echoes], b = n;
                        fwrite(&a, 4, 1, f); fwrite(built[echoes], 1, a, f);
                        fwrite(&b, 4, 1, f); fwrite(ip, 1, b, f);
                    }
                    ++echoes;
                } else {
                    ++other;
                }
            }
        }
        if (queued) {   /* releaseSend: one sendmmsg for the round (loop.c:75) */
            int done = 0;
            while (done < queued) {
                int s = sendmmsg(tx, tmsg + done, (unsigned) (queued - done), 0);
                ++send_calls;
                if (s < 0) {
                    printf("{\"error\": \"server sendmmsg: %s\"}\n", strerror(errno));
                    return 3;
                }
                done += s;
            }
            queued_total += queued;
        }
        if (sent >= nsegs && queued == 0 && burst == 0) {
            /* drain the remaining echoes */
            int r = recvmmsg(rx, rmsg, VLEN, 0, NULL);
            if (r <= 0) usleep(200);
            else {
                ++batches_rx;
                for (int i = 0; i < r; ++i) {
                    const uint8_t *ip = inbuf[i];
                    const unsigned int n = rmsg[i].msg_len;
                    if (n < 40) { ++other; continue; }
                    const uint8_t *t = ip + (ip[0] & 15u) * 4u;
                    const unsigned int sport = (t[0] << 8) | t[1], dport = (t[2] << 8) | t[3];
                    if (t[13] & 0x04) { ++kernel_rst; continue; }
                    if (sport == SERVER_PORT && dport == CLIENT_PORT && n > 44) {
                        if (echoes < nsegs && blen[echoes]) {
                            uint32_t a = (uint32_t) blen[echoes], b = n;
                            fwrite(&a, 4, 1, f); fwrite(built[echoes], 1, a, f);
                            fwrite(&b, 4, 1, f); fwrite(ip, 1, b, f);
                        }
                        ++echoes;
                    } else {
                        ++other;
                    }
                }
            }
        }
    }
    fclose(f);
    printf("{\"namespace\": \"%s\", \"server_checks\": \"%s\", \"segments\": %d, \"client_seen\": %ld, \"echoed\": %d, \"echoes_sniffed\": %ld, \"kernel_rst\": %ld, "
           "\"other\": %ld, \"send_calls\": %ld, \"rx_batches\": %ld, \"seconds\": %.3f}\n",
           ns, cpu_checks ? "cpu" : "left 0", nsegs, client_seen, queued_total, echoes, kernel_rst, other, send_calls, batches_rx, now_s() - t_start);
    return echoes >= nsegs ? 0 : 5;
}
