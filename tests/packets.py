"""Build raw IPv4/TCP packets the way the reference's segment builder does.

Layout follows /root/reference/context.c:169-206 (us_internal_socket_context_send_packet):
IPv4 header (ihl=5, version 4, tot_len, id, ttl 255, protocol 6, saddr, daddr;
IP checksum left 0 as at :179), then struct TcpHeader (Packets.h:46-50): a
20-byte struct tcphdr with doff=6, flags, window 8192 and check = 0 (:182),
plus options 03 03 05 00 (:199-202), then the payload (:190).

Used by the tests to make wire batches; the tests may also add IP options
(ihl > 5), odd packet offsets and malformed packets.
"""
import socket
import struct

import numpy as np


def tcp_segment(rng, payload_len, sport=4000, dport=45001, flags=0x18):
    seq = int(rng.integers(0, 2**32))
    ack = int(rng.integers(0, 2**32))
    hdr = struct.pack("!HHII", sport, dport, seq, ack)
    hdr += bytes([6 << 4, flags])                 # doff=6, flags (little-endian bitfields)
    hdr += struct.pack("!H", 8192) + b"\0\0" + b"\0\0"   # window, check=0, urg_ptr
    hdr += bytes([3, 3, 5, 0])                    # window-scale option
    return hdr + rng.integers(0, 256, payload_len, dtype=np.uint8).tobytes()


def ip_packet(rng, payload_len, saddr=None, daddr=None, ihl=5, version=4, proto=6, tot_len_delta=0):
    tcp = tcp_segment(rng, payload_len)
    opts = b"\x01" * (4 * (ihl - 5)) if ihl > 5 else b""
    tot = 4 * max(ihl, 5) + len(tcp) + tot_len_delta
    sa = saddr if saddr is not None else int(rng.integers(0, 2**32))
    da = daddr if daddr is not None else int(rng.integers(0, 2**32))
    ip = bytes([(version << 4) | ihl, 0]) + struct.pack("!HHHBBH", tot & 0xFFFF, 54321 & 0xFFFF, 0, 255, proto, 0)
    ip += struct.pack("<II", sa, da)   # stored as-is (network order bytes)
    return ip + opts + tcp


def build_batch(rng, n, slot=32768, malformed=False, odd_offsets=False, max_payload=1456, align=0,
                control_every=0):
    """A region of n packets. Returns (region uint8 array, offsets uint64, payload lengths).
    align > 0: packed, every packet starting at a multiple of `align` (plus 0..2 more of it);
    control_every = k: every k-th packet has no payload (a 44-B control segment)."""
    pkts, lens = [], []
    for i in range(n):
        pl = int(rng.integers(0, max_payload + 1))
        if control_every and i % control_every == 0:
            pl = 0
        kind = i % 11 if malformed else 0
        if kind == 3:
            p = ip_packet(rng, pl, version=6)
        elif kind == 5:
            p = ip_packet(rng, pl, proto=17)
        elif kind == 7:
            p = ip_packet(rng, pl, ihl=4)
        elif kind == 8:
            p = ip_packet(rng, pl, ihl=15)          # valid, longest IP options (check at byte 76)
        elif kind == 9:
            p = ip_packet(rng, pl, ihl=7)           # valid, with IP options
        elif kind == 10:
            p = ip_packet(rng, pl, tot_len_delta=-30)   # tot_len too small for the TCP header? still >= ihl*4+20
        else:
            p = ip_packet(rng, pl)
        pkts.append(p)
        lens.append(pl)
    offs = []
    pos = 0
    for i, p in enumerate(pkts):
        if align:
            pos = (pos + align - 1) // align * align + align * int(rng.integers(0, 3))
        elif odd_offsets:
            pos += int(rng.integers(0, 7))
        else:
            pos = i * slot
        offs.append(pos)
        if odd_offsets or align:
            pos += len(p)
    size = (offs[-1] + len(pkts[-1]) + 64) if (odd_offsets or align) else n * slot
    region = np.zeros(size, np.uint8)
    for o, p in zip(offs, pkts):
        region[o:o + len(p)] = np.frombuffer(p, np.uint8)
    return region, np.array(offs, np.uint64), np.array(lens)


def htons(x):
    return socket.htons(x)
