"""BASELINE configs[0] (the plumbing config) replayed from a committed capture.

tests/golden/plumbing_echoes.npz holds 256 echoes of 1456-byte payloads as they
crossed loopback in the plumbing configuration (tests/golden/make_plumbing_fixture.py):
framed as /root/reference/context.c:169-206 frames a segment, TCP check filled by
the CPU path of context.c:208-209, IPv4 id and header checksum filled by the
kernel for the IPPROTO_RAW send. Raw sockets are impossible on the GPU pool, so
the GPU side of that configuration runs here on the captured bytes: each echo is
put in its own 32 KiB out-buffer (loop.c:180-183), both checksums are zeroed as
context.c:182 (and the kernel) leave them, and the GPU's FILL at the sendmmsg
seam must reproduce the captured wire bytes exactly — then VERIFY them to 0.
"""
import os

import numpy as np
import pytest

import oracle

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "plumbing_echoes.npz")


def echoes():
    z = np.load(FIXTURE)   # allow_pickle defaults to False: plain arrays only
    wire, off, ln = z["wire"], z["off"], z["length"]
    return [wire[int(o):int(o) + int(n)].copy() for o, n in zip(off, ln)]


def zeroed(pkt: np.ndarray) -> np.ndarray:
    """The packet as send_packet leaves it before the checksum (context.c:182: check = 0) and before
    the kernel fills the IPv4 header checksum."""
    p = pkt.copy()
    p[10:12] = 0
    ihl = (int(p[0]) & 15) * 4
    p[ihl + 16:ihl + 18] = 0
    return p


def test_fixture_is_the_reference_framing():
    """Every captured echo is a 1500-B IPv4/TCP packet framed as context.c:169-206: ihl 5, ttl 255,
    TCP, doff 6, window-scale option 03 03 05 00, window 8192, ACK|PSH, 4000 -> 45001."""
    e = echoes()
    assert len(e) == 256
    for p in e:
        assert p.size == 1500 and p[0] == 0x45 and (int(p[2]) << 8 | int(p[3])) == 1500
        assert p[8] == 255 and p[9] == 6
        t = p[20:]
        assert (int(t[0]) << 8 | int(t[1])) == 4000 and (int(t[2]) << 8 | int(t[3])) == 45001
        assert t[12] >> 4 == 6 and t[13] == 0x18 and (int(t[14]) << 8 | int(t[15])) == 8192
        assert list(t[20:24]) == [3, 3, 5, 0]


def test_oracle_reproduces_captured_checks():
    """The oracle's FILL (TCP check, and the IPv4 header checksum the kernel wrote) of each zeroed
    echo reproduces the captured bytes exactly, and VERIFY gives 0."""
    for p in echoes():
        region = np.concatenate([zeroed(p), np.zeros(16, np.uint8)])
        out, st = oracle.ipv4_batch(region, np.array([0], np.uint64), 65535, 0 | 2)
        assert st[0] == 0
        assert np.array_equal(region[:p.size], p)
        v, vs = oracle.ipv4_batch(np.concatenate([p, np.zeros(16, np.uint8)]), np.array([0], np.uint64), 65535, 1 | 2)
        assert vs[0] == 0 and v[0] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["staged", "in_place", "region", "device"])
def test_plumbing_fill_on_gpu(path):
    """The plumbing config's checksum work on the GPU: the 256 captured echoes, zeroed, each in its
    own 32 KiB out-buffer (the loop's layout) — FILL|IPHDR through tcpcsum_ipv4_batch_ptrs_host (staged:
    pageable malloc'd buffers; in_place: the pool from tcpcsum_host_alloc, INTEGRATION.md level 2),
    through the region host path over one pool, or on device — reproduces the captured wire bytes
    exactly; VERIFY|IPHDR then gives 0."""
    torch = pytest.importorskip("torch")
    import tcp_amd
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    caps = echoes()
    mode_fill = tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR
    mode_verify = tcp_amd.IPV4_VERIFY | tcp_amd.IPV4_IPHDR
    if path in ("staged", "in_place"):
        pool = tcp_amd.pinned_empty(len(caps) * 32768) if path == "in_place" else None
        bufs = []
        for k, p in enumerate(caps):
            # malloc'd, pageable (loop.c:180-183) — or a slot of the page-locked pool
            b = np.empty(32768, np.uint8) if pool is None else pool[k * 32768:(k + 1) * 32768]
            b[:] = 0xA5
            b[:p.size] = zeroed(p)
            bufs.append(b)
        ptrs = [b.ctypes.data for b in bufs]
        lens = [p.size for p in caps]                  # iov_len = tot_len (loop.c:47,54)
        with tcp_amd.HostContext(0, blocking_wait=(path == "in_place")) as ctx:
            out, st = ctx.ipv4_batch_ptrs(ptrs, lens, mode_fill)
            assert np.all(st == tcp_amd.PKT_OK)
            for b, p in zip(bufs, caps):
                assert np.array_equal(b[:p.size], p)
                assert np.all(b[p.size:] == 0xA5)
            v, vs = ctx.ipv4_batch_ptrs(ptrs, lens, mode_verify)
            assert np.all(v == 0) and np.all(vs == tcp_amd.PKT_OK)
            s = ctx.stats()
            assert s["pkts_in_place"] == (2 * len(caps) if path == "in_place" else 0)
        return
    pool = np.full(len(caps) * 32768, 0xA5, np.uint8)
    off = np.arange(len(caps), dtype=np.uint64) * 32768
    for o, p in zip(off, caps):
        pool[int(o):int(o) + p.size] = zeroed(p)
    if path == "region":
        with tcp_amd.HostContext(0) as ctx:
            out, st = ctx.ipv4_batch(pool, off, 32768, mode_fill)
            v, vs = ctx.ipv4_batch(pool, off, 32768, mode_verify)
        got = pool
    else:
        dev = torch.device("cuda:0")
        d = torch.from_numpy(pool).to(dev)
        doff = torch.from_numpy(off.view(np.int64)).to(dev)
        o_ = torch.empty(len(caps), dtype=torch.int16, device=dev)
        s_ = torch.empty(len(caps), dtype=torch.uint8, device=dev)
        tcp_amd.ipv4_batch(d, doff, len(caps), 32768, mode_fill, o_, s_)
        st = s_.cpu().numpy()
        got = d.cpu().numpy()
        tcp_amd.ipv4_batch(d, doff, len(caps), 32768, mode_verify, o_, s_)
        v, vs = o_.cpu().numpy().view(np.uint16), s_.cpu().numpy()
    assert np.all(st == tcp_amd.PKT_OK)
    for o, p in zip(off, caps):
        assert np.array_equal(got[int(o):int(o) + p.size], p)
    assert np.all(v == 0) and np.all(vs == tcp_amd.PKT_OK)
