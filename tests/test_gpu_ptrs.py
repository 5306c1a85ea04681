"""GPU parity for scatter-gather wire batches (one buffer per packet).

The reference keeps every outgoing packet in its own malloc'd 32 KiB buffer
(/root/reference/loop.c:180-183) and hands sendmmsg one iov_base per message
(loop.c:53-54). tcpcsum_ipv4_batch_ptrs_dev / _host checksum such batches with
a per-packet byte bound (iov_len / msg_len): in place where the memory is
page-locked, through the context's pinned staging where it is pageable. Every result is
compared with the oracle's FILL / VERIFY of the same packet bytes
(context.c:104-145 framing of context.c:169-209), bit for bit.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from tests.tensors import host, to_dev, u16  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    import tcp_amd
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, arch = tcp_amd.device_check()
    assert rc == 0, f"tcpcsum_device_check -> {rc} ({arch}); the HIP path must run on gfx950"
    return torch.device("cuda:0")


def tot_len(buf: np.ndarray, o: int) -> int:
    return (int(buf[o + 2]) << 8) | int(buf[o + 3])


def expected(region: np.ndarray, off: np.ndarray, lens: np.ndarray, mode: int):
    """Oracle per packet, with the per-packet bound: tot_len > lens[i] or lens[i] < 20 -> SKIPPED,
    untouched, out 0. Mutates region (FILL) like the device."""
    import tcp_amd
    ok = np.array([l >= 20 and tot_len(region, int(o)) <= l for o, l in zip(off, lens)], bool)
    want_out = np.zeros(off.size, np.uint16)
    want_st = np.full(off.size, tcp_amd.PKT_SKIPPED, np.uint8)
    if ok.any():
        o2, s2 = oracle.ipv4_batch(region, off[ok], 65535, mode)
        want_out[ok] = o2
        want_st[ok] = s2
    return want_out, want_st


@pytest.mark.parametrize("shape", [-1, 0, 1, 3, 5, 8, 9])
def test_ipv4_ptrs_dev_vs_oracle(dev, shape):
    """Packets scattered through one device allocation, addressed by pointer in shuffled order,
    each bounded by its own length: exact, checks patched in place, nothing else touched."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(77)
    n = 1500
    region, off, _ = build_batch(rng, n, slot=2048, malformed=True)
    perm = rng.permutation(n)
    off = off[perm]
    lens = np.array([tot_len(region, int(o)) for o in off], np.int64)
    lens[::7] += rng.integers(1, 500, lens[::7].size)      # more room than the packet needs
    lens[3::13] -= 1                                        # tot_len one past the bound: SKIPPED
    lens[5::17] = rng.integers(0, 20, lens[5::17].size)     # no room for an IP header: SKIPPED
    lens = np.clip(lens, 0, 2048).astype(np.uint32)
    ref = region.copy()
    want_out, want_st = expected(ref, off, lens, tcp_amd.IPV4_FILL)
    dreg = to_dev(region, dev)
    ptrs = to_dev((off + np.uint64(dreg.data_ptr())).view(np.int64), dev)
    dl = to_dev(lens.view(np.int32), dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    tcp_amd.ipv4_batch_ptrs(ptrs, dl, n, 65535, tcp_amd.IPV4_FILL, out, st,
                            tune=tcp_amd.make_tuning(0, 0, shape, 0))
    assert np.array_equal(host(st), want_st)
    assert np.array_equal(u16(out), want_out)
    assert np.array_equal(host(dreg), ref)
    # verify round trip: every filled packet verifies to 0
    tcp_amd.ipv4_batch_ptrs(ptrs, dl, n, 65535, tcp_amd.IPV4_VERIFY, out, st,
                            tune=tcp_amd.make_tuning(0, 0, shape, 0))
    want_v, want_vs = expected(ref.copy(), off, lens, tcp_amd.IPV4_VERIFY)
    assert np.array_equal(u16(out), want_v)
    assert np.array_equal(host(st), want_vs)
    assert np.all(want_v[want_vs == tcp_amd.PKT_OK] == 0)


def test_ipv4_ptrs_dev_iphdr_and_tail(dev):
    """IPv4 header checksum through pointers; packets ending exactly at their bound, at the end of
    the allocation."""
    import tcp_amd
    from tests.packets import ip_packet
    rng = np.random.default_rng(3)
    pkts = [ip_packet(rng, int(rng.integers(0, 1456)), ihl=5 + (i % 3)) for i in range(300)]
    offs, pos = [], 0
    for p in pkts:
        pos += int(rng.integers(0, 9))
        offs.append(pos)
        pos += len(p)
    region = np.zeros(pos, np.uint8)        # the last packet ends at the last byte
    for o, p in zip(offs, pkts):
        region[o:o + len(p)] = np.frombuffer(p, np.uint8)
    off = np.array(offs, np.uint64)
    lens = np.array([len(p) for p in pkts], np.uint32)
    mode = tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR
    ref = region.copy()
    want_out, want_st = expected(ref, off, lens, mode)
    dreg = to_dev(region, dev)
    ptrs = to_dev((off + np.uint64(dreg.data_ptr())).view(np.int64), dev)
    out = torch.empty(off.size, dtype=torch.int16, device=dev)
    st = torch.empty(off.size, dtype=torch.uint8, device=dev)
    tcp_amd.ipv4_batch_ptrs(ptrs, to_dev(lens.view(np.int32), dev), off.size, 65535, mode, out, st)
    assert np.array_equal(host(st), want_st)
    assert np.array_equal(u16(out), want_out)
    assert np.array_equal(host(dreg), ref)
    tcp_amd.ipv4_batch_ptrs(ptrs, to_dev(lens.view(np.int32), dev), off.size, 65535,
                            tcp_amd.IPV4_VERIFY | tcp_amd.IPV4_IPHDR, out, st)
    assert np.all(u16(out) == 0) and np.all(host(st) == tcp_amd.PKT_OK)


def _loop_pool(rng, n, slot=32768, payload=None):
    """The reference's out-buffer pool: n separately allocated pageable 32 KiB buffers, each holding
    one packet at its start (loop.c:180-183, context.c:169-209)."""
    from tests.packets import ip_packet
    bufs, lens = [], []
    for i in range(n):
        pl = int(rng.integers(0, 1457)) if payload is None else payload
        p = ip_packet(rng, pl)
        b = np.empty(slot, np.uint8)      # malloc'd by numpy, pageable
        b[:] = rng.integers(0, 256, slot, dtype=np.uint8)
        b[:len(p)] = np.frombuffer(p, np.uint8)
        bufs.append(b)
        lens.append(len(p))
    return bufs, np.array(lens, np.uint32)


@pytest.mark.parametrize("layout", ["malloc", "pinned"])
def test_ipv4_ptrs_host_loop_layout(dev, layout):
    """1024 separate 32 KiB out-buffers (loop.c:180-183): FILL, then VERIFY, then a shuffled sub-batch
    with short bounds. malloc: pageable buffers, every packet copied into the context's pinned staging
    and its check stored back. pinned: the pool carved from one tcpcsum_host_alloc block (INTEGRATION.md
    level 2), every packet read and filled in place. Nothing is ever page-locked by the library; bytes
    outside the check fields never change."""
    import tcp_amd
    rng = np.random.default_rng(11)
    bufs, lens = _loop_pool(rng, 1024)
    if layout == "pinned":
        pool = tcp_amd.pinned_empty(1024 * 32768)
        for k, b in enumerate(bufs):
            pool[k * 32768:(k + 1) * 32768] = b
        bufs = [pool[k * 32768:(k + 1) * 32768] for k in range(1024)]
    refs = [b.copy() for b in bufs]
    want = []
    for r, l in zip(refs, lens):
        o, s = expected(r, np.array([0], np.uint64), np.array([l], np.uint32), tcp_amd.IPV4_FILL)
        want.append((o[0], s[0]))
    ptrs = [b.ctypes.data for b in bufs]
    with tcp_amd.HostContext(0) as ctx:
        out, st = ctx.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_FILL)
        assert [(int(a), int(b)) for a, b in zip(out, st)] == [(int(a), int(b)) for a, b in want]
        for b, r in zip(bufs, refs):
            assert np.array_equal(b, r)
        stats = ctx.stats()
        if layout == "pinned":
            assert stats["pkts_in_place"] == 1024 and stats["pkts_staged"] == 0
        else:
            assert stats["pkts_in_place"] == 0 and stats["pkts_staged"] == 1024
        assert stats["ns_cpu_caller"] > 0
        # same buffers again (a second releaseSend): same results
        out2, _ = ctx.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_FILL)
        assert np.array_equal(out2, out)
        v, vs = ctx.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_VERIFY)
        assert np.all(v == 0) and np.all(vs == tcp_amd.PKT_OK)
        # a sub-batch in another order, with a bound one byte short on some packets
        idx = rng.permutation(1024)[:300]
        sl = lens[idx].copy()
        sl[::5] -= 1
        v, vs = ctx.ipv4_batch_ptrs([ptrs[i] for i in idx], sl, tcp_amd.IPV4_VERIFY)
        short = np.zeros(300, bool)
        short[::5] = True
        assert np.all(vs[short] == tcp_amd.PKT_SKIPPED) and np.all(v[short] == 0)
        assert np.all(vs[~short] == tcp_amd.PKT_OK) and np.all(v[~short] == 0)
        for b, r in zip(bufs, refs):
            assert np.array_equal(b, r)


def test_round3_fault_sequence_in_process(dev):
    """The sequence that faulted in round 3, in the test process itself: host batches
    over 256 separately malloc'd 32 KiB buffers, the buffers freed, then pageable torch copies whose
    fresh host destinations reuse those heap addresses — three times over, and after a pinned-pool
    batch beside them. The library never page-locks or unlocks those pages (it cannot: ABI v4 has no
    registration), so every copy must come back exact."""
    import ctypes
    import tcp_amd
    from tests.packets import ip_packet
    libc = ctypes.CDLL(None)
    libc.malloc.restype = ctypes.c_void_p
    libc.malloc.argtypes = [ctypes.c_size_t]
    libc.free.argtypes = [ctypes.c_void_p]
    rng = np.random.default_rng(5)
    pool = tcp_amd.pinned_empty(64 * 32768)
    src = torch.arange(8 << 20, dtype=torch.uint8, device=dev) * 7
    want = (np.arange(8 << 20, dtype=np.uint64) * 7).astype(np.uint8)
    with tcp_amd.HostContext(0) as ctx:
        for rep in range(3):
            addrs, lens = [], []
            for k in range(256):
                a = libc.malloc(32768)
                p = ip_packet(rng, int(rng.integers(0, 1457)))
                ctypes.memmove(a, p, len(p))
                addrs.append(a)
                lens.append(len(p))
            out, st = ctx.ipv4_batch_ptrs(addrs, lens, tcp_amd.IPV4_FILL)
            assert np.all(st == tcp_amd.PKT_OK)
            v, vs = ctx.ipv4_batch_ptrs(addrs, lens, tcp_amd.IPV4_VERIFY)
            assert np.all(v == 0)
            for k in range(64):   # a pinned pool in the same process, filled in place
                p = ip_packet(rng, 1456)
                pool[k * 32768:k * 32768 + len(p)] = np.frombuffer(p, np.uint8)
            ctx.ipv4_batch_ptrs([pool.ctypes.data + k * 32768 for k in range(64)], [1500] * 64, tcp_amd.IPV4_FILL)
            for a in addrs:
                libc.free(a)
            # pageable copies over the freed heap: .cpu() of 8 MiB and of small slices, and an H2D back
            for _ in range(4):
                got = src.cpu().numpy()
                assert np.array_equal(got, want)
                small = [src[k * 30000:(k + 1) * 30000].cpu().numpy() for k in range(8)]
                assert all(np.array_equal(x, want[k * 30000:(k + 1) * 30000]) for k, x in enumerate(small))
                back = torch.from_numpy(got).to(dev)
                assert torch.equal(back, src)
        torch.cuda.synchronize()
        assert ctx.stats()["pkts_in_place"] == 3 * 64


def test_ipv4_ptrs_host_pinned_and_mixed(dev):
    """Packets in page-locked memory (tcpcsum_host_alloc) are used through their existing mapping
    (no registration, no copy); pageable buffers in the same batch are staged; NULL and short
    messages are SKIPPED."""
    import tcp_amd
    rng = np.random.default_rng(12)
    pinned = tcp_amd.pinned_empty(64 * 2048)
    pinned[:] = 0
    from tests.packets import ip_packet
    ptrs, lens, refs = [], [], []
    pageable, _ = _loop_pool(rng, 64, slot=4096)
    for i in range(64):
        p = ip_packet(rng, int(rng.integers(0, 1400)))
        pinned[i * 2048:i * 2048 + len(p)] = np.frombuffer(p, np.uint8)
    ref_pinned = pinned.copy()
    for i in range(64):
        ptrs += [pinned.ctypes.data + i * 2048, pageable[i].ctypes.data]
        lens += [tot_len(pinned, i * 2048), tot_len(pageable[i], 0)]
    ptrs += [0, pageable[0].ctypes.data]
    lens += [1500, 10]
    ref_page = [b.copy() for b in pageable]
    with tcp_amd.HostContext(0) as ctx:
        out, st = ctx.ipv4_batch_ptrs(ptrs, np.array(lens, np.uint32), tcp_amd.IPV4_FILL)
        w1, s1 = expected(ref_pinned, np.arange(64, dtype=np.uint64) * 2048,
                          np.array(lens[0:128:2], np.uint32), tcp_amd.IPV4_FILL)
        assert np.array_equal(out[0:128:2], w1) and np.array_equal(st[0:128:2], s1)
        for i in range(64):
            w2, s2 = expected(ref_page[i], np.array([0], np.uint64), np.array([lens[2 * i + 1]], np.uint32),
                              tcp_amd.IPV4_FILL)
            assert out[2 * i + 1] == w2[0] and st[2 * i + 1] == s2[0]
            assert np.array_equal(pageable[i], ref_page[i])
        assert np.array_equal(pinned, ref_pinned)
        assert list(st[-2:]) == [tcp_amd.PKT_SKIPPED] * 2 and list(out[-2:]) == [0, 0]
        stats = ctx.stats()
        assert stats["pkts_in_place"] == 64 and stats["pkts_staged"] == 64


def test_ipv4_ptrs_host_context_tuning(dev):
    """Tuning set on one context shapes only that context's batches (results identical)."""
    import tcp_amd
    rng = np.random.default_rng(13)
    bufs, lens = _loop_pool(rng, 200, slot=4096)
    ptrs = [b.ctypes.data for b in bufs]
    with tcp_amd.HostContext(0) as a, tcp_amd.HostContext(0) as b:
        b.set_tuning(0, 0, 5, tcp_amd.TUNE_WIN16)
        va, sa = a.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_VERIFY)
        vb, sb = b.ipv4_batch_ptrs(ptrs, lens, tcp_amd.IPV4_VERIFY)
        assert np.array_equal(va, vb) and np.array_equal(sa, sb)
        with pytest.raises(tcp_amd.TcpCsumError):
            b.set_tuning(0, 3)


@pytest.mark.parametrize("memory", ["pageable", "pinned"])
def test_ipv4_region_host_pool(dev, memory):
    """The region host path over a 512-packet pool in 32 KiB slots: staged when the pool is pageable,
    read and filled in place when it is one tcpcsum_host_alloc block. Results identical; the uniform
    host path over the same bytes too."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(21)
    region, off, _ = build_batch(rng, 512, slot=32768, malformed=True)
    if memory == "pinned":
        pin = tcp_amd.pinned_empty(region.nbytes)
        pin[:] = region
        region = pin
    ref = region.copy()
    want_out, want_st = oracle.ipv4_batch(ref, off, 32768, tcp_amd.IPV4_FILL)
    with tcp_amd.HostContext(0) as ctx:
        out, st = ctx.ipv4_batch(region, off, 32768, tcp_amd.IPV4_FILL)
        assert np.array_equal(st, want_st) and np.array_equal(out, want_out)
        assert np.array_equal(region, ref)
        stats = ctx.stats()
        assert (stats["pkts_in_place"], stats["pkts_staged"]) == ((512, 0) if memory == "pinned" else (0, 512))
        v, vs = ctx.ipv4_batch(region, off, 32768, tcp_amd.IPV4_VERIFY)
        assert np.all(v[vs == tcp_amd.PKT_OK] == 0)
        # the uniform host path over the same bytes, odd shapes
        u = ctx.batch_uniform(region, 1501, 1499, (region.nbytes - 1499) // 1501, 777)
        assert np.array_equal(u, oracle.batch_uniform(region, 1501, 1499, u.size, 777))


def test_ipv4_region_host_staging_large_bounds(dev):
    """A pageable region whose packets' readable bounds add up past the one-pass staging limit
    (64 MiB: 1400 packets in 32 KiB slots with cap 65535, so each bound is up to 64 KiB): the copy
    threads read every packet's tot_len first and pack the copies by it (two passes). Results,
    statuses and the caller's bytes match the oracle."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(31)
    n = 1400
    region, off, _ = build_batch(rng, n, slot=32768, malformed=True)
    ref = region.copy()
    for mode in (tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR, tcp_amd.IPV4_VERIFY | tcp_amd.IPV4_IPHDR):
        want_out, want_st = oracle.ipv4_batch(ref, off, 65535, mode)
        with tcp_amd.HostContext(0) as ctx:
            out, st = ctx.ipv4_batch(region, off, 65535, mode)
            stats = ctx.stats()
        assert np.array_equal(st, want_st) and np.array_equal(out, want_out)
        assert np.array_equal(region, ref)
        assert stats["pkts_staged"] == n and stats["pkts_in_place"] == 0
        # only the packets' bytes were copied, not their 64 KiB bounds
        assert stats["bytes_staged"] <= n * 1600
    ok = want_st == tcp_amd.PKT_OK
    assert ok.sum() > n // 2 and np.all(want_out[ok] == 0)
