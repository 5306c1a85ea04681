"""GPU parity: the gfx950 kernels vs the oracle, bit for bit (integer path: exact).

Small/medium cases compare every output with the oracle on the same seeded
bytes; the BASELINE configs at full size compare against the reference's own
Appendix B digests (tests/golden/reference_vectors.json); properties
(verify-to-zero, fill/verify round trip) cover the wire path. Every call goes
through the C ABI (libtcpcsum.so) — there is no CPU fallback to pass through.
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


def test_native_library_is_loaded(dev):
    """The mapped libtcpcsum.so is a product build of exactly the sources in this tree (no stale or
    measurement-built library: tcpcsum_build_info vs the tree's hash)."""
    import tcp_amd
    from tcp_amd import provenance
    tcp_amd.lib()
    with open("/proc/self/maps") as f:
        maps = f.read()
    assert "libtcpcsum.so" in maps
    info = provenance.check_product_build()
    print("build:", info)


LENGTHS = [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 24, 31, 32, 33, 44, 63, 64, 65, 100, 255, 256, 257, 511, 512,
           513, 1023, 1024, 1025, 1479, 1480, 1499, 1500, 1501, 1503, 1504, 2048, 4095, 4096, 4097, 8191, 8192,
           8193, 9000, 16383, 32767, 65535, 65536, 65537]


@pytest.mark.parametrize("length", LENGTHS)
def test_uniform_vs_oracle_lengths(dev, length):
    import tcp_amd
    rng = np.random.default_rng(length + 11)
    for base_off in (0, 1, 4, 12):
        for stride in sorted({max(length, 1), length + 3 if length else 7, length + 16}):
            n = int(min(300, max(8, (1 << 21) // max(stride, 1))))
            size = base_off + (n - 1) * stride + length + 64
            host = rng.integers(0, 256, size, dtype=np.uint8)
            ss = rng.integers(0, 6 * 0xFFFF + 1, n, dtype=np.uint32)
            d = to_dev(host, dev)
            got = u16(tcp_amd.batch_uniform(d, stride, length, n, to_dev(ss.view(np.int32), dev), offset=base_off))
            want = oracle.batch_uniform(host, stride, length, n, ss, offset=base_off)
            assert np.array_equal(got, want), (length, base_off, stride)
            # scalar start value
            got = u16(tcp_amd.batch_uniform(d, stride, length, n, 393210, offset=base_off))
            want = oracle.batch_uniform(host, stride, length, n, 393210, offset=base_off)
            assert np.array_equal(got, want), (length, base_off, stride, "scalar")


def test_uniform_overlapping_and_zero_stride(dev):
    import tcp_amd
    rng = np.random.default_rng(5)
    host = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    d = to_dev(host, dev)
    for stride, length, n in [(0, 1500, 50), (7, 1500, 500), (1, 64, 1000), (100, 1500, 400)]:
        got = u16(tcp_amd.batch_uniform(d, stride, length, n, 17))
        assert np.array_equal(got, oracle.batch_uniform(host, stride, length, n, 17)), (stride, length)


def test_uniform_all_unrolls_and_grids(dev):
    import tcp_amd
    rng = np.random.default_rng(9)
    host = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    d = to_dev(host, dev)
    try:
        for unroll in (1, 2, 4, 8):
            for max_blocks, flags in ((1, 1), (7, 0), (0, 1), (0, 2 | 8)):
                tcp_amd.set_tuning(max_blocks, unroll, -1, flags)
                for length in (64, 60, 1500, 1501, 2000, 8192, 20000):
                    n = (3 << 20) // (length + 1) - 1
                    got = u16(tcp_amd.batch_uniform(d, length, length, n, 99))
                    want = oracle.batch_uniform(host, length, length, n, 99)
                    assert np.array_equal(got, want), (unroll, max_blocks, flags, length)
    finally:
        tcp_amd.set_tuning(0, 0, -1, 0)


def test_forced_shapes(dev):
    import tcp_amd
    rng = np.random.default_rng(19)
    host = rng.integers(0, 256, 1 << 21, dtype=np.uint8)
    d = to_dev(host, dev)
    try:
        for shape in range(15):
            for unroll, flags in ((1, 0), (8, 0), (2, 1 | 8), (8, 1 | 4), (4, 2 | 8), (8, 16), (1, 16 | 8)):
                tcp_amd.set_tuning(0, unroll, shape, flags)
                for length, off in ((1500, 0), (1499, 1), (64, 4), (3000, 2), (64, 0), (60, 3), (100, 0),
                                    (1500, 4), (2048, 0), (1024, 12), (9000, 8)):
                    n = (1 << 21) // (length + 8) - 1
                    got = u16(tcp_amd.batch_uniform(d, length + 1, length, n, 3, offset=off))
                    want = oracle.batch_uniform(host, length + 1, length, n, 3, offset=off)
                    assert np.array_equal(got, want), (shape, unroll, flags, length, off)
    finally:
        tcp_amd.set_tuning(0, 0, -1, 0)


@pytest.mark.parametrize("shape", [13, 14])
def test_split_segments_round_edges(dev, shape):
    """Shape 13 (four waves per segment) and 14 (a workgroup of 4..16 waves per segment, segments
    XCD by XCD): lengths at the edges of their rounds (256*C chunks per round, C = 4..32; 1024*4,
    512*8, 1024*2, 256*16), every start alignment mod 16, a capped grid (grid-stride over
    segments, block order)."""
    import tcp_amd
    rng = np.random.default_rng(23)
    host = rng.integers(0, 256, 6 << 20, dtype=np.uint8)
    d = to_dev(host, dev)
    ss = rng.integers(0, 2**32, 4096, dtype=np.uint32)
    dss = to_dev(ss.view(np.int32), dev)
    try:
        for unroll in (1, 2, 4, 8):
            for max_blocks in (0, 3, 16):
                tcp_amd.set_tuning(max_blocks, unroll, shape, 0)
                for length in (8204, 16384, 16380, 16400, 32768, 32772, 65536, 131072 + 4, 262144):
                    for off in (0, 4, 12):
                        n = min(4096, ((6 << 20) - 16) // (length + 16))
                        stride = length + 16
                        got = u16(tcp_amd.batch_uniform(d, stride, length, n, dss[:n], offset=off))
                        want = oracle.batch_uniform(host, stride, length, n, ss[:n], offset=off)
                        assert np.array_equal(got, want), (unroll, max_blocks, length, off)
    finally:
        tcp_amd.set_tuning(0, 0, -1, 0)
    # the default plan takes the split for aligned segments up to 32 KiB, a workgroup per segment
    # past that up to 128 KiB, and matches too
    for length, shape in ((16384, 13), (32768, 13), (32772, 14), (65536, 14), (131072, 14)):
        n = ((6 << 20) - 64) // length
        assert tcp_amd.api.plan_uniform(0, length, length, n)[1] == shape, length
        got = u16(tcp_amd.batch_uniform(d, length, length, n, 7))
        assert np.array_equal(got, oracle.batch_uniform(host, length, length, n, 7)), length


def test_two_fold_semantics_above_4g(dev):
    """S = 0x1_0000_FFFF: the reference's exactly-two folds, not a full fold."""
    import tcp_amd
    seg = np.frombuffer(b"\xff\xff" * 65538 + b"\x01\x00", np.uint8)
    host = np.concatenate([seg, seg, np.zeros(64, np.uint8)])
    d = to_dev(host, dev)
    got = u16(tcp_amd.batch_uniform(d, seg.size, seg.size, 2, 0))
    want = oracle.batch_uniform(host, seg.size, seg.size, 2, 0)
    assert np.array_equal(got, want)
    assert want[0] == oracle.csum_continue(0, seg.tobytes())
    # all-zero segment with start 0 -> 0xFFFF (never conflated with 0x0000)
    z = torch.zeros(4096, dtype=torch.uint8, device=dev)
    assert np.all(u16(tcp_amd.batch_uniform(z, 64, 64, 64, 0)) == 0xFFFF)


def test_long_segments_and_big_sums(dev):
    import tcp_amd
    rng = np.random.default_rng(21)
    for length in (131072, 200003, 1 << 20):
        n = 6
        host = rng.integers(200, 256, n * length + 64, dtype=np.uint8)   # large bytes -> S well above 2^32
        d = to_dev(host, dev)
        for off in (0, 1, 2):
            got = u16(tcp_amd.batch_uniform(d, length, length - off, n, 0xFFFFFFFF, offset=off))
            want = oracle.batch_uniform(host, length, length - off, n, 0xFFFFFFFF, offset=off)
            assert np.array_equal(got, want), (length, off)
        # a workgroup per segment (shape 14), every variant: u32 lane partials per round, u64 above
        for unroll in (1, 2, 4, 8):
            got = u16(tcp_amd.batch_uniform(d, length, length, n, 0xFFFFFFFF,
                                            tune=tcp_amd.make_tuning(0, unroll, 14, 0)))
            assert np.array_equal(got, oracle.batch_uniform(host, length, length, n, 0xFFFFFFFF)), (length, unroll)


def _desc(off, lens, ss):
    from tcp_amd import DESC_DTYPE
    d = np.zeros(len(off), DESC_DTYPE)
    d["offset"], d["len"], d["sum_start"] = off, lens, ss
    return d.view(np.uint8)


@pytest.mark.parametrize("max_len", [64, 1500, 9000, 70000])
def test_desc_ragged_vs_oracle(dev, max_len):
    import tcp_amd
    rng = np.random.default_rng(max_len)
    size = 4 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    n = 3000
    lens = rng.integers(0, max_len + 1, n).astype(np.uint32)
    lens[:10] = [0, 1, 2, 3, max_len, max_len - 1, 0, 5, 1, max_len]
    off = np.array([rng.integers(0, size - l) for l in lens], np.uint64)
    ss = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d = to_dev(host, dev)
    dd = to_dev(_desc(off, lens, ss), dev)
    got = u16(tcp_amd.batch_desc(d, dd, n, max_len))
    assert np.array_equal(got, oracle.batch_desc(host, off, lens, ss))
    # a max_len hint that is too small is slower, never wrong
    got = u16(tcp_amd.batch_desc(d, dd, n, 16))
    assert np.array_equal(got, oracle.batch_desc(host, off, lens, ss))


@pytest.mark.parametrize("odd", [False, True])
def test_ipv4_fill_and_verify(dev, odd):
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(31 + odd)
    region, off, _ = build_batch(rng, 1024, malformed=True, odd_offsets=odd)
    ref_region = region.copy()
    want_out, want_st = oracle.ipv4_batch(ref_region, off, 32768, tcp_amd.IPV4_FILL)
    dreg = to_dev(region, dev)
    doff = to_dev(off.view(np.int64), dev)
    out = torch.empty(off.size, dtype=torch.int16, device=dev)
    st = torch.empty(off.size, dtype=torch.uint8, device=dev)
    tcp_amd.ipv4_batch(dreg, doff, off.size, 32768, tcp_amd.IPV4_FILL, out, st)
    assert np.array_equal(host(st), want_st)
    assert np.array_equal(u16(out), want_out)
    assert np.array_equal(host(dreg), ref_region)     # checks patched in place, nothing else touched
    # rx side: every filled segment verifies to zero (loop.c:314-399 has no verify; new behaviour)
    tcp_amd.ipv4_batch(dreg, doff, off.size, 32768, tcp_amd.IPV4_VERIFY, out, st)
    v = u16(out)
    ok = host(st) == tcp_amd.PKT_OK
    assert np.all(v[ok] == 0)
    want_v, _ = oracle.ipv4_batch(ref_region.copy(), off, 32768, tcp_amd.IPV4_VERIFY)
    assert np.array_equal(v, want_v)
    # corrupt one payload byte per packet -> verification fails exactly there
    bad = ref_region.copy()
    idx = [int(o) + 44 for o, s in zip(off, want_st) if s == 0 and int(o) + 60 < bad.size]
    bad[idx] ^= 0x5A
    dbad = to_dev(bad, dev)
    tcp_amd.ipv4_batch(dbad, doff, off.size, 32768, tcp_amd.IPV4_VERIFY, out, st)
    want_b, _ = oracle.ipv4_batch(bad.copy(), off, 32768, tcp_amd.IPV4_VERIFY)
    assert np.array_equal(u16(out), want_b)


@pytest.mark.parametrize("name", ["1Mx1500", "1Mx64", "256Kx64KiB"])
def test_baseline_configs_match_reference_digests(dev, golden, name):
    """Full-size BASELINE configs, generated on device, vs the reference's own Appendix B digests."""
    import tcp_amd
    g = golden["digests"][name]
    n, L = g["n"], g["seg_len"]
    data = torch.empty(n * L, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(data, g["seg0"] * L, n * L)
    ss = torch.empty(n, dtype=torch.int32, device=dev)
    tcp_amd.synth_pseudo(ss, g["seg0"], n, L)
    out = u16(tcp_amd.batch_uniform(data, L, L, n, ss))
    assert oracle.digest(out) == (g["fnv1a64"], g["sum"], g["xor"])
    assert [f"{v:04x}" for v in out[:4]] == g["first4"] and f"{out[-1]:04x}" == g["last"]
    # the device generator equals the oracle's generator
    assert np.array_equal(host(data[:4096]), oracle.gen_stream(g["seg0"] * L, 4096))
    del data


def test_8gpu_config_shard_by_shard(dev, golden):
    """8M x 1500 as eight contiguous 1M shards, as bench.py --gpus 8 partitions it."""
    import tcp_amd
    from bench import shard_range
    L = 1500
    parts = []
    data = torch.empty((1 << 20) * L, dtype=torch.uint8, device=dev)
    ss = torch.empty(1 << 20, dtype=torch.int32, device=dev)
    for k in range(8):
        s0, cnt = shard_range(8 << 20, 8, k)
        g = golden["digests"][f"8Mx1500_shard{k}"]
        assert (s0, cnt) == (g["seg0"], g["n"])
        tcp_amd.synth_fill(data, s0 * L, cnt * L)
        tcp_amd.synth_pseudo(ss, s0, cnt, L)
        out = u16(tcp_amd.batch_uniform(data, L, L, cnt, ss))
        assert oracle.digest(out) == (g["fnv1a64"], g["sum"], g["xor"]), k
        parts.append(out)
    g = golden["digests"]["8Mx1500"]
    assert oracle.digest(np.concatenate(parts)) == (g["fnv1a64"], g["sum"], g["xor"])


def test_synth_fill_unaligned(dev):
    import tcp_amd
    buf = torch.zeros(5000, dtype=torch.uint8, device=dev)
    for off, nb, dst in [(3, 100, 1), (8, 64, 0), (13, 4000, 7)]:
        buf.zero_()
        tcp_amd.synth_fill(buf, off, nb, dst_offset=dst)
        h = host(buf)
        assert np.array_equal(h[dst:dst + nb], oracle.gen_stream(off, nb))
        assert not h[:dst].any() and not h[dst + nb:].any()


def test_stream_probe_sums(dev):
    import tcp_amd
    rng = np.random.default_rng(4)
    host = rng.integers(0, 2**32, (1 << 20) // 4, dtype=np.uint64).astype(np.uint32)
    d = to_dev(host.view(np.uint8), dev)
    parts = torch.zeros(tcp_amd.api.PROBE_SLOTS, dtype=torch.int64, device=dev)
    want = int((host & 0xFFFF).astype(np.uint64).sum() + (host >> 16).astype(np.uint64).sum())
    # default (one 4 KiB tile per wave: 64 workgroups here), small and wide grids; the launch adds
    # into the slots, so they are zeroed first
    for blocks, unroll in ((0, 0), (7, 1), (3000, 4)):
        tcp_amd.set_tuning(blocks, unroll, -1, 0)
        parts.zero_()
        try:
            k = tcp_amd.stream_probe(d, host.nbytes, parts)
        finally:
            tcp_amd.set_tuning(0, 0, -1, 0)
        assert int(parts[:k].sum().item()) == want
    # 192 MiB: 49152 waves by default, more than the slots (partials fold into slot
    # wave % PROBE_SLOTS); the expected sum from torch on the device
    g = torch.Generator(device=dev).manual_seed(9)
    w = torch.randint(0, 2**32, (48 << 20,), dtype=torch.int64, device=dev, generator=g)
    want = int(((w & 0xFFFF) + (w >> 16)).sum().item())
    d = w.to(torch.int32)   # the same u32 words, two's complement
    del w
    parts.zero_()
    k = tcp_amd.stream_probe(d, d.numel() * 4, parts)
    assert k == tcp_amd.api.PROBE_SLOTS
    assert int(parts.sum().item()) == want


def test_nondefault_stream(dev):
    import tcp_amd
    rng = np.random.default_rng(8)
    host = rng.integers(0, 256, 1500 * 1000, dtype=np.uint8)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        d = to_dev(host, dev)
        out = tcp_amd.batch_uniform(d, 1500, 1500, 1000, 5)
    s.synchronize()
    assert np.array_equal(u16(out), oracle.batch_uniform(host, 1500, 1500, 1000, 5))


def test_host_context_uniform_and_wire(dev):
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(12)
    host = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    ss = rng.integers(0, 393211, 2000, dtype=np.uint32)
    with tcp_amd.HostContext(0, scratch_bytes=256 << 10) as ctx:   # small scratch -> many pipelined chunks
        for stride, length, n in [(1500, 1500, 2000), (1501, 1480, 2000), (64, 64, 2000), (70000, 65536, 40)]:
            s = ss if n <= ss.size else 7
            got = ctx.batch_uniform(host, stride, length, n, s[:n] if isinstance(s, np.ndarray) else s)
            assert np.array_equal(got, oracle.batch_uniform(host, stride, length, n,
                                                            s[:n] if isinstance(s, np.ndarray) else s))
        region, off, _ = build_batch(rng, 512, malformed=True, odd_offsets=True)
        ref = region.copy()
        want_out, want_st = oracle.ipv4_batch(ref, off, 32768, tcp_amd.IPV4_FILL)
        out, st = ctx.ipv4_batch(region, off, 32768, tcp_amd.IPV4_FILL)
        assert np.array_equal(st, want_st) and np.array_equal(out, want_out)
        assert np.array_equal(region, ref)
        out, st = ctx.ipv4_batch(region, off, 32768, tcp_amd.IPV4_VERIFY)
        assert np.all(out[st == 0] == 0)


def test_host_context_zero_copy_pinned(dev):
    """Pinned host memory: the kernels read (and FILL writes) it directly over PCIe."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(13)
    n, L = 5000, 1500
    host = tcp_amd.pinned_empty(n * L + 64)
    host[:] = rng.integers(0, 256, host.size, dtype=np.uint8)
    ss = tcp_amd.pinned_empty(n * 4, np.uint32)
    ss[:] = rng.integers(0, 393211, n, dtype=np.uint32)
    with tcp_amd.HostContext(0) as ctx:
        for off in (0, 3, 4):
            got = ctx.batch_uniform(host, L, L - off, n - 1, ss, offset=off)
            assert np.array_equal(got, oracle.batch_uniform(host, L, L - off, n - 1, ss[:n - 1], offset=off))
        region, off, _ = build_batch(rng, 700, malformed=True, odd_offsets=True)
        pin = tcp_amd.pinned_empty(region.size)
        pin[:] = region
        ref = region.copy()
        want_out, want_st = oracle.ipv4_batch(ref, off, 32768, tcp_amd.IPV4_FILL)
        out, st = ctx.ipv4_batch(pin, off, 32768, tcp_amd.IPV4_FILL)
        assert np.array_equal(st, want_st) and np.array_equal(out, want_out)
        assert np.array_equal(pin, ref)          # checks stored in place in host memory by the kernel
        out, st = ctx.ipv4_batch(pin, off, 32768, tcp_amd.IPV4_VERIFY)
        assert np.all(out[st == 0] == 0)


@pytest.mark.parametrize("memory", ["device", "pageable", "pinned"])
def test_ipv4_iphdr_mode(dev, memory):
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(77)
    region, off, _ = build_batch(rng, 300, malformed=True, odd_offsets=True)
    ref = region.copy()
    mode = tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR
    want_out, want_st = oracle.ipv4_batch(ref, off, 32768, mode)
    if memory == "device":
        dreg = to_dev(region, dev)
        doff = to_dev(off.view(np.int64), dev)
        out = torch.empty(off.size, dtype=torch.int16, device=dev)
        st = torch.empty(off.size, dtype=torch.uint8, device=dev)
        tcp_amd.ipv4_batch(dreg, doff, off.size, 32768, mode, out, st)
        got_out, got_st, got_reg = u16(out), host(st), host(dreg)
    else:
        buf = region if memory == "pageable" else tcp_amd.pinned_empty(region.size)
        buf[:] = region
        with tcp_amd.HostContext(0) as ctx:
            got_out, got_st = ctx.ipv4_batch(buf, off, 32768, mode)
        got_reg = np.array(buf)
    assert np.array_equal(got_st, want_st) and np.array_equal(got_out, want_out)
    assert np.array_equal(got_reg, ref)
    # verify with IP header check: OK everywhere it was filled; a corrupted TTL is flagged
    bad = ref.copy()
    okidx = np.flatnonzero(want_st == 0)
    bad[int(off[okidx[0]]) + 8] ^= 0x40
    want_v, want_vs = oracle.ipv4_batch(bad.copy(), off, 32768, tcp_amd.IPV4_VERIFY | tcp_amd.IPV4_IPHDR)
    dbad = to_dev(bad, dev)
    out = torch.empty(off.size, dtype=torch.int16, device=dev)
    st = torch.empty(off.size, dtype=torch.uint8, device=dev)
    tcp_amd.ipv4_batch(dbad, to_dev(off.view(np.int64), dev), off.size, 32768,
                       tcp_amd.IPV4_VERIFY | tcp_amd.IPV4_IPHDR, out, st)
    assert np.array_equal(host(st), want_vs) and np.array_equal(u16(out), want_v)
    assert want_vs[okidx[0]] == tcp_amd.PKT_IPHDR_BAD


def test_c_client_on_gpu(dev):
    """The plain-C ABI client (tests/c/abi_smoke.c) runs a host batch on the GPU."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "c", "abi_smoke")
    r = subprocess.run([exe, "--gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host-batch mismatches: 0 /" in r.stdout
    assert "pointer-batch (staged) mismatches: 0 /" in r.stdout
    assert "pointer-batch (in place) mismatches: 0 /" in r.stdout


@pytest.mark.parametrize("layout", ["packed", "packed_odd", "slots", "jumbo", "small"])
def test_tx_build_vs_oracle(dev, layout):
    """Device-side segment assembly + checksum == the oracle's context.c:150-213, byte for byte.
    "small": payloads up to 536 B (the 16-lane default shape)."""
    import tcp_amd
    from tests.test_oracle import make_txsegs
    rng = np.random.default_rng({"packed": 1, "packed_odd": 2, "slots": 3, "jumbo": 4, "small": 5}[layout])
    payload = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    max_len = {"jumbo": 9000, "small": 536}.get(layout, 1456)
    n = 400 if layout == "jumbo" else 3000
    segs, size = make_txsegs(rng, n, payload.size, max_len=max_len, odd=layout == "packed_odd",
                             slot=32768 if layout == "slots" else None)
    garbage = rng.integers(0, 256, size, dtype=np.uint8)     # bytes between packets must survive
    for mode in (0, tcp_amd.IPV4_IPHDR):
        want = garbage.copy()
        want_c = oracle.tx_build(payload, segs, want, iphdr=bool(mode))
        dout = to_dev(garbage, dev)
        dseg = to_dev(segs.view(np.uint8), dev)
        chk = torch.empty(n, dtype=torch.int16, device=dev)
        tcp_amd.tx_build(to_dev(payload, dev), dseg, n, max_len, dout, mode, chk)
        got = host(dout)
        assert np.array_equal(u16(chk), want_c), layout
        if not np.array_equal(got, want):
            bad = np.flatnonzero(got != want)
            raise AssertionError(f"{layout} mode={mode}: {bad.size} bytes differ, first at {bad[:8]}")
    # a too-small shape hint, or any forced shape / unroll, is slower, never wrong
    want = garbage.copy()
    oracle.tx_build(payload, segs, want)
    dpay, dseg = to_dev(payload, dev), to_dev(segs.view(np.uint8), dev)
    try:
        for shape, unroll, hint, fl in ((-1, 0, 16, 0), (0, 2, max_len, 0), (1, 4, max_len, 0), (3, 1, max_len, 0),
                                        (4, 2, 64, 0), (-1, 0, max_len, 128), (2, 2, max_len, 128), (-1, 0, max_len, 1024),
                                        (1, 2, max_len, 1024), (5, 1, max_len, 0), (6, 1, max_len, 0), (6, 2, 64, 0)):
            tcp_amd.set_tuning(0, unroll, shape, fl)   # 128 / 1024: non-temporal / written-through stores
            dout = to_dev(garbage, dev)
            tcp_amd.tx_build(dpay, dseg, n, hint, dout, 0, None)
            assert np.array_equal(host(dout), want), (shape, unroll, hint, fl)
    finally:
        tcp_amd.set_tuning(0, 0, -1, 0)


def test_tx_build_length_limits(dev):
    """The largest packet the IPv4 tot_len can describe (65491-B payload -> 65535 B) is built and
    checked; longer payloads (65492..65535) are not written and report check 0, like the oracle's
    restatement of context.c:150-213; without the DATA flag the length is ignored."""
    import tcp_amd
    from tests.test_oracle import make_txsegs
    rng = np.random.default_rng(77)
    payload = rng.integers(0, 256, 1 << 17, dtype=np.uint8)
    segs, _ = make_txsegs(rng, 8, payload.size, max_len=100)
    lens = [65491, 65492, 65535, 65490, 0, 1, 65491, 3]
    pos = 0
    for i, L in enumerate(lens):
        segs[i]["len"] = L
        segs[i]["payload_off"] = int(rng.integers(0, payload.size - L))
        segs[i]["out_off"] = pos
        segs[i]["flags"] = 16 | 1 if i != 6 else 1          # the last 65491: no DATA flag
        pos += 44 + (L if L <= 65491 else 0) + 16
    garbage = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    for mode in (0, tcp_amd.IPV4_IPHDR):
        want = garbage.copy()
        want_c = oracle.tx_build(payload, segs, want, iphdr=bool(mode))
        dout = to_dev(garbage, dev)
        chk = torch.empty(len(lens), dtype=torch.int16, device=dev)
        tcp_amd.tx_build(to_dev(payload, dev), to_dev(segs.view(np.uint8), dev), len(lens), 65535, dout, mode, chk)
        assert np.array_equal(u16(chk), want_c)
        assert np.array_equal(host(dout), want)
        assert want_c[1] == 0 and want_c[2] == 0


def test_ipv4_verify_flags_checksum_partial(dev):
    """New behaviour (no reference result — parity pinned to the oracle only): VERIFY marks
    CHECKSUM_PARTIAL segments (check = un-complemented pseudo sum) instead of plain failures."""
    import tcp_amd
    from tests.test_oracle import partial_offload_batch
    region, off = partial_offload_batch(seed=10, n=500)
    want_out, want_st = oracle.ipv4_batch(region.copy(), off, 32768, tcp_amd.IPV4_VERIFY)
    out = torch.empty(off.size, dtype=torch.int16, device=dev)
    st = torch.empty(off.size, dtype=torch.uint8, device=dev)
    tcp_amd.ipv4_batch(to_dev(region, dev), to_dev(off.view(np.int64), dev), off.size, 32768,
                       tcp_amd.IPV4_VERIFY, out, st)
    assert np.array_equal(u16(out), want_out) and np.array_equal(host(st), want_st)
    assert (want_st == tcp_amd.api.PKT_CSUM_PARTIAL).sum() > 300


@pytest.mark.parametrize("unroll", [1, 2, 4, 8])
def test_flat_tiles_vs_oracle(dev, unroll):
    """Shape 12 (flat tiles): packed and gapped layouts, aligned and 4-byte-misaligned bases."""
    import tcp_amd
    rng = np.random.default_rng(40 + unroll)
    host = rng.integers(0, 256, 6 << 20, dtype=np.uint8)
    d = to_dev(host, dev)
    try:
        tcp_amd.set_tuning(0, unroll, 12, 0)
        for stride, length, off in ((1500, 1500, 0), (1500, 1500, 4), (1504, 1500, 12), (2048, 1024, 8),
                                    (4096, 4096, 0), (9000, 8996, 4), (32000, 30000, 0), (1024, 1024, 4)):
            n = (host.size - off - length) // stride
            assert tcp_amd.api.plan_uniform(d.data_ptr() + off, stride, length, n)[1] == 12
            ss = rng.integers(0, 393211, n, dtype=np.uint32)
            got = u16(tcp_amd.batch_uniform(d, stride, length, n, to_dev(ss.view(np.int32), dev), offset=off))
            want = oracle.batch_uniform(host, stride, length, n, ss, offset=off)
            assert np.array_equal(got, want), (stride, length, off)
            for n2 in (1, 2, 63, 65):   # partial tiles
                got = u16(tcp_amd.batch_uniform(d, stride, length, n2, 7, offset=off))
                assert np.array_equal(got, oracle.batch_uniform(host, stride, length, n2, 7, offset=off))
    finally:
        tcp_amd.set_tuning(0, 0, -1, 0)


@pytest.mark.parametrize("shape", [-1, 8, 9])
def test_ipv4_region_bounds(dev, shape):
    """Reads never leave the region: a packet whose tot_len runs past it is skipped, offsets at the
    very end (no room for a header) are skipped, and the rest is still exact (lane-group and
    balanced kernels)."""
    import tcp_amd
    from tests.packets import ip_packet
    rng = np.random.default_rng(5)
    pkts = [ip_packet(rng, int(rng.integers(0, 1456))) for _ in range(40)]
    offs, pos = [], 0
    for p in pkts:
        offs.append(pos)
        pos += len(p)
    region = np.zeros(pos, np.uint8)
    for o, p in zip(offs, pkts):
        region[o:o + len(p)] = np.frombuffer(p, np.uint8)
    cut = offs[-1] + len(pkts[-1]) - 5            # last packet truncated by the region end
    region = region[:cut].copy()
    off = np.array(offs + [cut - 10, cut - 1], np.uint64)
    want_out, want_st = oracle.ipv4_batch(np.concatenate([region, np.zeros(64, np.uint8)]), off, 32768,
                                          tcp_amd.IPV4_FILL)
    # the oracle reads past the region for the cut packet; the device must skip it (region-bounded)
    want_st[-3:] = tcp_amd.PKT_SKIPPED
    want_out[-3:] = 0
    dreg = to_dev(region, dev)
    out = torch.empty(off.size, dtype=torch.int16, device=dev)
    st = torch.empty(off.size, dtype=torch.uint8, device=dev)
    tcp_amd.set_tuning(0, 0, shape, 0)
    try:
        tcp_amd.ipv4_batch(dreg, to_dev(off.view(np.int64), dev), off.size, 32768, tcp_amd.IPV4_FILL, out, st)
    finally:
        tcp_amd.set_tuning(0, 0, -1, 0)
    assert np.array_equal(host(st), want_st)
    assert np.array_equal(u16(out)[:-3], want_out[:-3])


@pytest.mark.parametrize("shape", range(10))
def test_ipv4_forced_shapes(dev, shape):
    """Every wire lane-group shape (tcpcsum.h: wire 0..7) and tile depth is exact, incl. IHL 5..15,
    odd offsets and malformed packets; the header fields come from the group's chunk registers."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(900 + shape)
    region, off, _ = build_batch(rng, 700, malformed=True, odd_offsets=True)
    for mode in (tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR, tcp_amd.IPV4_VERIFY):
        ref = region.copy()
        want_out, want_st = oracle.ipv4_batch(ref, off, 32768, mode)
        for un in (1, 2, 4):
            for mb, fl in ((0, 0), (3, 0), (0, tcp_amd.TUNE_WIN16), (3, tcp_amd.TUNE_WIN16 | tcp_amd.TUNE_WIRE_CACHED)):
                tcp_amd.set_tuning(mb, un, shape, fl)
                try:
                    dreg = to_dev(region, dev)
                    out = torch.empty(off.size, dtype=torch.int16, device=dev)
                    st = torch.empty(off.size, dtype=torch.uint8, device=dev)
                    tcp_amd.ipv4_batch(dreg, to_dev(off.view(np.int64), dev), off.size, 32768, mode, out, st)
                finally:
                    tcp_amd.set_tuning(0, 0, -1, 0)
                assert np.array_equal(host(st), want_st), (mode, un, mb, fl)
                assert np.array_equal(u16(out), want_out), (mode, un, mb, fl)
                assert np.array_equal(host(dreg), ref), (mode, un, mb, fl)
        region = ref   # VERIFY runs over the filled packets


@pytest.mark.parametrize("shape", [8, 9])
@pytest.mark.parametrize("align", [4, 16])
def test_ipv4_balanced_head_path(dev, shape, align):
    """The balanced wire kernel on tiles of 4-B aligned packets — the path that takes each packet's
    first 64 bytes in registers (header, first TCP bytes, a control segment whole, the FILL's check
    word) and sweeps only the rest: control segments beside MTU ones, IHL 5..15 (the TCP start and
    the check word past the 64 bytes), malformed packets, a packet cut by the region end and an
    offset with no room for a header; FILL then VERIFY for every tile size, against the oracle, the
    whole region byte-identical. IPHDR batches take the other path and are checked too."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(41 + shape + align)
    region, off, _ = build_batch(rng, 1200, malformed=True, align=align, control_every=2)
    cut = int(off[-1]) + 30                   # the last packet runs past the region: skipped
    off = np.concatenate([off, np.array([cut - 10], np.uint64)])  # no room for a header: skipped
    region = region[:cut].copy()
    for mode in (tcp_amd.IPV4_FILL, tcp_amd.IPV4_VERIFY, tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR):
        ref = np.concatenate([region, np.zeros(64, np.uint8)])
        want_out, want_st = oracle.ipv4_batch(ref, off, 32768, mode)
        want_st[-2:] = tcp_amd.PKT_SKIPPED
        want_out[-2:] = 0
        ref = ref[:cut]
        # the oracle filled the cut packet from the padding it read past the region: undo that
        ref[int(off[-2]):] = region[int(off[-2]):]
        for un in (1, 2, 4):
            tcp_amd.set_tuning(0, un, shape, 0)
            try:
                dreg = to_dev(region, dev)
                out = torch.empty(off.size, dtype=torch.int16, device=dev)
                st = torch.empty(off.size, dtype=torch.uint8, device=dev)
                tcp_amd.ipv4_batch(dreg, to_dev(off.view(np.int64), dev), off.size, 32768, mode, out, st)
            finally:
                tcp_amd.set_tuning(0, 0, -1, 0)
            assert np.array_equal(host(st), want_st), (mode, un)
            assert np.array_equal(u16(out), want_out), (mode, un)
            assert np.array_equal(host(dreg), ref), (mode, un)
        if mode == tcp_amd.IPV4_FILL:
            region = ref   # VERIFY runs over the filled packets


@pytest.mark.parametrize("layout", ["packed4", "slots1536", "sparse", "shuffled", "repeated", "tiny_hulls"])
@pytest.mark.parametrize("shape", [8, 9])
def test_ipv4_balanced_layouts(dev, shape, layout):
    """Balanced wire kernel over offset layouts a tile may see: packed 4-B aligned, MTU slots,
    sparse 32 KiB slots, shuffled order, every packet listed twice (VERIFY only) and packets
    whose offsets lie closer than 16 B (malformed, then valid ones in the same tile). Tiles in
    address order, non-overlapping and dense may be swept as one run (the span path); every
    other layout must give the same results through the per-packet sweep."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(77 + shape)
    n = 700
    if layout == "packed4":
        region, off, _ = build_batch(rng, n, malformed=True, align=4, control_every=3)
    elif layout == "slots1536":
        region, off, _ = build_batch(rng, n, slot=1536, malformed=True)
    elif layout == "sparse":
        region, off, _ = build_batch(rng, 96, slot=32768, malformed=True)
    else:
        region, off, _ = build_batch(rng, n, malformed=True, align=16, control_every=2)
        if layout == "shuffled":
            off = off[rng.permutation(off.size)]
        elif layout == "repeated":
            off = np.repeat(off, 2)
        elif layout == "tiny_hulls":   # offsets 4 and 8 B into a packet: headers that fail to parse
            extra = off[::5] + np.uint64(8)
            off = np.sort(np.concatenate([off, extra]))
    modes = [tcp_amd.IPV4_VERIFY] if layout in ("repeated", "tiny_hulls") else [tcp_amd.IPV4_FILL, tcp_amd.IPV4_VERIFY]
    for mode in modes:
        ref = region.copy()
        want_out, want_st = oracle.ipv4_batch(ref, off, 32768, mode)
        for un in (1, 2):
            tcp_amd.set_tuning(0, un, shape, 0)
            try:
                dreg = to_dev(region, dev)
                out = torch.empty(off.size, dtype=torch.int16, device=dev)
                st = torch.empty(off.size, dtype=torch.uint8, device=dev)
                tcp_amd.ipv4_batch(dreg, to_dev(off.view(np.int64), dev), off.size, 32768, mode, out, st)
            finally:
                tcp_amd.set_tuning(0, 0, -1, 0)
            assert np.array_equal(host(st), want_st), (mode, un)
            assert np.array_equal(u16(out), want_out), (mode, un)
            assert np.array_equal(host(dreg), ref), (mode, un)
        if mode == tcp_amd.IPV4_FILL:
            region = ref


@pytest.mark.parametrize("shape", range(9))
def test_desc_forced_shapes(dev, shape):
    """Every ragged lane-group shape (tcpcsum.h: ragged 0..6, balanced 7..8) and tile depth is exact
    on lengths 0..9000 at arbitrary offsets."""
    import tcp_amd
    rng = np.random.default_rng(700 + shape)
    size = 2 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    n = 2500
    lens = rng.choice(np.array([0, 1, 2, 3, 15, 16, 17, 64, 576, 1500, 9000], np.uint32), n)
    off = np.array([rng.integers(0, size - l) for l in lens], np.uint64)
    ss = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch_desc(host, off, lens, ss)
    d = to_dev(host, dev)
    dd = to_dev(_desc(off, lens, ss), dev)
    for un in (1, 2, 4):
        for mb in (0, 5):
            tcp_amd.set_tuning(mb, un, shape, 0)
            try:
                got = u16(tcp_amd.batch_desc(d, dd, n, 9000))
            finally:
                tcp_amd.set_tuning(0, 0, -1, 0)
            assert np.array_equal(got, want), (un, mb)


@pytest.mark.parametrize("shape", [7, 8])
@pytest.mark.parametrize("mix", ["all4", "one_odd_len", "one_odd_start"])
def test_desc_balanced_dword_tiles(dev, shape, mix):
    """Balanced kernels on tiles whose segments are all 4-B aligned in start and length (the
    dword-mask path: packed IPv4/TCP, IMIX) and on tiles where one segment breaks it."""
    import tcp_amd
    rng = np.random.default_rng({"all4": 1, "one_odd_len": 2, "one_odd_start": 3}[mix] + 10 * shape)
    size = 4 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    n = 3000
    lens = rng.choice(np.array([0, 4, 20, 60, 64, 576, 1480, 1500, 9000], np.uint32), n)
    off = (np.array([rng.integers(0, (size - l) // 4) for l in lens], np.uint64) * 4).astype(np.uint64)
    if mix == "one_odd_len":
        lens[::97] += 1
    elif mix == "one_odd_start":
        off[::89] += 2
    ss = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch_desc(host, off, lens, ss)
    d = to_dev(host, dev)
    dd = to_dev(_desc(off, lens, ss), dev)
    got = u16(tcp_amd.batch_desc(d, dd, n, 9001, tune=tcp_amd.make_tuning(0, 0, shape, 0)))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("shape", [8, 9])
def test_ipv4_balanced_dword_tiles(dev, shape):
    """Packed packets whose lengths are multiples of 4 (every tile on the dword-mask path), mixed with
    stretches of arbitrary lengths; FILL then VERIFY, against the oracle."""
    import tcp_amd
    from tests.packets import ip_packet
    rng = np.random.default_rng(90 + shape)
    pk, offs, pos = [], [], 0
    for i in range(4000):
        a4 = (i // 200) % 3 != 0
        pl = int(rng.integers(0, 365)) * 4 if a4 else int(rng.integers(0, 1457))
        if a4:
            pos = (pos + 3) & ~3
        pk.append(ip_packet(rng, pl))
        offs.append(pos)
        pos += len(pk[-1])
    off = np.array(offs, np.uint64)
    region = np.zeros(int(off[-1]) + len(pk[-1]) + 64, np.uint8)
    for o, p in zip(off, pk):
        region[int(o):int(o) + len(p)] = np.frombuffer(p, np.uint8)
    for mode in (tcp_amd.IPV4_FILL, tcp_amd.IPV4_VERIFY):
        ref = region.copy()
        want_out, want_st = oracle.ipv4_batch(ref, off, 1536, mode)
        dreg = to_dev(region, dev)
        out = torch.empty(off.size, dtype=torch.int16, device=dev)
        st = torch.empty(off.size, dtype=torch.uint8, device=dev)
        tcp_amd.ipv4_batch(dreg, to_dev(off.view(np.int64), dev), off.size, 1536, mode, out, st,
                           tune=tcp_amd.make_tuning(0, 0, shape, 0))
        assert np.array_equal(host(st), want_st), mode
        assert np.array_equal(u16(out), want_out), mode
        assert np.array_equal(host(dreg), ref), mode
        region = ref


@pytest.mark.parametrize("shape", [-1, 1, 3, 8, 9])
def test_ipv4_span_hint_mispredicted(dev, shape):
    """The next packet's offset only bounds the speculative span: shuffled offsets (gaps unrelated
    to lengths, negative gaps) and extra offsets inside packets (gap < tot_len: fix-up loads) are
    still exact."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(1234)
    region, off, _ = build_batch(rng, 600, malformed=True, odd_offsets=True)
    perm = rng.permutation(off.size)
    inside = off[rng.integers(0, off.size, 200)] + rng.integers(1, 90, 200).astype(np.uint64)
    cases = {"shuffled": (off[perm], (tcp_amd.IPV4_FILL, tcp_amd.IPV4_VERIFY)),
             "interleaved": (np.insert(off, rng.integers(0, off.size, 200), inside), (tcp_amd.IPV4_VERIFY,))}
    for name, (offs, modes) in cases.items():
        offs = np.ascontiguousarray(offs, np.uint64)
        reg = region.copy()
        for mode in modes:
            ref = reg.copy()
            want_out, want_st = oracle.ipv4_batch(ref, offs, 32768, mode)
            tcp_amd.set_tuning(0, 0, shape, 0)
            try:
                dreg = to_dev(reg, dev)
                out = torch.empty(offs.size, dtype=torch.int16, device=dev)
                st = torch.empty(offs.size, dtype=torch.uint8, device=dev)
                tcp_amd.ipv4_batch(dreg, to_dev(offs.view(np.int64), dev), offs.size, 32768, mode, out, st)
            finally:
                tcp_amd.set_tuning(0, 0, -1, 0)
            assert np.array_equal(host(st), want_st), name
            assert np.array_equal(u16(out), want_out), name
            assert np.array_equal(host(dreg), ref), name
            reg = ref


@pytest.mark.parametrize("shape,flags", [(-1, 0), (-1, 32), (-1, 64), (-1, 96), (8, 0), (9, 0),
                                         (-1, 256), (-1, 320), (0, 256), (1, 256),
                                         (-1, 512), (-1, 576), (5, 512), (1, 0), (2, 0), (4, 0), (5, 0), (7, 0),
                                         (-1, 544), (-1, 2048), (1, 2048), (5, 2048), (7, 2048)])
@pytest.mark.parametrize("layout", ["odd", "slot64", "slot16", "packed", "jumbo"])
def test_ipv4_window_and_store_variants(dev, shape, flags, layout):
    """Wire kernel variants (128-B or 16-B packet windows; non-temporal or default-policy loads;
    check|urg_ptr dword stores; the default whole-line write-through stores, 64-B block stores
    (TUNE_FILL_HALF) or forced 2-byte stores) are exact and FILL rewrites nothing but the checks, in every
    layout: odd packed offsets, 64-B aligned slots, 16-B (not 64-B) aligned slots, packed tiny
    packets, 9000-B jumbo frames at odd offsets (the multi-round path)."""
    import tcp_amd
    from tests.packets import build_batch, ip_packet
    rng = np.random.default_rng(4242 + flags)
    if layout == "odd":
        region, off, _ = build_batch(rng, 600, malformed=True, odd_offsets=True)
    elif layout == "jumbo":
        region, off, _ = build_batch(rng, 120, malformed=True, odd_offsets=True, max_payload=8956)
    elif layout in ("slot64", "slot16"):
        region, off, _ = build_batch(rng, 400, slot=1536, malformed=True)
        if layout == "slot16":
            region = np.concatenate([np.zeros(16, np.uint8), region])
            off = off + np.uint64(16)
    else:
        pkts = [ip_packet(rng, int(rng.integers(0, 40))) for _ in range(900)]
        off = np.cumsum([0] + [len(p) for p in pkts[:-1]]).astype(np.uint64)
        region = np.zeros(int(off[-1]) + len(pkts[-1]), np.uint8)
        for o, p in zip(off, pkts):
            region[int(o):int(o) + len(p)] = np.frombuffer(p, np.uint8)
    for mode in (tcp_amd.IPV4_FILL, tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR, tcp_amd.IPV4_VERIFY | tcp_amd.IPV4_IPHDR):
        ref = region.copy()
        want_out, want_st = oracle.ipv4_batch(ref, off, 1536 if layout not in ("odd", "jumbo") else 32768, mode)
        tcp_amd.set_tuning(0, 0, shape, flags)
        try:
            dreg = to_dev(region, dev)
            out = torch.empty(off.size, dtype=torch.int16, device=dev)
            st = torch.empty(off.size, dtype=torch.uint8, device=dev)
            tcp_amd.ipv4_batch(dreg, to_dev(off.view(np.int64), dev), off.size,
                               1536 if layout not in ("odd", "jumbo") else 32768, mode, out, st)
        finally:
            tcp_amd.set_tuning(0, 0, -1, 0)
        assert np.array_equal(host(st), want_st), mode
        assert np.array_equal(u16(out), want_out), mode
        assert np.array_equal(host(dreg), ref), mode
        region = ref   # the VERIFY pass runs over filled packets


@pytest.mark.parametrize("shape", [7, 8])
def test_desc_balanced_long_segments(dev, shape):
    """The balanced ragged kernel on tiles that mix tiny, 64 KiB and > 1 MiB segments (the latter
    summed by the whole wave) at odd offsets, with byte values that push sums above 2^32."""
    import tcp_amd
    rng = np.random.default_rng(88 + shape)
    size = 24 << 20
    host = rng.integers(200, 256, size, dtype=np.uint8)
    n = 300
    lens = rng.choice(np.array([0, 1, 3, 64, 1500, 65536, 65537, 300000, (1 << 20) + 1, 3 << 20], np.uint32), n)
    off = np.array([rng.integers(0, size - l) for l in lens], np.uint64)
    ss = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch_desc(host, off, lens, ss)
    d = to_dev(host, dev)
    dd = to_dev(_desc(off, lens, ss), dev)
    tcp_amd.set_tuning(0, 0, shape, 0)
    try:
        got = u16(tcp_amd.batch_desc(d, dd, n, int(lens.max())))
    finally:
        tcp_amd.set_tuning(0, 0, -1, 0)
    assert np.array_equal(got, want)


def test_host_context_staging_reuse_and_null_outputs(dev):
    """One context across wire batches of growing / shrinking size (its pinned staging of offsets,
    results and status is reallocated and reused), pageable and pinned regions, and the C ABI's
    NULL h_out / h_status (FILL still patches the packets)."""
    import ctypes
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(515)
    with tcp_amd.HostContext(0) as ctx:
        for n, pinned in ((100, False), (3000, True), (1500, False), (5000, False), (7, True)):
            region, off, _ = build_batch(rng, n, slot=1536, malformed=True, max_payload=1400)
            ref = region.copy()
            want_out, want_st = oracle.ipv4_batch(ref, off, 1536, tcp_amd.IPV4_FILL)
            buf = region
            if pinned:
                buf = tcp_amd.pinned_empty(region.size)
                buf[:] = region
            out, st = ctx.ipv4_batch(buf, off, 1536, tcp_amd.IPV4_FILL)
            assert np.array_equal(st, want_st) and np.array_equal(out, want_out), (n, pinned)
            assert np.array_equal(np.asarray(buf), ref), (n, pinned)
        # NULL outputs through the raw ABI
        region, off, _ = build_batch(rng, 800, slot=1536, malformed=True)
        ref = region.copy()
        oracle.ipv4_batch(ref, off, 1536, tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR)
        off = np.ascontiguousarray(off, np.uint64)
        rc = tcp_amd.lib().tcpcsum_ipv4_batch_host(ctx._h, region.ctypes.data, region.nbytes, off.ctypes.data,
                                                   off.size, 1536, tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR,
                                                   None, None)
        assert rc == 0
        assert np.array_equal(region, ref)


@pytest.mark.parametrize("shape", [7, 8])
def test_desc_balanced_tile_edges(dev, shape):
    """Balanced ragged kernel at tile edges: n = 1, 63, 64, 65, 129 segments; all-empty tiles; a
    single segment spanning many windows; segments sharing bytes (overlapping descriptors)."""
    import tcp_amd
    rng = np.random.default_rng(shape)
    size = 1 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    d = to_dev(host, dev)
    cases = []
    for n in (1, 63, 64, 65, 129):
        lens = rng.integers(0, 3000, n).astype(np.uint32)
        cases.append(lens)
    cases.append(np.zeros(130, np.uint32))                       # nothing to sum
    cases.append(np.array([0] * 10 + [200000] + [0] * 60, np.uint32))   # one long segment
    for lens in cases:
        n = lens.size
        off = np.array([rng.integers(0, size - l) for l in lens], np.uint64)
        if n > 3:
            off[1] = off[0]                                      # identical / overlapping descriptors
        ss = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        tcp_amd.set_tuning(0, 0, shape, 0)
        try:
            got = u16(tcp_amd.batch_desc(d, to_dev(_desc(off, lens, ss), dev), n, int(max(lens.max(), 1))))
        finally:
            tcp_amd.set_tuning(0, 0, -1, 0)
        assert np.array_equal(got, oracle.batch_desc(host, off, lens, ss)), n


@pytest.mark.parametrize("shape", [7, 8])
@pytest.mark.parametrize("max_len", [1500, 4096, 9000, 40000, 65536])
def test_desc_balanced_segments_per_wave(dev, shape, max_len):
    """The balanced kernel's wave tile holds fewer segments as max_len grows (64 at 1.5 KiB down
    to 1 at 64 KiB): tiles of every size, ragged lengths up to max_len, odd offsets, batches that
    end mid-tile — exact against the oracle."""
    import tcp_amd
    rng = np.random.default_rng(max_len + shape)
    size = 24 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    d = to_dev(host, dev)
    n = int(min(3001, (size // max_len) * 2 + 3))
    lens = rng.integers(0, max_len + 1, n).astype(np.uint32)
    lens[::5] = max_len
    off = np.array([rng.integers(0, size - l) for l in lens], np.uint64)
    ss = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    tcp_amd.set_tuning(0, 0, shape, 0)
    try:
        got = u16(tcp_amd.batch_desc(d, to_dev(_desc(off, lens, ss), dev), n, max_len))
    finally:
        tcp_amd.set_tuning(0, 0, -1, 0)
    assert np.array_equal(got, oracle.batch_desc(host, off, lens, ss))


@pytest.mark.parametrize("slot,max_payload", [(2048, 1990), (4608, 4500)])
def test_ipv4_large_batch_size_classes(dev, slot, max_payload):
    """Large wire batches of 2-4.5 KiB packets take the 4- / 6-chunk-round shapes by size class
    (auto); FILL then VERIFY, every result and every byte of the region against the oracle."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(slot)
    n = 65536
    region, off, _ = build_batch(rng, n, slot=slot, malformed=True, max_payload=max_payload)
    ref = region.copy()
    want_out, want_st = oracle.ipv4_batch(ref, off, slot, tcp_amd.IPV4_FILL)
    dreg = to_dev(region, dev)
    doff = to_dev(off.view(np.int64), dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    tcp_amd.ipv4_batch(dreg, doff, n, slot, tcp_amd.IPV4_FILL, out, st)
    assert np.array_equal(host(st), want_st)
    assert np.array_equal(u16(out), want_out)
    assert np.array_equal(host(dreg), ref)
    tcp_amd.ipv4_batch(dreg, doff, n, slot, tcp_amd.IPV4_VERIFY, out, st)
    ok = want_st == tcp_amd.PKT_OK
    assert np.all(u16(out)[ok] == 0) and np.array_equal(host(st), want_st)
