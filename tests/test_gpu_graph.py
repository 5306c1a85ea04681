"""Device entry points captured into a HIP graph and replayed.

A loop that flushes batch after batch (``releaseSend``, /root/reference/loop.c:27-94) can capture
its launches once and replay them: every device entry point is asynchronous on the caller's
stream, allocates nothing, never synchronises and takes its descriptors by value (the multi-batch
launch reads its batch table out of the kernel-argument segment), so it captures. These tests
capture each one with ``torch.cuda.graph``, replay it, and compare with the oracle — including
after the input bytes were rewritten in place, which shows the graph reads live memory rather than
anything fixed at capture time.
"""
import numpy as np
import pytest

import oracle
from tests.tensors import host, to_dev, u16

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    import tcp_amd
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, arch = tcp_amd.device_check()
    assert rc == 0, f"tcpcsum_device_check -> {rc} ({arch})"
    return torch.device("cuda:0")


def _capture(fn):
    """fn() once eagerly on a side stream (warm-up, as torch.cuda.graph asks), then captured."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def test_uniform_graph_replay(dev):
    import tcp_amd
    rng = np.random.default_rng(71)
    n, L = 20000, 1500
    a = rng.integers(0, 256, n * L, dtype=np.uint8)
    ss = rng.integers(0, 1 << 19, n, dtype=np.uint32)
    data, dss = to_dev(a, dev), to_dev(ss.view(np.int32), dev)
    out = torch.zeros(n, dtype=torch.int16, device=dev)
    g = _capture(lambda: tcp_amd.batch_uniform(data, L, L, n, dss, out=out))
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(u16(out), oracle.batch_uniform(a, L, L, n, ss))
    # new bytes in the same buffer: the replay sees them
    b = rng.integers(0, 256, n * L, dtype=np.uint8)
    data.copy_(to_dev(b, dev))
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(u16(out), oracle.batch_uniform(b, L, L, n, ss))


def test_multi_batch_graph_replay(dev):
    """Four small-segment batches in one launch, its batch table captured by value."""
    import tcp_amd
    rng = np.random.default_rng(72)
    specs = [(4096, 64, 64), (3000, 80, 64), (5000, 64, 61), (777, 1500, 1500)]
    hosts, batches, outs = [], [], []
    for j, (n, stride, L) in enumerate(specs):
        a = rng.integers(0, 256, n * stride, dtype=np.uint8)
        o = torch.zeros(n, dtype=torch.int16, device=dev)
        hosts.append((a, n, stride, L, 1000 + j))
        batches.append((to_dev(a, dev), stride, L, n, 1000 + j, o))
        outs.append(o)
    arr = tcp_amd.ubatches(batches)
    g = _capture(lambda: tcp_amd.batch_uniform_multi(arr))
    for o in outs:
        o.zero_()
    g.replay()
    torch.cuda.synchronize()
    for (a, n, stride, L, s0), o in zip(hosts, outs):
        assert np.array_equal(u16(o), oracle.batch_uniform(a, stride, L, n, s0)), (n, stride, L)


def test_ipv4_fill_graph_replay(dev):
    """Wire FILL in place (context.c:208) from a graph: the replay over freshly written packets
    fills them exactly as the oracle does, malformed packets included (skipped, untouched)."""
    import tcp_amd
    from tests.packets import build_batch
    rng = np.random.default_rng(73)
    n = 2048
    region, off, _ = build_batch(rng, n, slot=2048, malformed=True)
    want = region.copy()
    want_out, want_st = oracle.ipv4_batch(want, off, 2048, tcp_amd.IPV4_FILL)
    dreg, doff = to_dev(region, dev), to_dev(off.view(np.int64), dev)
    out = torch.zeros(n, dtype=torch.int16, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    g = _capture(lambda: tcp_amd.ipv4_batch(dreg, doff, n, 2048, tcp_amd.IPV4_FILL, out, st))
    dreg.copy_(to_dev(region, dev))   # the capture's warm-up filled them: start again from the wire
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(host(dreg), want)
    assert np.array_equal(u16(out), want_out)
    assert np.array_equal(host(st), want_st)


def test_tx_build_graph_replay(dev):
    import tcp_amd
    from tests.test_oracle import make_txsegs
    rng = np.random.default_rng(74)
    payload = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    n = 1500
    segs, size = make_txsegs(rng, n, payload.size, max_len=1456)
    want = np.zeros(size, np.uint8)
    want_c = oracle.tx_build(payload, segs, want)
    dpay, dseg = to_dev(payload, dev), to_dev(segs.view(np.uint8), dev)
    dout = torch.zeros(size, dtype=torch.uint8, device=dev)
    chk = torch.zeros(n, dtype=torch.int16, device=dev)
    g = _capture(lambda: tcp_amd.tx_build(dpay, dseg, n, 1456, dout, 0, chk))
    dout.zero_()
    chk.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(host(dout), want)
    assert np.array_equal(u16(chk), want_c)
