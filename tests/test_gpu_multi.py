"""GPU parity for tcpcsum_batch_uniform_multi_dev: several uniform batches in one launch.

Batch j must come out exactly as tcpcsum_batch_uniform_dev would compute it —
csum_continue (/root/reference/context.c:121-145) per segment with its start
value — whatever the mix of lengths, alignments, start-value forms and sizes
shares the launch. Checked against the oracle on every batch, and on the
BASELINE 64-B config against the reference's Appendix B digest.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from tests.tensors import to_dev, u16  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    import tcp_amd
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rc, arch = tcp_amd.device_check()
    assert rc == 0, f"tcpcsum_device_check -> {rc} ({arch})"
    return torch.device("cuda:0")


def _run(dev, rng, specs, tune=None):
    """specs: (stride, length, n, offset, ss_kind) per batch; each batch gets its own host buffer.
    Returns the list of (got, want)."""
    import tcp_amd
    batches, wants, outs = [], [], []
    for stride, length, n, offset, ss_kind in specs:
        size = offset + max(0, (n - 1)) * stride + length + 64
        host = rng.integers(0, 256, size, dtype=np.uint8)
        d = to_dev(host, dev)
        if ss_kind == "array":
            ss_h = rng.integers(0, 6 * 0xFFFF + 1, max(n, 1), dtype=np.uint32)
            ss = to_dev(ss_h.view(np.int32), dev)
            want = oracle.batch_uniform(host, stride, length, n, ss_h[:n], offset=offset)
        else:
            ss = int(rng.integers(0, 6 * 0xFFFF + 1))
            want = oracle.batch_uniform(host, stride, length, n, ss, offset=offset)
        out = torch.full((max(n, 1) + 8,), 0x5a5a, dtype=torch.int16, device=dev)
        batches.append((d, stride, length, n, ss, out, offset))
        wants.append(want)
        outs.append((out, n))
    tcp_amd.batch_uniform_multi(batches, tune=tune)
    res = []
    for (out, n), want in zip(outs, wants):
        o = u16(out)
        assert np.all(o[n:] == 0x5a5a), "a batch wrote past its n results"
        res.append((o[:n], want))
    return res


def test_multi_64b_batches(dev):
    """The BASELINE small-segment shape: sixteen batches of 64-B segments, 16-B aligned."""
    rng = np.random.default_rng(64)
    specs = [(64, 64, int(rng.integers(1, 20000)), 0, "array" if j % 2 else "scalar") for j in range(16)]
    for j, (got, want) in enumerate(_run(dev, rng, specs)):
        assert np.array_equal(got, want), j


@pytest.mark.parametrize("mix", ["aligned", "dword", "bytes", "lane_shapes"])
def test_multi_mixed_batches(dev, mix):
    """Batches of different lengths, strides, alignments and start-value forms in one launch (the
    launch runs in the most general mode and the widest shape any of them needs)."""
    rng = np.random.default_rng({"aligned": 1, "dword": 2, "bytes": 3, "lane_shapes": 4}[mix])
    if mix == "aligned":
        specs = [(64, 64, 5000, 0, "array"), (128, 112, 3000, 16, "scalar"), (1504, 1504, 2000, 0, "array"),
                 (64, 48, 1, 0, "scalar"), (2048, 2048, 700, 32, "array")]
    elif mix == "dword":
        specs = [(1500, 1500, 4000, 0, "array"), (64, 64, 6000, 4, "scalar"), (1500, 1480, 999, 12, "array"),
                 (84, 84, 3333, 8, "scalar")]
    elif mix == "bytes":
        specs = [(1501, 1499, 1000, 1, "array"), (64, 63, 7000, 3, "scalar"), (101, 97, 600, 5, "array"),
                 (2, 1, 9000, 0, "scalar"), (1500, 1500, 2000, 0, "array")]
    else:
        specs = [(L + 3, L, 800, 0, "array") for L in (16, 40, 120, 250, 500, 1000, 1500, 2000, 4096, 8000)]
    for j, (got, want) in enumerate(_run(dev, rng, specs)):
        assert np.array_equal(got, want), (mix, j, specs[j])


def test_multi_long_segments_fall_back(dev):
    """Segments past the lane-group shapes (jumbo, 64 KiB, odd) beside short ones: launched batch by
    batch, still exact; empty batches do nothing."""
    rng = np.random.default_rng(5)
    specs = [(9000, 9000, 40, 0, "array"), (64, 64, 3000, 0, "scalar"), (65536, 65536, 6, 0, "scalar"),
             (12301, 12301, 9, 1, "array"), (64, 64, 0, 0, "scalar"), (1500, 1500, 100, 4, "array")]
    for j, (got, want) in enumerate(_run(dev, rng, specs)):
        assert np.array_equal(got, want), j


def test_multi_more_than_one_launch_and_tuning(dev):
    """More batches than TCPCSUM_MULTI_MAX (split over launches), and forced grids / unrolls /
    thin lane-group shapes."""
    import tcp_amd
    rng = np.random.default_rng(6)
    specs = [(64 + 4 * (j % 3), 64, int(rng.integers(100, 3000)), 4 * (j % 4), "array" if j % 3 else "scalar")
             for j in range(37)]
    for j, (got, want) in enumerate(_run(dev, rng, specs)):
        assert np.array_equal(got, want), j
    for tune in ((1, 0, -1, 0), (7, 8, -1, 0), (0, 2, 10, 0), (0, 1, 11, 0), (0, 4, 3, 0)):
        t = tcp_amd.make_tuning(*tune)
        specs = [(68, 64, 2000, 4, "array"), (64, 40, 1500, 0, "scalar"), (80, 80, 1111, 0, "array")]
        for j, (got, want) in enumerate(_run(dev, rng, specs, tune=t)):
            assert np.array_equal(got, want), (tune, j)


def test_multi_baseline_64b_digest(dev, golden):
    """Sixteen copies of BASELINE's 1M x 64-B batch (Appendix B) in one launch: every batch's
    results match the reference's digest."""
    import tcp_amd
    n, L = 1 << 20, 64
    data = torch.empty(n * L, dtype=torch.uint8, device=dev)
    tcp_amd.synth_fill(data, 0, n * L)
    ss = torch.empty(n, dtype=torch.int32, device=dev)
    tcp_amd.synth_pseudo(ss, 0, n, L)
    outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(16)]
    tcp_amd.batch_uniform_multi([(data, L, L, n, ss, o) for o in outs])
    g = golden["digests"]["1Mx64"]
    for o in outs:
        r = u16(o)
        assert int(r.astype(np.uint64).sum()) == g["sum"] and f"{int(np.bitwise_xor.reduce(r)):04x}" == g["xor"]
        assert oracle.digest(r)[0] == g["fnv1a64"]
