"""GPU fuzz parity for the wire kernels: random bytes shaped into IPv4/TCP packets.

Each trial fills a region with random bytes and lays packets into it with
random gaps and odd alignments; most headers are made valid (version 4, IHL
5..15, protocol 6, tot_len matching the packet), the rest are left or made
invalid (random version/protocol/IHL, tot_len too small, above cap, random).
Lengths mix tiny, IMIX, MTU and jumbo. Every wire kernel shape (lane groups
0..7, balanced 8..9, auto) in FILL, FILL|IPHDR, VERIFY and VERIFY|IPHDR is
compared with the oracle (the reference's context.c:104-145 / :169-209
restated) on out, status and every byte of the region. FILL packets never
overlap (the reference writes each check into its own buffer); VERIFY batches
may overlap, since nothing is written.
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
    assert rc == 0, f"tcpcsum_device_check -> {rc} ({arch})"
    return torch.device("cuda:0")


def make_batch(rng, n, overlap):
    lens = rng.choice(np.array([20, 40, 44, 64, 84, 300, 596, 1500, 1520, 4000, 9000]), n,
                      p=[.04, .06, .1, .15, .1, .1, .15, .15, .05, .05, .05])
    lens = lens + rng.integers(0, 4, n) * (rng.random(n) < 0.4)      # some lengths not 4-B multiples
    offs, pos = [], int(rng.integers(0, 64))
    for L in lens:
        offs.append(pos)
        pos += int(L) + int(rng.integers(0, 24))
        if overlap and rng.random() < 0.3:
            pos = max(offs[-1] + 1, pos - int(rng.integers(0, int(L) + 1)))   # next packet inside this one
    size = pos + 65536 + 64          # never bounded by the region end
    region = rng.integers(0, 256, size, dtype=np.uint8)
    for o, L in zip(offs, lens):
        kind = rng.random()
        ihl = int(rng.integers(5, 16)) if rng.random() < 0.3 else 5
        if L < ihl * 4 + 20:
            ihl = 5
        region[o] = (4 << 4) | ihl
        region[o + 9] = 6
        tot = int(L)
        if kind < 0.06:
            region[o] = int(rng.integers(0, 256))                  # random version / IHL
        elif kind < 0.10:
            region[o + 9] = int(rng.integers(0, 256))              # random protocol
        elif kind < 0.14:
            tot = int(rng.integers(0, ihl * 4 + 20))               # too short for a TCP header
        elif kind < 0.18:
            # anything — but a FILL batch's packets stay inside their own bytes (the
            # check store of one must not land in another packet being summed)
            tot = int(rng.integers(0, 65536)) if overlap else int(rng.integers(0, int(L) + 1))
        region[o + 2], region[o + 3] = tot >> 8, tot & 255
    return region, np.array(offs, np.uint64)


@pytest.mark.parametrize("seed", range(6))
def test_wire_fuzz_vs_oracle(dev, seed):
    import tcp_amd
    rng = np.random.default_rng(1000 + seed)
    for mode in (tcp_amd.IPV4_FILL, tcp_amd.IPV4_FILL | tcp_amd.IPV4_IPHDR, tcp_amd.IPV4_VERIFY,
                 tcp_amd.IPV4_VERIFY | tcp_amd.IPV4_IPHDR):
        verify = bool(mode & tcp_amd.IPV4_VERIFY)
        region, off = make_batch(rng, 1200, overlap=verify)
        cap = int(rng.choice([64, 1536, 9216, 65535]))
        ref = region.copy()
        want_out, want_st = oracle.ipv4_batch(ref, off, cap, mode)
        doff = to_dev(off.view(np.int64), dev)
        for shape in (-1,) + tuple(range(10)):
            dreg = to_dev(region, dev)
            out = torch.empty(off.size, dtype=torch.int16, device=dev)
            st = torch.empty(off.size, dtype=torch.uint8, device=dev)
            tcp_amd.ipv4_batch(dreg, doff, off.size, cap, mode, out, st, tune=tcp_amd.make_tuning(0, 0, shape, 0))
            ctx = (seed, mode, shape, cap)
            assert np.array_equal(host(st), want_st), ctx
            assert np.array_equal(host(out).view(np.uint16), want_out), ctx
            assert np.array_equal(host(dreg), ref), ctx


@pytest.mark.parametrize("seed", range(4))
def test_wire_ptrs_fuzz_vs_oracle(dev, seed):
    """The same packets addressed one pointer each, in shuffled order, each bounded by a random
    per-packet length (at, above or below its tot_len): skipped exactly when tot_len exceeds it."""
    import tcp_amd
    rng = np.random.default_rng(2000 + seed)
    for mode in (tcp_amd.IPV4_FILL, tcp_amd.IPV4_VERIFY | tcp_amd.IPV4_IPHDR):
        verify = bool(mode & tcp_amd.IPV4_VERIFY)
        region, off = make_batch(rng, 1200, overlap=verify)
        perm = rng.permutation(off.size)
        off = off[perm]
        tot = np.array([(int(region[o + 2]) << 8) | int(region[o + 3]) for o in off], np.int64)
        lens = tot + rng.integers(-3, 4, off.size) * (rng.random(off.size) < 0.3)
        lens = np.where(rng.random(off.size) < 0.05, rng.integers(0, 80, off.size), lens)
        lens = np.clip(lens, 0, 65535).astype(np.uint32)
        cap = int(rng.choice([1536, 65535]))
        ok = (lens >= 20) & (tot <= lens)
        ref = region.copy()
        want_out = np.zeros(off.size, np.uint16)
        want_st = np.full(off.size, tcp_amd.PKT_SKIPPED, np.uint8)
        if ok.any():
            o2, s2 = oracle.ipv4_batch(ref, off[ok], cap, mode)
            want_out[ok], want_st[ok] = o2, s2
        dreg = to_dev(region, dev)
        ptrs = to_dev((off + np.uint64(dreg.data_ptr())).view(np.int64), dev)
        dl = to_dev(lens.view(np.int32), dev)
        for shape in (-1, 0, 1, 3, 5, 8, 9):
            if not verify and shape != -1:
                dreg.copy_(to_dev(region, dev))
            out = torch.empty(off.size, dtype=torch.int16, device=dev)
            st = torch.empty(off.size, dtype=torch.uint8, device=dev)
            tcp_amd.ipv4_batch_ptrs(ptrs, dl, off.size, cap, mode, out, st, tune=tcp_amd.make_tuning(0, 0, shape, 0))
            ctx = (seed, mode, shape, cap)
            assert np.array_equal(host(st), want_st), ctx
            assert np.array_equal(host(out).view(np.uint16), want_out), ctx
            assert np.array_equal(host(dreg), ref), ctx
