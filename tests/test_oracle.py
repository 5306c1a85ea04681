"""CPU: the oracle (oracle/csum_oracle.c) pinned against the reference's own outputs.

Pins (tests/golden/reference_vectors.json, transcribed from SURVEY.md):
  * Appendix A KATs computed by /root/reference/context.c:104-145,
  * Appendix B digests of every BASELINE config computed by the same code.
Plus a cross-check against an independent Python restatement (tests/pyspec.py)
on random inputs, including odd lengths, negative nbytes and raw sums >= 2^32.
"""
import random
import socket

import numpy as np
import pytest

import oracle
from tests import pyspec


def test_generator_first_bytes(golden):
    assert oracle.gen_stream(0, 16).tobytes().hex() == golden["generator"]["first16"]
    # counter-based: any offset reproduces the same bytes
    a = oracle.gen_stream(0, 4096)
    for off in (1, 7, 8, 13, 1000):
        assert np.array_equal(oracle.gen_stream(off, 4096 - off), a[off:])


def test_kat_csum_continue(golden):
    for k in golden["kat_csum_continue"]:
        assert oracle.csum_continue(k["sum_start"], bytes.fromhex(k["bytes"]), k["nbytes"]) == int(k["out"], 16)


def test_kat_pseudo(golden):
    for k in golden["kat_pseudo"]:
        sa = socket.htonl(int(k["saddr_host"], 16))
        da = socket.htonl(int(k["daddr_host"], 16))
        len_be = socket.htons(k["len_host"] & 0xFFFF)   # u16 truncation: 65536 -> 0
        assert oracle.pseudo(sa, da, len_be) == k["out"]


@pytest.mark.parametrize("name", ["1Mx1500", "1Mx64", "256Kx64KiB"])
def test_appendix_b_digest(golden, name):
    g = golden["digests"][name]
    out = oracle.synth_batch(g["seg0"], g["n"], g["seg_len"])
    fnv, s, x = oracle.digest(out)
    assert (fnv, s, x) == (g["fnv1a64"], g["sum"], g["xor"])
    assert [f"{v:04x}" for v in out[:4]] == g["first4"]
    assert f"{out[-1]:04x}" == g["last"]


def test_appendix_b_8gpu_shards(golden):
    """8M x 1500 split in contiguous 1M shards: per-shard digests and the whole."""
    parts = []
    for k in range(8):
        g = golden["digests"][f"8Mx1500_shard{k}"]
        out = oracle.synth_batch(g["seg0"], g["n"], 1500)
        assert oracle.digest(out) == (g["fnv1a64"], g["sum"], g["xor"]), k
        parts.append(out)
    g = golden["digests"]["8Mx1500"]
    assert oracle.digest(np.concatenate(parts)) == (g["fnv1a64"], g["sum"], g["xor"])


def test_cross_check_pyspec_random():
    rng = random.Random(1234)
    for _ in range(400):
        n = rng.choice([0, 1, 2, 3, 4, 5, 17, 63, 64, 65, 1499, 1500, 1501, rng.randrange(0, 5000)])
        p = bytes(rng.getrandbits(8) for _ in range(n))
        ss = rng.choice([0, 1, 0xFFFF, 393210, rng.getrandbits(32), rng.getrandbits(40)])
        for nb in (n, n - 1 if n else 0, -5):
            assert oracle.csum_continue(ss, p, nb) == pyspec.csum_continue(ss, p, nb)
        sa, da, ln = rng.getrandbits(32), rng.getrandbits(32), rng.getrandbits(16)
        assert oracle.pseudo(sa, da, ln) == pyspec.pseudo(sa, da, ln)


def test_two_fold_differs_from_full_fold_above_4g():
    """Raw sum >= 2^32: the reference's exactly-two folds (context.c:140-141)."""
    p = b"\xff\xff" * 65538 + b"\x01\x00"   # S = 65538*0xFFFF + 1 = 0x1_0000_FFFF
    S = pyspec.exact_sum(0, p)
    assert S == 0x1_0000_FFFF
    full = S
    while full >> 16:
        full = (full & 0xFFFF) + (full >> 16)
    ref = oracle.csum_continue(0, p, len(p))
    assert ref == pyspec.csum_continue(0, p, len(p))
    assert ref != (~full) & 0xFFFF   # the divergence is real, and the oracle follows the reference


def test_zero_vs_ffff_not_conflated():
    # S == 0 -> 0xFFFF;  S > 0 with S % 65535 == 0 -> 0x0000  (Appendix A)
    assert oracle.csum_continue(0, b"\0" * 64, 64) == 0xFFFF
    assert oracle.csum_continue(0, b"\xff\xff", 2) == 0x0000


def test_verify_to_zero_property():
    rng = np.random.default_rng(7)
    for n in (24, 25, 64, 1480, 1501):
        seg = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        seg[16:18] = b"\0\0"
        ps = oracle.pseudo(rng.integers(0, 2**32), rng.integers(0, 2**32), socket.htons(n))
        c = oracle.csum_continue(ps, bytes(seg), n)
        seg[16:18] = c.to_bytes(2, "little")
        assert oracle.csum_continue(ps, bytes(seg), n) == 0


def test_oracle_ipv4_fill_then_verify():
    from tests.packets import build_batch
    region, off, _ = build_batch(np.random.default_rng(3), 64, malformed=True)
    out, st = oracle.ipv4_batch(region, off, 32768, 0)
    out2, st2 = oracle.ipv4_batch(region, off, 32768, 1)
    assert np.array_equal(st, st2)
    assert np.all(out2[st == 0] == 0)
    assert np.any(st == 1)


def test_cpu_bench_harness_runs():
    r = oracle.cpu_bench(2, 1500, 4096, 0.05)
    assert r["passes"] >= 5
    # best >= median >= the mean's harmonic counterpart; all positive
    assert r["best"] >= r["median"] > 0 and r["mean"] > 0
    # the harness checksums the Appendix B stream: its digest equals synth_batch's
    assert r["digest"] == oracle.digest(oracle.synth_batch(0, 4096, 1500))[0]


def test_oracle_ipv4_iphdr_fill_then_verify():
    """FILL|IPHDR writes an IPv4 header checksum that verifies; a flipped header byte is caught."""
    import struct
    from tests.packets import build_batch
    region, off, _ = build_batch(np.random.default_rng(4), 40, malformed=True)
    out, st = oracle.ipv4_batch(region, off, 32768, 0 | 2)
    ok = st == 0
    for o, good in zip(off, ok):
        if good:
            ihl = region[o] & 15
            hdr = region[o:o + 4 * ihl].tobytes()
            assert pyspec.csum_continue(0, hdr, len(hdr)) == 0
            # RFC 1071 form: complemented 16-bit big-endian sum of the header words is zero too
            words = struct.unpack("!%dH" % (2 * ihl), hdr)
            s = sum(words)
            while s >> 16:
                s = (s & 0xFFFF) + (s >> 16)
            assert s == 0xFFFF
    _, st2 = oracle.ipv4_batch(region, off, 32768, 1 | 2)
    assert np.array_equal(st2, st)
    bad = region.copy()
    first = int(off[np.flatnonzero(ok)[0]])
    bad[first + 8] ^= 1                                  # TTL
    _, st3 = oracle.ipv4_batch(bad, off, 32768, 1 | 2)
    assert st3[np.flatnonzero(ok)[0]] == 2


def make_txsegs(rng, n, payload_size, max_len=1456, odd=False, slot=None):
    """Random tx descriptors (TXSEG layout) with non-overlapping packets; returns (segs, out_size)."""
    import tcp_amd
    segs = np.zeros(n, tcp_amd.TXSEG_DTYPE)
    lens = rng.integers(0, max_len + 1, n)
    lens[:4] = [0, 1, max_len, 3][:min(4, n)]
    pos = 0
    for i in range(n):
        L = int(lens[i])
        segs[i]["payload_off"] = int(rng.integers(0, payload_size - L)) if payload_size > L else 0
        if slot:
            segs[i]["out_off"] = i * slot + (int(rng.integers(0, 8)) if odd else 0)
        else:
            pos += int(rng.integers(0, 9)) if odd else 0
            segs[i]["out_off"] = pos
            pos += 44 + L
        segs[i]["saddr_be"] = int(rng.integers(0, 2**32))
        segs[i]["daddr_be"] = int(rng.integers(0, 2**32))
        segs[i]["seq"] = int(rng.integers(0, 2**32))
        segs[i]["ack"] = int(rng.integers(0, 2**32))
        segs[i]["sport"] = int(rng.integers(0, 2**16))
        segs[i]["dport"] = int(rng.integers(0, 2**16))
        segs[i]["len"] = L
        segs[i]["flags"] = int(rng.integers(0, 32)) | (16 if i % 3 else 0)
    out_size = (n * slot + 64) if slot else pos + 64
    return segs, out_size


def test_oracle_tx_build_layout_and_verify():
    """The builder's packets carry the reference's header fields and verify to zero."""
    import struct
    rng = np.random.default_rng(6)
    payload = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    segs, size = make_txsegs(rng, 200, payload.size, odd=True)
    out = np.zeros(size, np.uint8)
    checks = oracle.tx_build(payload, segs, out, iphdr=True)
    offs = segs["out_off"].astype(np.uint64)
    v, st = oracle.ipv4_batch(out.copy(), offs, 65535, 1 | 2)
    assert np.all(st == 0) and np.all(v == 0)
    for s, c in zip(segs[:50], checks[:50]):
        o = int(s["out_off"])
        data = bool(s["flags"] & 16)
        L = int(s["len"]) if data else 0
        ip = out[o:o + 44 + L].tobytes()
        ver_ihl, tos, tot, ident, frag, ttl, proto = struct.unpack("!BBHHHBB", ip[:10])
        assert (ver_ihl, tos, tot, ident, frag, ttl, proto) == (0x45, 0, 44 + L, 0, 0, 255, 6)
        sport, dport, seq, ack, offf, flg, win = struct.unpack("!HHIIBBH", ip[20:36])
        assert (sport, dport, seq, ack) == (s["sport"], s["dport"], s["seq"], s["ack"])
        assert offf == 0x60 and win == 8192 and ip[40:44] == bytes([3, 3, 5, 0])
        f = int(s["flags"])
        assert flg == ((f >> 2 & 1) | (f >> 1 & 1) << 1 | (f >> 3 & 1) << 2 | int(data) << 3 | (f & 1) << 4)
        assert struct.unpack("<H", ip[36:38])[0] == c
        if data:
            po = int(s["payload_off"])
            assert ip[44:] == payload[po:po + L].tobytes()


def partial_offload_batch(seed=9, n=64):
    """Packets whose TCP check holds the un-complemented folded pseudo-header sum, as Linux leaves
    CHECKSUM_PARTIAL segments on loopback; every 3rd packet is fully checksummed."""
    import socket
    import struct
    from tests.packets import build_batch
    region, off, _ = build_batch(np.random.default_rng(seed), n)
    oracle.ipv4_batch(region, off, 32768, 0)          # FILL: valid checks everywhere
    for k, o in enumerate(off):
        if k % 3 == 0:
            continue
        o = int(o)
        tot = struct.unpack("!H", region[o + 2:o + 4].tobytes())[0]
        sa, da = struct.unpack("<II", region[o + 12:o + 20].tobytes())
        ps = oracle.pseudo(sa, da, socket.htons(tot - 20))
        partial = (~oracle.csum_continue(ps, b"", 0)) & 0xFFFF
        region[o + 36:o + 38] = np.frombuffer(struct.pack("<H", partial), np.uint8)
    return region, off


def test_oracle_flags_checksum_partial():
    region, off = partial_offload_batch()
    out, st = oracle.ipv4_batch(region, off, 32768, 1)
    for k in range(off.size):
        if k % 3 == 0:
            assert out[k] == 0 and st[k] == 0
        else:
            assert out[k] != 0 and st[k] == 4
