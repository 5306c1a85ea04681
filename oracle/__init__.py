"""oracle — TEST INFRASTRUCTURE ONLY.

ctypes front end of the C restatement in ``oracle/csum_oracle.c``
(``/root/reference/context.c:104-145`` and the IPv4/TCP framing of
``context.c:169-209``). Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg import this package, and only to check or
time the reference algorithm on the CPU; the product (``tcp_amd``) never
touches it.

Parity pin: SURVEY.md Appendix A KATs and Appendix B digests, both produced by
the reference's own code (see ``tests/golden/``). Building the reference itself
here was refused by the environment ("Oracle and parity pin").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
_libs: dict = {}

vp = ctypes.c_void_p
u64 = ctypes.c_uint64
u32 = ctypes.c_uint32

_SIGS = {
    "oracle_pseudo": (ctypes.c_ulong, [u32, u32, ctypes.c_uint16]),
    "oracle_csum_continue": (ctypes.c_ushort, [ctypes.c_ulong, ctypes.c_char_p, ctypes.c_int]),
    "oracle_mix64": (u64, [u64]),
    "oracle_gen_stream": (None, [vp, u64, u64]),
    "oracle_saddr": (u32, [u64]),
    "oracle_daddr": (u32, [u64]),
    "oracle_synth_batch": (ctypes.c_int, [u64, u64, u32, vp, ctypes.c_int]),
    "oracle_batch_desc": (None, [vp, vp, vp, vp, u64, vp]),
    "oracle_ipv4_batch": (None, [vp, vp, u64, u32, ctypes.c_int, vp, vp]),
    "oracle_tx_build": (None, [vp, vp, u64, vp, ctypes.c_int, vp]),
    "oracle_digest": (None, [vp, u64, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_uint16)]),
    "oracle_cpu_bench": (ctypes.c_double, [ctypes.c_int, u32, u64, ctypes.c_double, ctypes.POINTER(u64),
                                           ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double)]),
}


def lib(opt: str = "O2") -> ctypes.CDLL:
    """Load oracle/build/liboracle{,_O0}.so, building it with gcc if absent."""
    if opt in _libs:
        return _libs[opt]
    name = "liboracle.so" if opt == "O2" else f"liboracle_{opt}.so"
    path = os.path.join(_HERE, "build", name)
    if not os.path.exists(path):
        subprocess.run(["make", "-C", _REPO, f"oracle/build/{name}"], check=True, capture_output=True)
    L = ctypes.CDLL(path)
    for fn, (res, args) in _SIGS.items():
        f = getattr(L, fn)
        f.restype = res
        f.argtypes = args
    _libs[opt] = L
    return L


def pseudo(saddr: int, daddr: int, len_be: int) -> int:
    return int(lib().oracle_pseudo(saddr, daddr, len_be))


def csum_continue(sum_start: int, p: bytes, nbytes: int | None = None) -> int:
    if nbytes is None:
        nbytes = len(p)
    return int(lib().oracle_csum_continue(sum_start & 0xFFFFFFFFFFFFFFFF, bytes(p), nbytes))


def gen_stream(off: int, nbytes: int) -> np.ndarray:
    a = np.empty(nbytes, np.uint8)
    lib().oracle_gen_stream(a.ctypes.data, off, nbytes)
    return a


def saddr(i: int) -> int:
    return int(lib().oracle_saddr(i))


def daddr(i: int) -> int:
    return int(lib().oracle_daddr(i))


def synth_batch(seg0: int, n: int, seg_len: int, threads: int = 8) -> np.ndarray:
    out = np.empty(n, np.uint16)
    if lib().oracle_synth_batch(seg0, n, seg_len, out.ctypes.data, threads) != 0:
        raise MemoryError("oracle_synth_batch")
    return out


def batch_desc(base: np.ndarray, off, lens, sum_start) -> np.ndarray:
    off = np.ascontiguousarray(off, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    ss = np.ascontiguousarray(sum_start, np.uint32)
    base = np.ascontiguousarray(base, np.uint8)
    out = np.empty(off.size, np.uint16)
    lib().oracle_batch_desc(base.ctypes.data, off.ctypes.data, lens.ctypes.data, ss.ctypes.data, off.size,
                            out.ctypes.data)
    return out


def batch_uniform(base: np.ndarray, stride: int, length: int, n: int, sum_start, offset: int = 0) -> np.ndarray:
    off = offset + np.arange(n, dtype=np.uint64) * np.uint64(stride)
    lens = np.full(n, length, np.uint32)
    if isinstance(sum_start, (int, np.integer)):
        sum_start = np.full(n, int(sum_start), np.uint32)
    return batch_desc(base, off, lens, sum_start)


def ipv4_batch(region: np.ndarray, off, cap: int, mode: int):
    """Mutates region in FILL mode, like the device path. Returns (out, status)."""
    off = np.ascontiguousarray(off, np.uint64)
    out = np.empty(off.size, np.uint16)
    st = np.empty(off.size, np.uint8)
    lib().oracle_ipv4_batch(region.ctypes.data, off.ctypes.data, off.size, cap, mode, out.ctypes.data,
                            st.ctypes.data)
    return out, st


def digest(out: np.ndarray) -> tuple[str, int, str]:
    """(fnv1a64 hex, sum, xor hex) as in SURVEY.md Appendix B."""
    out = np.ascontiguousarray(out, np.uint16)
    f, s, x = u64(), u64(), ctypes.c_uint16()
    lib().oracle_digest(out.ctypes.data, out.size, ctypes.byref(f), ctypes.byref(s), ctypes.byref(x))
    return f"{f.value:016x}", int(s.value), f"{x.value:04x}"


def cpu_bench(threads: int, seg_len: int, nseg: int, min_seconds: float, opt: str = "O2") -> dict:
    """Time the restatement over a host-resident synthetic batch (>= 5 passes and min_seconds):
    best and median pass in GiB/s, mean over all passes, the outputs' digest and the pass count."""
    d = u64()
    p = ctypes.c_int()
    tot = ctypes.c_double()
    med = ctypes.c_double()
    best = lib(opt).oracle_cpu_bench(threads, seg_len, nseg, min_seconds, ctypes.byref(d), ctypes.byref(p),
                                     ctypes.byref(tot), ctypes.byref(med))
    mean = nseg * seg_len * p.value / tot.value / 2**30 if tot.value > 0 else 0.0
    return {"best": float(best), "median": float(med.value), "mean": float(mean), "digest": f"{d.value:016x}",
            "passes": int(p.value)}


def tx_build(payload: np.ndarray, segs: np.ndarray, out: np.ndarray, iphdr: bool = False) -> np.ndarray:
    """context.c:150-213 for every record of segs (TXSEG layout); mutates out, returns the TCP checks."""
    payload = np.ascontiguousarray(payload, np.uint8)
    segs = np.ascontiguousarray(segs)
    assert segs.dtype.itemsize == 48 and out.dtype == np.uint8 and out.flags.c_contiguous
    checks = np.empty(segs.size, np.uint16)
    lib().oracle_tx_build(payload.ctypes.data, segs.ctypes.data, segs.size, out.ctypes.data, int(iphdr),
                          checks.ctypes.data)
    return checks
