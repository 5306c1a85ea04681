"""ctypes bindings of include/tcpcsum.h and torch-tensor conveniences.

Device buffers are torch tensors on ``cuda`` (HIP); kernels are launched on
``torch.cuda.current_stream()`` unless a stream is given, so torch events and
synchronisation see them. torch is imported before the library is loaded so
that both use the one HIP runtime already in the process (torch ships a
``libamdhip64.so.7`` with the same SONAME the library links against).
"""
from __future__ import annotations

import atexit
import ctypes
import os
import sys
import threading
import weakref
from typing import Optional

import numpy as np

try:  # torch first: its HIP runtime must be the one the library binds to
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always present in this image
    torch = None

__all__ = [
    "DESC_DTYPE", "TXSEG_DTYPE", "IPV4_FILL", "IPV4_VERIFY", "IPV4_IPHDR", "PKT_OK", "PKT_SKIPPED",
    "PKT_IPHDR_BAD", "PKT_CSUM_PARTIAL", "CTX_BLOCKING_WAIT", "TUNE_WIRE_CACHED", "TUNE_WIN16", "TUNE_TX_NT_STORE", "TUNE_FILL_DWORD", "TUNE_FILL_U16",
    "TUNE_TX_WT_STORE", "TUNE_FILL_HALF", "TUNE_PROBE_WRITE",
    "TcpCsumError", "Tuning", "HostContext", "lib", "lib_path", "device_check", "build_info", "make_tuning", "set_tuning",
    "get_tuning", "plan_uniform", "getPseudoHeaderSum", "csum_continue", "batch_uniform", "batch_uniform_multi",
    "ubatches", "batch_desc",
    "ipv4_batch", "ipv4_batch_ptrs", "tx_build", "synth_fill", "synth_pseudo", "stream_probe", "pinned_empty",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_NAME = "libtcpcsum.so"

OK = 0
EINVAL = -1
ENODEV = -2
EHIP = -3
ENOMEM = -4
IPV4_FILL = 0
IPV4_VERIFY = 1
IPV4_IPHDR = 2
PKT_OK = 0
PKT_SKIPPED = 1
PKT_IPHDR_BAD = 2
PKT_CSUM_PARTIAL = 4
CTX_BLOCKING_WAIT = 2

# tcpcsum_desc_t {u64 offset; u32 len; u32 sum_start}
DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("sum_start", "<u4")])
# tcpcsum_txseg_t (48 bytes)
TXSEG_DTYPE = np.dtype([("payload_off", "<u8"), ("out_off", "<u8"), ("saddr_be", "<u4"), ("daddr_be", "<u4"),
                        ("seq", "<u4"), ("ack", "<u4"), ("sport", "<u2"), ("dport", "<u2"), ("len", "<u2"),
                        ("flags", "u1"), ("reserved0", "u1"), ("reserved1", "<u8")])
TXF_ACK, TXF_SYN, TXF_FIN, TXF_RST, TXF_DATA = 1, 2, 4, 8, 16

_ERRNAMES = {EINVAL: "EINVAL", ENODEV: "ENODEV", EHIP: "EHIP", ENOMEM: "ENOMEM"}


class TcpCsumError(RuntimeError):
    def __init__(self, code: int, where: str):
        self.code = code
        msg = f"{where}: {_ERRNAMES.get(code, code)}"
        try:
            msg += f" ({lib().tcpcsum_strerror(code).decode()})"
            if code == EHIP:
                msg += f" hipError={lib().tcpcsum_last_hip_error()}"
        except Exception:
            pass
        super().__init__(msg)


_lib = None
_lock = threading.Lock()

# Teardown. Contexts still open when the interpreter exits are closed by an
# atexit hook — their stream drained and copy threads joined while the HIP runtime is still up
# (torch, imported first, registered its own hooks earlier, so they run after this one). From
# then on no finalizer calls into HIP: pinned blocks still referenced are left to the OS, since
# their hipHostFree could otherwise run during interpreter shutdown, after the runtime's own
# static destructors.
_live_contexts: "weakref.WeakSet[HostContext]" = weakref.WeakSet()
_exiting = False


def _close_at_exit() -> None:
    global _exiting
    for ctx in list(_live_contexts):
        try:
            ctx.close()
        except Exception:
            pass
    _exiting = True


atexit.register(_close_at_exit)


def _finalizer_may_call_hip() -> bool:
    return not _exiting and not sys.is_finalizing()

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u16p = ctypes.POINTER(ctypes.c_uint16)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p
u32 = ctypes.c_uint32
u64 = ctypes.c_uint64


class Tuning(ctypes.Structure):
    """tcpcsum_tuning_t: a launch-shape override passed per call (None = built-in shapes)."""
    _fields_ = [("max_blocks", ctypes.c_int32), ("unroll", ctypes.c_int32), ("shape", ctypes.c_int32),
                ("flags", ctypes.c_int32)]


tunep = ctypes.POINTER(Tuning)


class UBatch(ctypes.Structure):
    """tcpcsum_ubatch_t: one batch of a multi-batch uniform launch."""
    _fields_ = [("d_base", ctypes.c_void_p), ("stride", ctypes.c_uint64), ("d_sum_start", ctypes.c_void_p),
                ("d_out", ctypes.c_void_p), ("n", ctypes.c_uint64), ("len", ctypes.c_uint32),
                ("sum_start", ctypes.c_uint32)]


MULTI_MAX = 16


class CtxStats(ctypes.Structure):
    """tcpcsum_ctx_stats_t."""
    _fields_ = [("batches", ctypes.c_uint64), ("pkts_in_place", ctypes.c_uint64), ("pkts_staged", ctypes.c_uint64),
                ("bytes_staged", ctypes.c_uint64), ("copy_threads", ctypes.c_uint64),
                ("bulk_threads", ctypes.c_uint64), ("ns_copy", ctypes.c_uint64), ("ns_wait", ctypes.c_uint64),
                ("ns_cpu_caller", ctypes.c_uint64), ("ns_cpu_workers", ctypes.c_uint64),
                ("gpu_numa_node", ctypes.c_uint64), ("staging_numa_node", ctypes.c_uint64)]

# name -> (restype, argtypes); must cover every function in include/tcpcsum.h
SIGNATURES = {
    "tcpcsum_abi_version": (ctypes.c_int, []),
    "tcpcsum_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "tcpcsum_last_hip_error": (ctypes.c_int, []),
    "tcpcsum_device_check": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "tcpcsum_build_info": (ctypes.c_char_p, []),
    "tcpcsum_pseudo": (ctypes.c_ulong, [u32, u32, ctypes.c_uint16]),
    "tcpcsum_continue": (ctypes.c_ushort, [ctypes.c_ulong, ctypes.c_char_p, ctypes.c_int]),
    "tcpcsum_batch_uniform_dev": (ctypes.c_int, [vp, u64, u32, vp, u32, vp, u64, vp, tunep]),
    "tcpcsum_batch_desc_dev": (ctypes.c_int, [vp, vp, u64, u32, vp, vp, tunep]),
    "tcpcsum_batch_uniform_multi_dev": (ctypes.c_int, [vp, u32, vp, tunep]),
    "tcpcsum_ipv4_batch_dev": (ctypes.c_int, [vp, u64, vp, u64, u32, ctypes.c_int, vp, vp, vp, tunep]),
    "tcpcsum_ipv4_batch_ptrs_dev": (ctypes.c_int, [vp, vp, u64, u32, u64, ctypes.c_int, vp, vp, vp, tunep]),
    "tcpcsum_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(vp)]),
    "tcpcsum_ctx_destroy": (None, [vp]),
    "tcpcsum_ctx_set_tuning": (ctypes.c_int, [vp, tunep]),
    "tcpcsum_ctx_set_flags": (ctypes.c_int, [vp, u32]),
    "tcpcsum_ctx_get_stats": (ctypes.c_int, [vp, vp]),
    "tcpcsum_host_alloc": (vp, [ctypes.c_size_t]),
    "tcpcsum_host_free": (None, [vp]),
    "tcpcsum_host_alloc_on": (vp, [ctypes.c_int, ctypes.c_size_t]),
    "tcpcsum_on_library_thread": (ctypes.c_int, []),
    "tcpcsum_batch_uniform_host": (ctypes.c_int, [vp, vp, u64, u32, vp, u32, vp, u64]),
    "tcpcsum_ipv4_batch_host": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp, u64, u32, ctypes.c_int, vp, vp]),
    "tcpcsum_ipv4_batch_ptrs_host": (ctypes.c_int, [vp, vp, vp, u64, ctypes.c_int, vp, vp]),
    "tcpcsum_tx_build_dev": (ctypes.c_int, [vp, vp, u64, u32, vp, ctypes.c_int, vp, vp, tunep]),
    "tcpcsum_synth_fill_dev": (ctypes.c_int, [vp, u64, u64, vp]),
    "tcpcsum_synth_pseudo_dev": (ctypes.c_int, [vp, u64, u64, u32, vp]),
    "tcpcsum_stream_probe_dev": (ctypes.c_int, [vp, u64, vp, ctypes.POINTER(ctypes.c_int), vp, tunep]),
    "tcpcsum_tuning_check": (ctypes.c_int, [tunep]),
    "tcpcsum_plan_uniform": (ctypes.c_int, [u64, u64, u32, u64, tunep, ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_int)]),
}


def lib_path() -> str:
    return os.environ.get("TCPCSUM_LIB", os.path.join(_HERE, _LIB_NAME))


def lib() -> ctypes.CDLL:
    """Load libtcpcsum.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            path = lib_path()
            if not os.path.exists(path):
                raise ImportError(
                    f"tcp_amd: {path} not found — build it with `make` (or __graft_entry__.build()); "
                    "the checksum path has no CPU fallback")
            L = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def _check(rc: int, where: str) -> None:
    if rc != OK:
        raise TcpCsumError(rc, where)


# ------------------------------------------------------------------ scalar
def getPseudoHeaderSum(saddr: int, daddr: int, tcpLength: int) -> int:
    """context.c:104-119: saddr/daddr in network order (as in struct iphdr), tcpLength = htons(len)."""
    return int(lib().tcpcsum_pseudo(saddr & 0xFFFFFFFF, daddr & 0xFFFFFFFF, tcpLength & 0xFFFF))


def csum_continue(sumStart: int, p: bytes, nbytes: Optional[int] = None) -> int:
    """context.c:121-145, synchronous scalar form (one segment, calling thread)."""
    if nbytes is None:
        nbytes = len(p)
    if nbytes > len(p):
        raise ValueError("nbytes exceeds buffer")
    return int(lib().tcpcsum_continue(sumStart & 0xFFFFFFFFFFFFFFFF, bytes(p), int(nbytes)))


def build_info() -> dict:
    """tcpcsum_build_info(): source hash, compile-time knobs, product or measurement build."""
    import json
    return json.loads(lib().tcpcsum_build_info().decode())


def device_check() -> tuple[int, str]:
    buf = ctypes.create_string_buffer(64)
    rc = lib().tcpcsum_device_check(buf, 64)
    return rc, buf.value.decode()


PROBE_SLOTS = 8192
TUNE_PIPE_ON, TUNE_PIPE_OFF, TUNE_NT_ON, TUNE_NT_OFF = 1, 2, 4, 8
TUNE_WIRE_CACHED, TUNE_WIN16 = 32, 64   # wire kernel variants (tcpcsum.h)
TUNE_TX_NT_STORE, TUNE_FILL_DWORD, TUNE_FILL_U16, TUNE_TX_WT_STORE, TUNE_FILL_HALF = 128, 256, 512, 1024, 2048
TUNE_PROBE_WRITE = 4096   # stream probe: write back every shape-th 128-B line (the wire FILL's traffic)


# The C library holds no tuning state: every device call takes an explicit
# tcpcsum_tuning_t* (NULL = built-in shapes). For the test / tool front end the
# wrappers below pass `tune=` when given, else this thread's default set with
# set_tuning() — per thread, so one thread's sweep never reshapes another's.
_tls = threading.local()


def make_tuning(max_blocks: int = 0, unroll: int = 0, shape: int = -1, flags: int = 0) -> Optional[Tuning]:
    """A validated Tuning, or None for the built-in shapes (all defaults)."""
    t = Tuning(int(max_blocks), int(unroll), int(shape), int(flags))
    _check(lib().tcpcsum_tuning_check(ctypes.byref(t)), "tcpcsum_tuning_check")
    if (t.max_blocks, t.unroll, t.shape, t.flags) == (0, 0, -1, 0):
        return None
    return t


def set_tuning(max_blocks: int = 0, unroll: int = 0, shape: int = -1, flags: int = 0) -> None:
    """This thread's default tuning for the wrappers (raises TcpCsumError on invalid values)."""
    _tls.tune = make_tuning(max_blocks, unroll, shape, flags)


def get_tuning() -> Optional[Tuning]:
    return getattr(_tls, "tune", None)


def _tune(tune):
    t = get_tuning() if tune is None else tune
    if t is None:
        return None
    if isinstance(t, tuple):
        t = make_tuning(*t)
        if t is None:
            return None
    return ctypes.byref(t)


def plan_uniform(base_addr: int, stride: int, length: int, n: int, tune=None) -> tuple[int, int, int, int]:
    """(mode, shape, unroll, max_blocks) the library picks for a uniform batch — host logic only."""
    mode, shape, unroll, mb = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(lib().tcpcsum_plan_uniform(base_addr, stride, length, n, _tune(tune), ctypes.byref(mode),
                                      ctypes.byref(shape), ctypes.byref(unroll), ctypes.byref(mb)),
           "tcpcsum_plan_uniform")
    return mode.value, shape.value, unroll.value, mb.value


# ------------------------------------------------------------------ device batches (torch tensors)
def _stream_handle(stream) -> int:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _dev_ptr(t, what: str) -> int:
    if t is None:
        return 0
    if not t.is_cuda:
        raise ValueError(f"{what} must be a device tensor")
    return t.data_ptr()


def batch_uniform(data, stride: int, length: int, n: int, sum_start=0, out=None, offset: int = 0,
                  stream=None, tune=None):
    """d_out[i] = csum_continue(start_i, data[offset+i*stride : +length], length) on the GPU.

    ``sum_start``: an int (same start for every segment) or a device int32 tensor of n entries.
    Returns ``out`` (device int16 tensor holding the u16 results)."""
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=data.device)
    if n:
        last = offset + (n - 1) * stride + length
        if last > data.numel() * data.element_size():
            raise ValueError("batch runs past the end of data")
    if isinstance(sum_start, int):
        ss_ptr, ss0 = 0, sum_start
    else:
        if sum_start.numel() < n:
            raise ValueError("sum_start too short")
        ss_ptr, ss0 = _dev_ptr(sum_start, "sum_start"), 0
    rc = lib().tcpcsum_batch_uniform_dev(_dev_ptr(data, "data") + offset, stride, length, ss_ptr, ss0,
                                         _dev_ptr(out, "out"), n, _stream_handle(stream), _tune(tune))
    _check(rc, "tcpcsum_batch_uniform_dev")
    return out


def ubatches(batches) -> ctypes.Array:
    """A host tcpcsum_ubatch_t array from (data, stride, length, n, sum_start, out[, offset]) tuples:
    ``data`` a device uint8 tensor, ``sum_start`` an int or a device int32 tensor, ``out`` a device
    int16 tensor of >= n entries."""
    arr = (UBatch * len(batches))()
    for j, b in enumerate(batches):
        data, stride, length, n, ss, out = b[:6]
        offset = b[6] if len(b) > 6 else 0
        if n and offset + (n - 1) * stride + length > data.numel() * data.element_size():
            raise ValueError(f"batch {j} runs past the end of its data")
        if out.numel() < n:
            raise ValueError(f"batch {j}: out too short")
        if isinstance(ss, int):
            ss_ptr, ss0 = 0, ss
        else:
            if ss.numel() < n:
                raise ValueError(f"batch {j}: sum_start too short")
            ss_ptr, ss0 = _dev_ptr(ss, "sum_start"), 0
        arr[j] = UBatch(_dev_ptr(data, "data") + offset, stride, ss_ptr or None, _dev_ptr(out, "out"), n, length,
                        ss0 & 0xFFFFFFFF)
    return arr


def batch_uniform_multi(batches, stream=None, tune=None) -> None:
    """Several uniform batches in one launch (tcpcsum_batch_uniform_multi_dev). ``batches``: a list of
    (data, stride, length, n, sum_start, out[, offset]) tuples or a ready ``ubatches()`` array."""
    arr = batches if isinstance(batches, ctypes.Array) else ubatches(batches)
    rc = lib().tcpcsum_batch_uniform_multi_dev(ctypes.cast(arr, ctypes.c_void_p), len(arr),
                                               _stream_handle(stream), _tune(tune))
    _check(rc, "tcpcsum_batch_uniform_multi_dev")


def batch_desc(data, desc, n: int, max_len: int, out=None, stream=None, tune=None):
    """Ragged batch; ``desc`` is a device uint8/int64 tensor holding n tcpcsum_desc_t records."""
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=data.device)
    rc = lib().tcpcsum_batch_desc_dev(_dev_ptr(data, "data"), _dev_ptr(desc, "desc"), n, max_len,
                                      _dev_ptr(out, "out"), _stream_handle(stream), _tune(tune))
    _check(rc, "tcpcsum_batch_desc_dev")
    return out


def ipv4_batch(pkts, pkt_off, n: int, cap: int, mode: int, out=None, status=None, stream=None, tune=None):
    """Wire batch over the device tensor ``pkts`` (its whole size is the region)."""
    region = pkts.numel() * pkts.element_size()
    rc = lib().tcpcsum_ipv4_batch_dev(_dev_ptr(pkts, "pkts"), region, _dev_ptr(pkt_off, "pkt_off"), n, cap, mode,
                                      _dev_ptr(out, "out"), _dev_ptr(status, "status"), _stream_handle(stream),
                                      _tune(tune))
    _check(rc, "tcpcsum_ipv4_batch_dev")
    return out, status


def ipv4_batch_ptrs(pkt_ptrs, lens, n: int, cap: int, mode: int, out=None, status=None, stream=None, tune=None,
                    bytes_hint: int = 0):
    """Scatter-gather wire batch: ``pkt_ptrs`` a device int64 tensor of packet addresses (device-accessible),
    ``lens`` a device int32 tensor of per-packet readable bytes; ``bytes_hint`` their sum if known (shape only)."""
    rc = lib().tcpcsum_ipv4_batch_ptrs_dev(_dev_ptr(pkt_ptrs, "pkt_ptrs"), _dev_ptr(lens, "lens"), n, cap,
                                           bytes_hint, mode,
                                           _dev_ptr(out, "out"), _dev_ptr(status, "status"), _stream_handle(stream),
                                           _tune(tune))
    _check(rc, "tcpcsum_ipv4_batch_ptrs_dev")
    return out, status


def tx_build(payload, segs, n: int, max_len: int, out_pkts, mode: int = 0, checks=None, stream=None, tune=None):
    """Assemble + checksum n IPv4/TCP packets on the GPU (device-side context.c:150-213).
    ``segs``: device tensor holding n TXSEG_DTYPE records (16-B aligned)."""
    rc = lib().tcpcsum_tx_build_dev(_dev_ptr(payload, "payload"), _dev_ptr(segs, "segs"), n, max_len,
                                    _dev_ptr(out_pkts, "out_pkts"), mode, _dev_ptr(checks, "checks"),
                                    _stream_handle(stream), _tune(tune))
    _check(rc, "tcpcsum_tx_build_dev")
    return checks


def synth_fill(dst, stream_off: int, nbytes: int, dst_offset: int = 0, stream=None) -> None:
    if dst_offset + nbytes > dst.numel() * dst.element_size():
        raise ValueError("synth_fill past end of dst")
    _check(lib().tcpcsum_synth_fill_dev(_dev_ptr(dst, "dst") + dst_offset, stream_off, nbytes,
                                        _stream_handle(stream)), "tcpcsum_synth_fill_dev")


def synth_pseudo(dst, seg0: int, n: int, seg_len: int, stream=None) -> None:
    if n > dst.numel():
        raise ValueError("synth_pseudo past end of dst")
    _check(lib().tcpcsum_synth_pseudo_dev(_dev_ptr(dst, "dst"), seg0, n, seg_len, _stream_handle(stream)),
           "tcpcsum_synth_pseudo_dev")


def stream_probe(src, nbytes: int, partials, stream=None, tune=None) -> int:
    """Launch the read-only probe; ``partials`` is a device int64 tensor of >= PROBE_SLOTS.
    The launch adds into the leading partials and returns how many: zeroed first, their sum is
    the lo16+hi16 word sum."""
    if partials.numel() < PROBE_SLOTS:
        raise ValueError("partials needs PROBE_SLOTS entries")
    n = ctypes.c_int()
    _check(lib().tcpcsum_stream_probe_dev(_dev_ptr(src, "src"), nbytes, _dev_ptr(partials, "partials"),
                                          ctypes.byref(n), _stream_handle(stream), _tune(tune)),
           "tcpcsum_stream_probe_dev")
    return n.value


# ------------------------------------------------------------------ host-memory batches
def _np_ptr(a: Optional[np.ndarray]) -> int:
    return 0 if a is None else a.ctypes.data


class _Pinned:
    """Owner of one tcpcsum_host_alloc block; freed when the last view dies."""

    def __init__(self, nbytes: int):
        self.ptr = lib().tcpcsum_host_alloc(nbytes)
        if not self.ptr:
            raise TcpCsumError(ENOMEM, "tcpcsum_host_alloc")
        self.nbytes = nbytes

    def __del__(self):
        try:
            if self.ptr and _finalizer_may_call_hip():
                lib().tcpcsum_host_free(self.ptr)
            self.ptr = None
        except Exception:
            pass


def pinned_empty(nbytes: int, dtype=np.uint8) -> np.ndarray:
    """A numpy array in page-locked host memory (tcpcsum_host_alloc). Host-path
    calls on such memory run zero-copy: the kernel reads it over PCIe."""
    owner = _Pinned(max(int(nbytes), 1))
    raw = (ctypes.c_uint8 * owner.nbytes).from_address(owner.ptr)
    raw._owner = owner
    return np.frombuffer(raw, np.uint8)[:nbytes].view(dtype)


class HostContext:
    """tcpcsum_ctx_t: host-memory batches, synchronous, on one stream. Memory its owner page-locked
    (pinned_empty / tcpcsum_host_alloc) is read in place (a uniform batch of 32 MiB or more: DMA'd to
    HBM from those pages in 256 MiB pieces); pageable memory is copied into the context's pinned
    staging and never page-locked. ``blocking_wait`` (TCPCSUM_CTX_BLOCKING_WAIT): sleep, not spin, while the
    device works."""

    def __init__(self, device: int = 0, scratch_bytes: int = 0, blocking_wait: bool = False):
        h = vp()
        self._h = vp()
        _check(lib().tcpcsum_ctx_create(device, scratch_bytes, ctypes.byref(h)), "tcpcsum_ctx_create")
        self._h = h
        _live_contexts.add(self)
        if blocking_wait:
            self.set_flags(CTX_BLOCKING_WAIT)

    def set_flags(self, flags: int) -> None:
        _check(lib().tcpcsum_ctx_set_flags(self._h, flags), "tcpcsum_ctx_set_flags")

    def stats(self) -> dict:
        st = CtxStats()
        _check(lib().tcpcsum_ctx_get_stats(self._h, ctypes.byref(st)), "tcpcsum_ctx_get_stats")
        d = {k: int(getattr(st, k)) for k, _ in CtxStats._fields_}
        for k in ("gpu_numa_node", "staging_numa_node"):   # UINT64_MAX: unknown
            if d[k] == 2**64 - 1:
                d[k] = None
        return d

    def close(self) -> None:
        if self._h:
            lib().tcpcsum_ctx_destroy(self._h)
            self._h = vp()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            if _finalizer_may_call_hip():
                self.close()
        except Exception:
            pass

    def set_tuning(self, max_blocks: int = 0, unroll: int = 0, shape: int = -1, flags: int = 0) -> None:
        """Launch shapes of this context's batches only (tcpcsum_ctx_set_tuning)."""
        t = make_tuning(max_blocks, unroll, shape, flags)
        _check(lib().tcpcsum_ctx_set_tuning(self._h, None if t is None else ctypes.byref(t)),
               "tcpcsum_ctx_set_tuning")

    def batch_uniform(self, data: np.ndarray, stride: int, length: int, n: int, sum_start=0,
                      offset: int = 0) -> np.ndarray:
        data = np.ascontiguousarray(data).view(np.uint8)
        if n and offset + (n - 1) * stride + length > data.nbytes:
            raise ValueError("batch runs past the end of data")
        out = np.empty(n, np.uint16)
        if isinstance(sum_start, (int, np.integer)):
            ss, ss0 = None, int(sum_start)
        else:
            ss, ss0 = np.ascontiguousarray(sum_start, np.uint32), 0
        rc = lib().tcpcsum_batch_uniform_host(self._h, data.ctypes.data + offset, stride, length, _np_ptr(ss), ss0,
                                              out.ctypes.data, n)
        _check(rc, "tcpcsum_batch_uniform_host")
        return out

    def ipv4_batch(self, region: np.ndarray, pkt_off: np.ndarray, cap: int, mode: int):
        """region: writable uint8 array holding the packets (FILL patches it in place)."""
        assert region.dtype == np.uint8 and region.flags.c_contiguous and region.flags.writeable
        off = np.ascontiguousarray(pkt_off, np.uint64)
        n = off.size
        out = np.empty(n, np.uint16)
        status = np.empty(n, np.uint8)
        rc = lib().tcpcsum_ipv4_batch_host(self._h, region.ctypes.data, region.nbytes, off.ctypes.data, n, cap,
                                           mode, out.ctypes.data, status.ctypes.data)
        _check(rc, "tcpcsum_ipv4_batch_host")
        return out, status

    def ipv4_batch_ptrs(self, ptrs, lens, mode: int):
        """Scatter-gather wire batch over host buffers: ``ptrs`` host addresses (ints), ``lens`` readable
        bytes per packet. Page-locked buffers are used in place; pageable ones are copied into staging.
        FILL patches the checks in place."""
        p = np.ascontiguousarray(np.asarray(ptrs, dtype=np.uint64))
        ln = np.ascontiguousarray(np.asarray(lens, dtype=np.uint32))
        if p.size != ln.size:
            raise ValueError("ptrs and lens differ in length")
        n = p.size
        out = np.empty(n, np.uint16)
        status = np.empty(n, np.uint8)
        rc = lib().tcpcsum_ipv4_batch_ptrs_host(self._h, p.ctypes.data, ln.ctypes.data, n, mode, out.ctypes.data,
                                                status.ctypes.data)
        _check(rc, "tcpcsum_ipv4_batch_ptrs_host")
        return out, status
