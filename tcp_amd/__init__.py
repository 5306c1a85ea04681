"""tcp_amd — MI355X-native (gfx950) TCP checksum engine for uNetworking/tcp's hot path.

This package is the Python front end of ``libtcpcsum.so`` (C ABI:
``include/tcpcsum.h``). The checksum itself runs only in the library's HIP
kernels; nothing here computes a checksum. If the library is missing, every
entry point raises — there is no fallback.

Reference path (``/root/reference``):
  * ``context.c:104-119`` getPseudoHeaderSum -> :func:`getPseudoHeaderSum`
  * ``context.c:121-145`` csum_continue      -> :func:`csum_continue` (scalar) and
    the batch entry points (:func:`batch_uniform`, :func:`batch_desc`,
    :func:`ipv4_batch`, :func:`ipv4_batch_ptrs`) that replace the per-packet call at ``context.c:208-209``
    with one GPU launch per batch (the ``releaseSend`` seam, ``loop.c:27-94``).
"""
from __future__ import annotations

from .api import (  # noqa: F401
    DESC_DTYPE,
    IPV4_FILL,
    IPV4_IPHDR,
    IPV4_VERIFY,
    PKT_IPHDR_BAD,
    PKT_OK,
    PKT_SKIPPED,
    TUNE_WIRE_CACHED,
    TUNE_WIN16,
    TcpCsumError,
    HostContext,
    batch_desc,
    batch_uniform,
    csum_continue,
    device_check,
    getPseudoHeaderSum,
    ipv4_batch,
    ipv4_batch_ptrs,
    lib,
    lib_path,
    pinned_empty,
    make_tuning,
    set_tuning,
    Tuning,
    stream_probe,
    synth_fill,
    synth_pseudo,
    tx_build,
    TXSEG_DTYPE,
)

__all__ = [
    "DESC_DTYPE", "IPV4_FILL", "IPV4_IPHDR", "PKT_IPHDR_BAD", "IPV4_VERIFY", "PKT_OK", "PKT_SKIPPED", "TcpCsumError",
    "HostContext", "batch_desc", "batch_uniform", "csum_continue", "device_check",
    "getPseudoHeaderSum", "ipv4_batch", "ipv4_batch_ptrs", "lib", "lib_path", "make_tuning", "pinned_empty",
    "set_tuning", "Tuning", "stream_probe",
    "synth_fill", "synth_pseudo", "tx_build", "TXSEG_DTYPE",
]
