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

from . import api  # noqa: F401
from .api import *  # noqa: F401,F403  (the public names: api.__all__)
from .api import __all__  # noqa: F401
