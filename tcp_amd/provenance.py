"""Build provenance: which sources the loaded libtcpcsum.so was compiled from.

The Makefile bakes sha256(cat HASH_SRCS) into the library (tcpcsum_build_info);
``tree_hash()`` computes the same over the files next to this package, so a
caller can tell a product build of the tree it runs in from a stale or
measurement-built library.
"""
from __future__ import annotations

import hashlib
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# the Makefile's HASH_SRCS, in the same order
HASH_SRCS = (
    "include/tcpcsum.h", "tcp_amd/csrc/tcpcsum_internal.h", "tcp_amd/csrc/host_registry.h",
    "tcp_amd/csrc/copy_pool.h", "tcp_amd/csrc/tcpcsum_kernels.hip", "tcp_amd/csrc/tcpcsum_api.hip",
    "tcp_amd/csrc/tcpcsum_host.hip", "tcp_amd/csrc/scalar_dropin.c", "Makefile",
)


def tree_hash(repo: str = REPO) -> str:
    h = hashlib.sha256()
    for rel in HASH_SRCS:
        with open(os.path.join(repo, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def library_info() -> dict:
    """tcpcsum_build_info() of the loaded library, parsed."""
    from tcp_amd.api import lib
    return json.loads(lib().tcpcsum_build_info().decode())


def check_product_build(repo: str = REPO) -> dict:
    """Raise unless the loaded library is a product build of exactly these sources."""
    info = library_info()
    want = tree_hash(repo)
    if not info.get("product"):
        raise RuntimeError(f"libtcpcsum.so is a measurement build, not a product library: {info}")
    if info.get("src_sha256") != want:
        raise RuntimeError(f"libtcpcsum.so is stale: built from sources {info.get('src_sha256')}, "
                           f"the tree holds {want} — rebuild with `make`")
    return info
