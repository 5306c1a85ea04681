"""Host <-> device copies for the GPU tests, always through page-locked memory.

The library never hands pageable memory to a HIP copy: HIP's own
pin-in-place of a pageable source, in a process that also registers and
unregisters heap pages (the host paths under test do), raised
hipErrorIllegalAddress on later copies. The tests follow the same rule: every
torch copy between numpy and the device goes through a pinned tensor, so the
only pageable-memory accesses in a test are the library's own.
"""
import numpy as np
import torch


def to_dev(a: np.ndarray, dev) -> torch.Tensor:
    """numpy -> device via a pinned staging tensor (CPU memcpy, then DMA)."""
    a = np.ascontiguousarray(a)
    h = torch.empty(a.shape, dtype=torch.from_numpy(a[:0]).dtype, pin_memory=True)
    h.numpy()[...] = a
    return h.to(dev)


def host(t: torch.Tensor) -> np.ndarray:
    """device -> numpy via a pinned tensor; a copy the caller owns."""
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h.numpy().copy()


def u16(t: torch.Tensor) -> np.ndarray:
    return host(t).view(np.uint16)
