"""numpy <-> device tensors for the GPU tests: plain torch copies.

numpy arrays are pageable, so every copy here takes HIP's own pageable path
(pin-in-place for large sources) — in the same process as the library's host
paths. Round 2's GPU tests had to stage these copies through pinned memory,
because the library then page-locked and unlocked pageable heap pages per call
and a later pageable HIP copy faulted. The library no longer
page-locks anything it was not asked to, so the tests copy the ordinary way.
"""
import numpy as np
import torch


def to_dev(a: np.ndarray, dev) -> torch.Tensor:
    """numpy -> device (pageable source)."""
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def host(t: torch.Tensor) -> np.ndarray:
    """device -> numpy (pageable destination)."""
    return t.cpu().numpy()


def u16(t: torch.Tensor) -> np.ndarray:
    return host(t).view(np.uint16)
