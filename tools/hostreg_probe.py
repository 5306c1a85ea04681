#!/usr/bin/env python3
"""Probe: how does hipHostRegister map malloc'd host buffers on this box?

Registers a few 32 KiB malloc'd buffers (the loop.c:180-183 layout) page by
page and prints whether the device pointer equals the host pointer, whether
registering an overlapping page range fails, and the cost of one registration.
Host logic only; no kernel runs.
"""
import ctypes
import json
import time

import torch  # noqa: F401  (loads the HIP runtime torch ships)

hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
libc = ctypes.CDLL("libc.so.6")
libc.malloc.restype = ctypes.c_void_p
libc.malloc.argtypes = [ctypes.c_size_t]
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
hip.hipSetDevice(0)

PAGE = 4096
bufs = [libc.malloc(32 * 1024) for _ in range(8)]
res = {"bufs": [hex(b) for b in bufs]}
rows = []
for flags in (0, 2):   # hipHostRegisterDefault, hipHostRegisterMapped
    b = bufs[0 if flags == 0 else 2]
    lo = b & ~(PAGE - 1)
    hi = (b + 32 * 1024 + PAGE - 1) & ~(PAGE - 1)
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(lo, hi - lo, flags)
    t1 = time.perf_counter()
    d = ctypes.c_void_p()
    rc2 = hip.hipHostGetDevicePointer(ctypes.byref(d), lo, 0)
    d2 = ctypes.c_void_p()
    rc3 = hip.hipHostGetDevicePointer(ctypes.byref(d2), b, 0)
    # overlapping registration of the last page plus the next buffer
    nb = bufs[1 if flags == 0 else 3]
    lo2 = (hi - PAGE)
    hi2 = (nb + 32 * 1024 + PAGE - 1) & ~(PAGE - 1)
    rc4 = hip.hipHostRegister(lo2, max(hi2 - lo2, PAGE), flags)
    if rc4 == 0:
        hip.hipHostUnregister(lo2)
    rows.append({"flags": flags, "register_rc": rc, "register_us": round((t1 - t0) * 1e6, 1),
                 "devptr_rc": rc2, "host": hex(lo), "dev": hex(d.value or 0), "equal": d.value == lo,
                 "interior_rc": rc3, "interior_dev": hex(d2.value or 0), "interior_equal": d2.value == b,
                 "overlap_register_rc": rc4})
    hip.hipHostUnregister(lo)
res["rows"] = rows
print(json.dumps(res))
