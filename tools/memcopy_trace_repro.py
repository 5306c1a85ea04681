#!/usr/bin/env python3
"""Round 4's exit-time SIGSEGV without this library: torch alone, pinned host-to-device copies
(what the host leg's DMA does), under rocprofv3 --memory-copy-trace. Exits 0 when nothing
crashes at teardown.

  rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o t -- python3 tools/memcopy_trace_repro.py
"""
import torch

x = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
y = torch.empty_like(x, device="cuda")
for _ in range(20):
    y.copy_(x, non_blocking=True)
torch.cuda.synchronize()
z = torch.empty(1 << 20, dtype=torch.uint8)
z.copy_(y[:1 << 20])
print("copies done", int(z.sum()))
