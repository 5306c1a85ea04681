#!/usr/bin/env python3
"""Run a Python script (argv[1:]) and, at interpreter exit, copy /proc/self/maps to
$MAPS_OUT — the address map a native crash during exit-time teardown (after Python's
atexit handlers, in the C runtime's __cxa_finalize) is resolved against.

  rocprofv3 ... -- python3 tools/maps_at_exit.py bench.py --host-path-only
"""
import atexit
import os
import runpy
import sys


def _dump():
    out = os.environ.get("MAPS_OUT", "gpurun_out/maps_at_exit.txt")
    with open("/proc/self/maps") as f, open(out, "w") as g:
        g.write(f.read())


if __name__ == "__main__":
    atexit.register(_dump)   # registered first: runs after every other atexit handler
    sys.argv = sys.argv[1:]
    runpy.run_path(sys.argv[0], run_name="__main__")
