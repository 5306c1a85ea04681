"""Run a GPU test body in a child process, with its own HIP runtime state.

Tests that page-lock pageable host memory (tcpcsum_ctx_register_host, or
TCPCSUM_CTX_AUTO_REGISTER) run in a child: in round 3 a pageable HIP copy
(torch ``.cpu()`` of a device tensor) faulted with hipErrorIllegalAddress in
the test right after one that had registered, unregistered and freed 256 heap
buffers — the copy's fresh destination reused those heap addresses
(DESIGN.md §7). That is HIP runtime behaviour the library cannot undo; the
library never page-locks memory unless its caller asks, so the main test
process — like an application that never registers — keeps the ordinary
pageable copies the other tests make.

Usage: decorate a test with ``@isolated(lambda **kw: <run this case in a child?>)``;
the child process re-imports the test module and calls the same function with
the same parameters (``dev`` = cuda:0), and the parent asserts it exited 0.
"""
import functools
import inspect
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD_ENV = "TCPCSUM_TEST_CHILD"

_CHILD = """
import importlib, inspect, json, sys
sys.path.insert(0, {repo!r})
import torch
m = importlib.import_module({module!r})
f = getattr(m, {func!r})
kw = json.loads({kwargs!r})
if "dev" in inspect.signature(f).parameters:
    kw["dev"] = torch.device("cuda:0")
f(**kw)
torch.cuda.synchronize()
print("child ok")
"""


def isolated(pred=lambda **kw: True):
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            if os.environ.get(CHILD_ENV) == "1" or not pred(**kwargs):
                return fn(*args, **kwargs)
            params = {k: v for k, v in kwargs.items() if k != "dev"}
            code = _CHILD.format(repo=REPO, module=fn.__module__, func=fn.__name__, kwargs=json.dumps(params))
            env = dict(os.environ, **{CHILD_ENV: "1"})
            r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            assert r.returncode == 0 and "child ok" in r.stdout, (r.stdout[-3000:] + r.stderr[-3000:])
        wrapper.__signature__ = inspect.signature(fn)
        return wrapper
    return deco
