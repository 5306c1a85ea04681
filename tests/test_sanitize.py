"""CPU: the host-side C under AddressSanitizer + UndefinedBehaviorSanitizer.

Builds tests/c/sanitize_host.c with the library's scalar drop-ins
(tcp_amd/csrc/scalar_dropin.c) and the oracle's C restatement
(oracle/csum_oracle.c) under -fsanitize=address,undefined and runs it: exact-size
heap buffers make any out-of-bounds byte an error ("ASan/UBSan on
the host C"). Host code only — GPU sanitizers are not available on this pool.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_host_c_under_asan_ubsan(tmp_path):
    exe = tmp_path / "sanitize_host"
    cmd = ["gcc", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-Wall", "-Wextra",
           "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "oracle"),
           os.path.join(REPO, "tests", "c", "sanitize_host.c"),
           os.path.join(REPO, "tcp_amd", "csrc", "scalar_dropin.c"),
           os.path.join(REPO, "oracle", "csum_oracle.c"),
           "-lpthread", "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ)
    # the environment may preload a library ahead of the ASan runtime: tolerate the link order
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1"
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize_host: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_registry_under_asan_ubsan(tmp_path):
    """The page-locking bookkeeping of tcpcsum_ipv4_batch_ptrs_host (tcp_amd/csrc/host_registry.h)
    against a modelled host: every resolved packet lies wholly in locked pages under one device
    mapping (flat and non-flat hosts), no page is locked twice, release() unlocks what was locked."""
    exe = tmp_path / "registry_test"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-Wall", "-Wextra",
           os.path.join(REPO, "tests", "c", "registry_test.cpp"), "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0"
    r = subprocess.run([str(exe), "11"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_copy_pool_under_tsan(tmp_path):
    """The host copy threads every staged host batch runs on (tcp_amd/csrc/copy_pool.h) under
    ThreadSanitizer: each piece of each job exactly once, run() returning only after all of them,
    sleeping and woken workers, the streaming-store copy at every alignment, teardown."""
    exe = tmp_path / "copy_pool_test"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-Wall", "-Wextra",
           os.path.join(REPO, "tests", "c", "copy_pool_test.cpp"), "-o", str(exe), "-lpthread"]
    b = subprocess.run(cmd, capture_output=True, text=True)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1:exitcode=66"
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stdout + r.stderr
    assert "copy_pool_test: OK" in r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_rx_drop_compaction_under_asan_ubsan(tmp_path):
    """The interposer's rx drop (tcp_amd/csrc/rx_compact.h): after the drop, the caller's own
    iovec array read by index — the reference's getIpPacket, loop.c:96-100 — holds exactly the
    passing messages in arrival order, with their lengths, flags and senders; no buffer is lost or
    doubled; a receive with a scatter-gather message is reordered by vector entries instead."""
    exe = tmp_path / "rx_compact_test"
    cmd = ["gcc", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-Wall", "-Wextra",
           os.path.join(REPO, "tests", "c", "rx_compact_test.c"), "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0"
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rx_compact_test: OK" in r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_preload_arena_under_sanitizers(tmp_path, san):
    """The interposer's packet-buffer arena (tcp_amd/csrc/preload_arena.h, TCPCSUM_PRELOAD_POOL=1):
    the loop's 2 x 1024 malloc(32 KiB) (loop.c:180-183) served in address order, the rest falling
    through; free / realloc / size-0 realloc routed back; churn from 8 threads with every holder's tag
    intact; interior and double frees abort. ASan/UBSan and ThreadSanitizer builds."""
    exe = tmp_path / "arena_test"
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}"]
    if san != "thread":
        flags.append("-fno-sanitize-recover=all")
    cmd = ["gcc"] + flags + ["-Wall", "-Wextra", os.path.join(REPO, "tests", "c", "arena_test.c"),
                             "-o", str(exe), "-lpthread"]
    b = subprocess.run(cmd, capture_output=True, text=True)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0"
    env["TSAN_OPTIONS"] = "halt_on_error=1:exitcode=66"
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "Sanitizer" not in r.stderr, r.stdout + r.stderr
    assert "OK" in r.stdout
