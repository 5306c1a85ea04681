"""The zero-edit seam: libtcpcsum_preload.so interposing sendmmsg / recvmmsg.

tests/c/mmsg_loop builds packets with the reference's framing in separate
32 KiB buffers and pushes them through sendmmsg/recvmmsg over UDP loopback
(no root needed). With TCPCSUM_PRELOAD_TX=fill every received packet must equal
the oracle's FILL of the packet as built (check computed per context.c:208).
"""
import errno
import json
import os
import re
import socket
import struct
import subprocess
import sys

import numpy as np
import pytest

import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "tests", "c", "mmsg_loop")
EXE_WRAP = os.path.join(REPO, "tests", "c", "mmsg_loop_wrap")   # the seam linked in (-Wl,--wrap=...)
EXE_WRAP_NOPOOL = os.path.join(REPO, "tests", "c", "mmsg_loop_wrap_nopool")   # --wrap=sendmmsg,recvmmsg only
PRELOAD = os.path.join(REPO, "tcp_amd", "libtcpcsum_preload.so")


def _ensure_built():
    if not all(os.path.exists(p) for p in (EXE, PRELOAD, EXE_WRAP, EXE_WRAP_NOPOOL)):
        subprocess.run(["make", "-C", REPO, "tests/c/mmsg_loop", "tests/c/mmsg_loop_wrap",
                        "tests/c/mmsg_loop_wrap_nopool", "tcp_amd/libtcpcsum_preload.so"], check=True)


def run_loop(tmp_path, n, env_extra, cpu_checks=False, corrupt=False, trunc=False, forge=False, pinned=False,
             iov2=False, wrap=False, fork=False, threads=False, exe=None):
    """Run mmsg_loop under the LD_PRELOAD interposer, or (wrap) its build with the seam linked in."""
    _ensure_built()
    out = tmp_path / "mm.bin"
    env = {k: v for k, v in os.environ.items() if not k.startswith("TCPCSUM_PRELOAD") and k != "LD_PRELOAD"}
    env.update({"TCPCSUM_PRELOAD_ANY_SOCKET": "1", "TCPCSUM_PRELOAD_STATS": "1"})
    if not wrap:
        env["LD_PRELOAD"] = PRELOAD
    env.update(env_extra)
    mode = ("trunc" if trunc else "corrupt" if corrupt else "forge" if forge else
            "cpu-checks" if cpu_checks else "plain")
    args = [exe or (EXE_WRAP if wrap else EXE), str(n), str(out), mode] + (
        ["pinned"] if pinned else ["iov2"] if iov2 else ["fork"] if fork else ["threads"] if threads else [])
    r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=120)
    pkts = []
    if r.returncode == 0:
        data = out.read_bytes()
        pos = 0
        while pos < len(data):
            (lo,) = struct.unpack_from("<I", data, pos)
            built = data[pos + 4:pos + 4 + lo]
            pos += 4 + lo
            (li,) = struct.unpack_from("<I", data, pos)
            got = data[pos + 4:pos + 4 + li]
            pos += 4 + li
            pkts.append((built, got))
    stats = {}
    m = re.search(r"tcpcsum_preload: (tx batches=.*)", r.stderr)
    if m:
        for side, body in zip(("tx", "rx", "all", "ctx", "pool"), m.group(1).split("|")[:5]):
            for k, v in re.findall(r"(\w+)=(\d+)", body):
                stats[f"{side}_{k}"] = int(v)
    return r, pkts, stats


def route_localnet_any() -> bool:
    """Whether any interface but lo has net.ipv4.conf.<if>.route_localnet = 1 (as the interposer
    reads it): 127/8 may then arrive on other interfaces."""
    base = "/proc/sys/net/ipv4/conf"
    try:
        names = os.listdir(base)
    except OSError:
        return False
    for name in names:
        if name == "lo":
            continue
        try:
            if int(open(os.path.join(base, name, "route_localnet")).read().strip() or 0):
                return True
        except (OSError, ValueError):
            pass
    return False


def oracle_fill(pkt: bytes, mode=0) -> bytes:
    region = np.frombuffer(pkt + b"\0" * 16, np.uint8).copy()
    oracle.ipv4_batch(region, np.array([0], np.uint64), 65535, mode)
    return region[:len(pkt)].tobytes()


def test_passthrough_when_off(tmp_path):
    r, pkts, stats = run_loop(tmp_path, 150, {"TCPCSUM_PRELOAD_TX": "off"})
    assert r.returncode == 0, r.stderr
    assert len(pkts) == 150 and all(b == g for b, g in pkts)
    assert stats["tx_packets"] == 0


def test_pool_request_without_gpu_falls_back_to_libc(tmp_path):
    """TCPCSUM_PRELOAD_POOL=1 where no page-locked memory can be had: the constructor says so, every
    malloc goes to libc (the loop still runs, free() of its buffers included), nothing is served."""
    import tcp_amd
    if tcp_amd.device_check()[0] == 0:
        pytest.skip("a GPU is present")
    r, pkts, stats = run_loop(tmp_path, 1500, {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_POOL": "1"})
    assert r.returncode == 0, r.stderr
    assert "TCPCSUM_PRELOAD_POOL: no page-locked pool" in r.stderr
    assert len(pkts) == 1500 and all(b == g for b, g in pkts)
    assert stats["pool_on"] == 0 and stats["pool_served"] == 0


@pytest.mark.parametrize("name,tried", [("mmsg_loop", True), ("stress", False), ("0", False)])
def test_pool_only_for_the_named_program(tmp_path, name, tried):
    """TCPCSUM_PRELOAD_POOL=<executable name>: only that program takes the pool (and starts HIP for it);
    a wrapper or any other program the preload reaches leaves it alone. Here without a GPU, so the
    named program's attempt fails loudly and falls back; the others never try."""
    import tcp_amd
    if tcp_amd.device_check()[0] == 0:
        pytest.skip("a GPU is present")
    r, pkts, stats = run_loop(tmp_path, 300, {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_POOL": name})
    assert r.returncode == 0, r.stderr
    assert ("TCPCSUM_PRELOAD_POOL: no page-locked pool" in r.stderr) == tried
    assert stats["pool_on"] == 0 and len(pkts) == 300


def test_wrap_seam_passthrough_and_refusal(tmp_path):
    """The link-time form (-Wl,--wrap=sendmmsg,recvmmsg,malloc,calloc,free,realloc against
    tcp_amd/libtcpcsum_wrap.a): with TX off every packet goes through untouched; without a GPU,
    FILL refuses loudly (ENXIO) exactly as the preload does."""
    import tcp_amd
    r, pkts, stats = run_loop(tmp_path, 150, {"TCPCSUM_PRELOAD_TX": "off"}, wrap=True)
    assert r.returncode == 0, r.stderr
    assert len(pkts) == 150 and all(b == g for b, g in pkts) and stats["tx_packets"] == 0
    if tcp_amd.device_check()[0] != 0:
        r, _, _ = run_loop(tmp_path, 10, {"TCPCSUM_PRELOAD_TX": "fill"}, wrap=True)
        assert r.returncode == 3 and "No such device or address" in r.stderr


def test_wrap_mmsg_wraps_alone_link_and_run(tmp_path):
    """the archive's seams link with only -Wl,--wrap=sendmmsg,--wrap=recvmmsg (the allocation
    member, which needs __real_malloc & co, stays out of the link): the loop runs, TX off passes every
    packet through, and without a GPU FILL refuses loudly."""
    import tcp_amd
    r, pkts, stats = run_loop(tmp_path, 150, {"TCPCSUM_PRELOAD_TX": "off"}, wrap=True, exe=EXE_WRAP_NOPOOL)
    assert r.returncode == 0, r.stderr
    assert len(pkts) == 150 and all(b == g for b, g in pkts) and stats["tx_packets"] == 0
    nm = subprocess.run(["nm", EXE_WRAP_NOPOOL], capture_output=True, text=True).stdout
    assert "__wrap_sendmmsg" in nm and "__wrap_malloc" not in nm
    if tcp_amd.device_check()[0] != 0:
        r, _, _ = run_loop(tmp_path, 10, {"TCPCSUM_PRELOAD_TX": "fill"}, wrap=True, exe=EXE_WRAP_NOPOOL)
        assert r.returncode == 3 and "No such device or address" in r.stderr


@pytest.mark.parametrize("call", ["os.execv('/bin/echo', ['echo', 'EXECED'])",
                                  "os.execve('/bin/echo', ['echo', 'EXECED'], dict(os.environ))",
                                  "os.execvp('echo', ['echo', 'EXECED'])"])
def test_exec_refused_once_the_pool_started_hip(tmp_path, call):
    """with TCPCSUM_PRELOAD_POOL=1 the constructor starts HIP in whatever process loads the
    interposer, and a process that has must not exec. Every exec entry point then fails with EPERM
    (here in Python, which calls execv / execve from libc); without the pool the same exec runs. A
    forked child may still exec (subprocess from the same process works). CPU only: on a GPU box the
    refused call would be an exec after HIP started if the guard failed."""
    import tcp_amd
    if tcp_amd.device_check()[0] == 0 or os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is present: never exec after HIP started, guarded or not")
    _ensure_built()
    prog = ("import os, subprocess, sys\n"
            "print(subprocess.run(['/bin/echo', 'CHILD'], capture_output=True, text=True).stdout.strip(), flush=True)\n"
            "try:\n"
            f"    {call}\n"
            "except PermissionError as e:\n"
            "    print('REFUSED', e.errno)\n")
    env = {k: v for k, v in os.environ.items() if not k.startswith("TCPCSUM_PRELOAD") and k != "LD_PRELOAD"}
    env["LD_PRELOAD"] = PRELOAD
    on = subprocess.run([sys.executable, "-c", prog], env=dict(env, TCPCSUM_PRELOAD_POOL="1"),
                        capture_output=True, text=True, timeout=120)
    assert on.stdout.split() == ["CHILD", "REFUSED", str(errno.EPERM)], (on.stdout, on.stderr)
    assert "refused: this process started HIP" in on.stderr
    off = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True, timeout=120)
    assert off.stdout.split() == ["CHILD", "EXECED"], (off.stdout, off.stderr)


def fork_child_line(r):
    m = re.search(r"fork child parent_owned=(-?\d+) child_owned=(-?\d+) send=(-?\d+) errno=(\d+)", r.stdout)
    assert m, (r.stdout, r.stderr)
    return tuple(int(x) for x in m.groups())


@pytest.mark.parametrize("wrap", [False, True])
def test_fork_child_of_a_process_without_hip(tmp_path, wrap):
    """A forked child of a loop whose interposer never started HIP (TX off, no pool): its mallocs are
    libc's, freeing a parent's buffer is fine, and its sendmmsg goes straight through."""
    r, pkts, stats = run_loop(tmp_path, 200, {"TCPCSUM_PRELOAD_TX": "off"}, wrap=wrap, fork=True)
    assert r.returncode == 0, r.stderr
    assert len(pkts) == 200 and all(b == g for b, g in pkts)
    assert fork_child_line(r) == (0, 0, 1, 0)


def test_fails_loudly_without_gpu(tmp_path):
    import tcp_amd
    if tcp_amd.device_check()[0] == 0:
        pytest.skip("a GPU is present")
    r, _, stats = run_loop(tmp_path, 10, {"TCPCSUM_PRELOAD_TX": "fill"})
    assert r.returncode == 3 and "No such device or address" in r.stderr
    assert "refusing" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
def test_tx_fill_on_gpu(tmp_path, pinned):
    """Separately malloc'd 32 KiB out-buffers (loop.c:180-183): copied into pinned staging and the checks
    stored back. pinned: the same pool carved from tcpcsum_host_alloc (INTEGRATION.md level 2): the
    interposer fills the caller's buffers in place, no copy, nothing registered."""
    r, pkts, stats = run_loop(tmp_path, 3000, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_RX": "verify"},
                              pinned=pinned)
    assert r.returncode == 0, r.stderr
    assert len(pkts) == 3000
    for built, got in pkts:
        assert got == oracle_fill(built)
    assert stats["tx_filled"] == 3000 and stats["rx_verified"] == 3000 and stats["rx_verify_failed"] == 0
    assert stats["rx_partial"] == 0
    # tx packets in the pinned pool go in place; rx scratch buffers (and malloc'd tx buffers) are staged
    assert (stats["ctx_in_place"] == 3000) == pinned
    assert stats["ctx_staged"] == (3000 if pinned else 6000)


@pytest.mark.gpu
def test_pool_zero_copy_loop_unedited(tmp_path):
    """TCPCSUM_PRELOAD_POOL=1 with mmsg_loop's plain mallocs (loop.c:180-183 unedited):
    the interposer serves the loop's 2 x 1024 32-KiB buffers from its own page-locked arena, so every
    tx packet is filled and every rx packet verified in place — nothing staged — and each received
    packet is the oracle's FILL of what was built."""
    n = 3000
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_RX": "verify",
                                            "TCPCSUM_PRELOAD_POOL": "mmsg_loop"})
    assert r.returncode == 0, r.stderr
    assert len(pkts) == n
    for built, got in pkts:
        assert got == oracle_fill(built)
    assert stats["pool_on"] == 1 and stats["pool_served"] == 2048 and stats["pool_full"] == 0
    assert stats["pool_released"] == 2048                      # the loop's free()s came back to the arena
    assert stats["tx_filled"] == n and stats["rx_verified"] == n and stats["rx_verify_failed"] == 0
    assert stats["ctx_in_place"] == 2 * n and stats["ctx_staged"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("pool", ["0", "mmsg_loop_wrap"])
def test_wrap_seam_on_gpu(tmp_path, pool):
    """The seam linked in at build time (-Wl,--wrap=..., tcp_amd/libtcpcsum_wrap.a), no LD_PRELOAD:
    every packet filled on the GPU equals the oracle's FILL and verifies on receive. With the pool, the
    wrapped mallocs of the loop's 2 x 1024 buffers come from the arena and both seams run in place —
    while the HIP runtime's own allocations never pass through the wrap at all."""
    n = 2500
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_RX": "verify",
                                            "TCPCSUM_PRELOAD_POOL": pool}, wrap=True)
    assert r.returncode == 0, r.stderr
    assert len(pkts) == n and all(got == oracle_fill(built) for built, got in pkts)
    assert stats["tx_filled"] == n and stats["rx_verified"] == n and stats["rx_verify_failed"] == 0
    if pool != "0":
        assert stats["pool_served"] == 2048 and stats["ctx_in_place"] == 2 * n and stats["ctx_staged"] == 0
    else:
        assert stats["pool_on"] == 0 and stats["ctx_staged"] == 2 * n


@pytest.mark.gpu
@pytest.mark.parametrize("wrap", [False, True])
def test_pool_fork_child(tmp_path, wrap):
    """fork() in a loop whose interposer holds the pool and a GPU context: the child's malloc(32 KiB)
    comes from libc (the arena is closed in the child), it may free a parent's arena buffer, and its
    sendmmsg fails with ENXIO (HIP does not survive fork) instead of sending an unchecked packet. The
    parent runs on unharmed and prints its counters once."""
    n = 1200
    pool = "mmsg_loop_wrap" if wrap else "mmsg_loop"
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_POOL": pool},
                              wrap=wrap, fork=True)
    assert r.returncode == 0, r.stderr
    assert len(pkts) == n and all(got == oracle_fill(built) for built, got in pkts)
    assert fork_child_line(r) == (1, 0, -1, errno.ENXIO)
    assert "forked child of a process that started HIP" in r.stderr
    assert r.stderr.count("tcpcsum_preload: tx batches=") == 1
    assert stats["pool_served"] == 2048 and stats["pool_released"] == 2048 and stats["ctx_staged"] == 0


@pytest.mark.gpu
def test_pool_guards_runtime_threads(tmp_path):
    """under the pool a thread of the loop's own gets a block of the loop's size from the
    arena, a HIP host callback (the GPU runtime's thread) never does, and the loop's 2 x 1024 buffers
    are then all served and every batch runs in place (the library's copy threads are marked too:
    tcpcsum_on_library_thread, tests/c/copy_pool_test.cpp)."""
    n = 2100
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_RX": "verify",
                                            "TCPCSUM_PRELOAD_POOL": "mmsg_loop"}, threads=True)
    assert r.returncode == 0, r.stderr
    m = re.search(r"threads app_owned=(\d) cb_owned=(\d) cb_guarded=(-?\d)", r.stdout)
    assert m and m.groups() == ("1", "0", "1"), (r.stdout, r.stderr)
    assert len(pkts) == n and all(got == oracle_fill(built) for built, got in pkts)
    assert stats["pool_served"] == 2049 and stats["pool_released"] == 2049 and stats["pool_full"] == 0
    assert stats["ctx_in_place"] == 2 * n and stats["ctx_staged"] == 0


@pytest.mark.gpu
def test_pool_on_the_named_device(tmp_path):
    """the pool's block is allocated for TCPCSUM_PRELOAD_DEVICE's GPU (tcpcsum_host_alloc_on),
    the device the seams then use; a device that does not exist gets no pool (said once) and its
    seams refuse (ENXIO), never a block placed for another GPU."""
    n = 1500
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_POOL": "mmsg_loop",
                                            "TCPCSUM_PRELOAD_DEVICE": "0"})
    assert r.returncode == 0, r.stderr
    assert len(pkts) == n and all(got == oracle_fill(built) for built, got in pkts)
    assert stats["pool_served"] == 2048 and stats["ctx_staged"] == 0 and stats["pool_device"] == 0
    r, _, stats = run_loop(tmp_path, 10, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_POOL": "mmsg_loop",
                                          "TCPCSUM_PRELOAD_DEVICE": "64"})
    assert "no page-locked pool on device 64" in r.stderr
    assert r.returncode == 3 and "No such device or address" in r.stderr


@pytest.mark.gpu
def test_pool_rx_drop_in_place(tmp_path):
    """rx drop on the arena's in-buffers: the corrupted segments (every 7th) never reach the caller,
    the rest arrive byte-identical; verified in place, nothing staged."""
    n = 2100
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_RX": "drop",
                                            "TCPCSUM_PRELOAD_POOL": "1"}, corrupt=True)
    assert r.returncode == 0, r.stderr
    bad = 0
    for i, (built, got) in enumerate(pkts):
        if i % 7 == 3:
            assert got == b""
            bad += 1
        else:
            assert got == built
    assert stats["rx_verify_failed"] == bad and stats["rx_dropped"] == bad
    assert stats["ctx_in_place"] == n and stats["ctx_staged"] == 0


@pytest.mark.gpu
def test_rx_drop_multi_iov_messages(tmp_path):
    """a message received into two iovecs (800 bytes, then the rest) is verified from its
    first iovec when that holds the whole packet — corrupted ones are dropped — and otherwise passed
    through unverified (a scatter read), counted as skipped, never silently dropped."""
    n = 1400
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_RX": "drop"},
                              corrupt=True, iov2=True)
    assert r.returncode == 0, r.stderr
    dropped = whole = 0
    for i, (built, got) in enumerate(pkts):
        fits = len(built) <= 800
        whole += fits
        if i % 7 == 3 and fits:
            assert got == b""
            dropped += 1
        else:
            assert got == built
    assert 0 < whole < n
    assert stats["rx_dropped"] == dropped and stats["rx_verify_failed"] == dropped
    assert stats["rx_skipped"] == n - whole and stats["rx_verified"] == whole


@pytest.mark.gpu
def test_preload_device_choice(tmp_path):
    """TCPCSUM_PRELOAD_DEVICE (one loop process per GPU): device 0 named explicitly
    fills every packet; a device this box does not have makes the interposer refuse loudly (ENXIO,
    naming the device) instead of falling back to another GPU or to unchecked packets."""
    import torch
    r, pkts, stats = run_loop(tmp_path, 400, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_DEVICE": "0"})
    assert r.returncode == 0, r.stderr
    assert all(got == oracle_fill(built) for built, got in pkts)
    assert stats["pool_device"] == 0 and stats["tx_filled"] == 400
    missing = torch.cuda.device_count()
    r, _, stats = run_loop(tmp_path, 10, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_DEVICE": str(missing)})
    assert r.returncode == 3 and "No such device or address" in r.stderr
    assert f"unavailable on device {missing}" in r.stderr


@pytest.mark.gpu
def test_tx_verify_live_parity_with_cpu_checks(tmp_path):
    """Checks written by the reference's CPU path (tcpcsum_continue == csum_continue) verify on the GPU."""
    r, pkts, stats = run_loop(tmp_path, 2000, {"TCPCSUM_PRELOAD_TX": "verify"}, cpu_checks=True)
    assert r.returncode == 0, r.stderr
    assert stats["tx_verified"] == 2000 and stats["tx_verify_failed"] == 0
    assert all(b == g for b, g in pkts)            # verify mode never edits packets
    # and without checks every packet fails verification
    r, _, stats = run_loop(tmp_path, 500, {"TCPCSUM_PRELOAD_TX": "verify"})
    assert stats["tx_verify_failed"] == 500


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
def test_tx_fill_with_ip_header(tmp_path, pinned):
    r, pkts, stats = run_loop(tmp_path, 700, {"TCPCSUM_PRELOAD_TX": "fill", "TCPCSUM_PRELOAD_IPHDR": "1",
                                              "TCPCSUM_PRELOAD_RX": "verify"}, pinned=pinned)
    assert r.returncode == 0, r.stderr
    for built, got in pkts:
        assert got == oracle_fill(built, 2)
    assert stats["rx_verify_failed"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
def test_rx_drop_on_gpu(tmp_path, pinned):
    """TCPCSUM_PRELOAD_RX=drop: segments whose checksum does not verify (one TCP header byte of every
    7th packet flipped after the CPU computed its check) never reach the caller; every other segment
    arrives byte-identical, and which ones were dropped is exactly what the oracle's VERIFY says."""
    n = 2100
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_RX": "drop"},
                              corrupt=True, pinned=pinned)
    assert r.returncode == 0, r.stderr
    assert len(pkts) == n
    bad = 0
    for built, got in pkts:
        region = np.frombuffer(built + b"\0" * 16, np.uint8).copy()
        v, st = oracle.ipv4_batch(region, np.array([0], np.uint64), 65535, 1)
        ok = st[0] == 0 and v[0] == 0
        bad += not ok
        if ok:
            assert got == built                      # delivered untouched
        else:
            assert got == b""                        # never delivered
    assert bad == n // 7
    assert stats["rx_verified"] == n and stats["rx_verify_failed"] == bad and stats["rx_dropped"] == bad


@pytest.mark.gpu
def test_rx_drop_forged_checksum_partial(tmp_path):
    """The CHECKSUM_PARTIAL exception holds on loopback only: a segment whose check
    word is the un-complemented pseudo-header fold — what Linux loopback leaves for offload — passes
    drop mode only when both its addresses are in 127/8 (martian anywhere but lo). The same forged
    word from 192.0.2.1 is a failed verification and never reaches the caller."""
    n = 2100
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_RX": "drop"},
                              forge=True)
    assert r.returncode == 0, r.stderr
    assert len(pkts) == n
    # with route_localnet set on any interface (kube-proxy does), 127/8 is no proof of lo:
    # the exception is off and the 127/8 partial segments are dropped as well
    localnet = route_localnet_any()
    assert stats["pool_localnet"] == int(localnet)
    forged = loop = 0
    for i, (built, got) in enumerate(pkts):
        region = np.frombuffer(built + b"\0" * 16, np.uint8).copy()
        v, st = oracle.ipv4_batch(region, np.array([0], np.uint64), 65535, 1)
        if i % 7 == 3:
            assert built[12] == 192 and st[0] & 4 and v[0] != 0   # looks CHECKSUM_PARTIAL, not loopback
            assert got == b""
            forged += 1
        elif i % 7 == 5:
            assert built[12] == 127 and built[16] == 127 and st[0] & 4
            assert got == (b"" if localnet else built)
            loop += 1
        else:
            assert st[0] == 0 and v[0] == 0 and got == built
    failed = forged + (loop if localnet else 0)
    assert stats["rx_verified"] == n and stats["rx_verify_failed"] == failed and stats["rx_dropped"] == failed
    assert stats["rx_partial"] == (0 if localnet else loop)


@pytest.mark.gpu
def test_rx_drop_truncated_tcp(tmp_path):
    """Drop mode with MSG_TRUNC into 600-byte buffers: an IPv4/TCP segment cut short
    cannot be verified, so it never reaches the caller's TCP handler; the ones that fit verify and
    arrive whole."""
    n = 1200
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_RX": "drop"},
                              trunc=True)
    assert r.returncode == 0, r.stderr
    fit = 0
    for built, got in pkts:
        if len(built) <= 600:
            assert got == built
            fit += 1
        else:
            assert got == b""
    assert 0 < fit < n
    assert stats["rx_skipped"] == n - fit and stats["rx_dropped"] == n - fit and stats["rx_verify_failed"] == 0


@pytest.mark.gpu
def test_rx_truncated_messages_bounded_by_buffer(tmp_path):
    """recvmmsg with MSG_TRUNC into 600-byte buffers: msg_len reports each datagram's full length,
    but only the 600 bytes the buffer holds are the segment's. Longer segments are truncated and
    SKIPPED (tot_len exceeds the bytes received) — never verified from bytes past the buffer —
    and the ones that fit verify (CPU checks, context.c:208)."""
    n = 1200
    r, pkts, stats = run_loop(tmp_path, n, {"TCPCSUM_PRELOAD_TX": "off", "TCPCSUM_PRELOAD_RX": "verify"},
                              trunc=True)
    assert r.returncode == 0, r.stderr
    assert len(pkts) == n
    fit = sum(len(built) <= 600 for built, _ in pkts)
    for built, got in pkts:
        assert got == built[:600]
    assert 0 < fit < n
    assert stats["rx_packets"] == n and stats["rx_skipped"] == n - fit
    assert stats["rx_verified"] == fit and stats["rx_verify_failed"] == 0


# ----------------------------------------------------------------- raw sockets
# The plumbing configuration (BASELINE configs[0]: stress over loopback, 1500-B
# MTU): tests/c/raw_echo echoes data segments through SOCK_RAW/IPPROTO_RAW
# sockets in a private network namespace, with the interposer in its DEFAULT
# mode (SOCK_RAW sockets only — no TCPCSUM_PRELOAD_ANY_SOCKET).
RAW = os.path.join(REPO, "tests", "c", "raw_echo")


def run_raw(tmp_path, n, env_extra, cpu=False):
    if not os.path.exists(RAW):
        subprocess.run(["make", "-C", REPO, "tests/c/raw_echo", "tcp_amd/libtcpcsum_preload.so"], check=True)
    out = tmp_path / "raw.bin"
    env = {k: v for k, v in os.environ.items() if not k.startswith("TCPCSUM_PRELOAD")}
    env.update({"LD_PRELOAD": PRELOAD, "TCPCSUM_PRELOAD_STATS": "1"})
    env.update(env_extra)
    r = subprocess.run([RAW, str(n), str(out)] + (["cpu"] if cpu else []), env=env, capture_output=True,
                       text=True, timeout=120)
    if r.returncode == 77:
        pytest.skip("no CAP_NET_RAW: neither user namespaces nor root: " + r.stdout.strip())
    summary = json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else {}
    pkts = []
    if r.returncode == 0:
        data = out.read_bytes()
        pos = 0
        while pos < len(data):
            (lo,) = struct.unpack_from("<I", data, pos)
            built = data[pos + 4:pos + 4 + lo]
            pos += 4 + lo
            (li,) = struct.unpack_from("<I", data, pos)
            got = data[pos + 4:pos + 4 + li]
            pos += 4 + li
            pkts.append((built, got))
    stats = {}
    m = re.search(r"tcpcsum_preload: (tx batches=.*)", r.stderr)
    if m:
        for side, body in zip(("tx", "rx"), m.group(1).split("|")[:2]):
            for k, v in re.findall(r"(\w+)=(\d+)", body):
                stats[f"{side}_{k}"] = int(v)
    return r, summary, pkts, stats


def ip_header_ok(pkt: bytes) -> bool:
    """The kernel fills the IPv4 header checksum of IPPROTO_RAW sends: RFC 1071 verify."""
    ihl = (pkt[0] & 15) * 4
    return oracle.csum_continue(0, pkt[:ihl], ihl) == 0


def same_but_kernel_fields(built: bytes, got: bytes) -> bool:
    """Equal except what the kernel writes into a raw IP_HDRINCL send: id when zero (the
    reference's (u16)htonl(54321) is 0 on little-endian) and the IP header checksum."""
    return len(built) == len(got) and built[:4] == got[:4] and built[6:10] == got[6:10] and built[12:] == got[12:]


def test_raw_echo_plumbing_passthrough(tmp_path):
    """The raw-socket echo runs end to end with the interposer passing through (TX/RX off)."""
    r, summary, pkts, stats = run_raw(tmp_path, 600, {"TCPCSUM_PRELOAD_TX": "off"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert summary["echoes_sniffed"] == 600 and len(pkts) == 600
    for built, got in pkts:
        assert same_but_kernel_fields(built, got) and ip_header_ok(got)
        assert got[36:38] == b"\0\0"                 # nobody filled the TCP check
    # Linux's own TCP receive path drops the unchecked echoes (no RST for them) and answers
    # only the client's correctly checked segments
    assert summary["kernel_rst"] == 600


def test_raw_echo_plumbing_config_cpu(tmp_path):
    """BASELINE configs[0] as the reference runs it: the echo server fills every check on the CPU
    (context.c:208-209) and the packets cross loopback through raw sockets; every sniffed echo equals
    the oracle's FILL and verifies to zero. No interposer."""
    env = {k: v for k, v in os.environ.items() if k != "LD_PRELOAD"}
    if not os.path.exists(RAW):
        subprocess.run(["make", "-C", REPO, "tests/c/raw_echo"], check=True)
    out = tmp_path / "raw.bin"
    r = subprocess.run([RAW, "2000", str(out), "cpu"], env=env, capture_output=True, text=True, timeout=120)
    if r.returncode == 77:
        pytest.skip("no CAP_NET_RAW: " + r.stdout.strip())
    assert r.returncode == 0, r.stdout + r.stderr
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    data = out.read_bytes()
    pos, n = 0, 0
    while pos < len(data):
        (lo,) = struct.unpack_from("<I", data, pos)
        built = data[pos + 4:pos + 4 + lo]
        pos += 4 + lo
        (li,) = struct.unpack_from("<I", data, pos)
        got = data[pos + 4:pos + 4 + li]
        pos += 4 + li
        assert built == oracle_fill(built)           # the server's CPU check is the reference's
        assert same_but_kernel_fields(built, got) and ip_header_ok(got)
        tcp = got[20:]
        ps = oracle.pseudo(int.from_bytes(got[12:16], "little"), int.from_bytes(got[16:20], "little"),
                           socket.htons(len(tcp)))
        assert oracle.csum_continue(ps, tcp, len(tcp)) == 0
        n += 1
    assert n == 2000 and summary["echoes_sniffed"] == 2000 and summary["server_checks"] == "cpu"
    # the Linux TCP stack accepts every echo's checksum: it answers each (no listener) with a RST,
    # as it does the client's segments
    assert summary["kernel_rst"] == 2 * 2000


@pytest.mark.gpu
def test_raw_echo_plumbing_on_gpu(tmp_path):
    """stress-style echo over SOCK_RAW: every echo's TCP check filled on the GPU at the server's
    sendmmsg equals the oracle's (context.c:208), every received batch verified on the GPU, the
    kernel's CHECKSUM_PARTIAL RSTs counted apart."""
    n = 3000
    r, summary, pkts, stats = run_raw(tmp_path, n, {"TCPCSUM_PRELOAD_RX": "verify"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert len(pkts) == n
    for built, got in pkts:
        assert same_but_kernel_fields(oracle_fill(built), got)
        assert ip_header_ok(got)
    assert stats["tx_filled"] == n and stats["tx_skipped"] == 0
    # rx: client segments (CPU checks) + sniffed echoes (GPU checks) verify; RSTs are partial
    assert stats["rx_verify_failed"] == 0
    assert stats["rx_partial"] == summary["kernel_rst"]
    # independent check by the Linux TCP stack: it RSTs every echo (so it accepted the GPU's
    # checksum) as well as every client segment
    assert summary["kernel_rst"] == 2 * n
    assert stats["rx_verified"] >= 2 * n + summary["kernel_rst"]
