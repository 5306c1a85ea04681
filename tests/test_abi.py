"""CPU: the C-ABI library loads, exports every symbol include/tcpcsum.h declares,
its host-side logic behaves, and the scalar drop-ins equal the oracle.
No GPU compute here."""
import ctypes
import os
import random
import re
import socket
import subprocess

import numpy as np
import pytest

import oracle
import tcp_amd
from tcp_amd import api

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "tcpcsum.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(tcpcsum_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    L = tcp_amd.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    # the ctypes signature table covers the whole header
    assert set(names) == set(api.SIGNATURES)


def test_nm_exports_match_header():
    out = subprocess.run(["nm", "-D", "--defined-only", tcp_amd.lib_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (tcpcsum_[a-z0-9_]+)", out))
    assert set(declared_functions()) <= exported


def test_header_constants_match_python():
    text = open(HEADER).read()
    consts = dict(re.findall(r"#define (TCPCSUM_[A-Z0-9_]+) \(?(-?\d+)\)?", text))
    assert int(consts["TCPCSUM_OK"]) == api.OK
    assert int(consts["TCPCSUM_EINVAL"]) == api.EINVAL
    assert int(consts["TCPCSUM_ENODEV"]) == api.ENODEV
    assert int(consts["TCPCSUM_EHIP"]) == api.EHIP
    assert int(consts["TCPCSUM_ENOMEM"]) == api.ENOMEM
    assert int(consts["TCPCSUM_IPV4_FILL"]) == api.IPV4_FILL
    assert int(consts["TCPCSUM_IPV4_VERIFY"]) == api.IPV4_VERIFY
    assert int(consts["TCPCSUM_PKT_SKIPPED"]) == api.PKT_SKIPPED
    assert int(consts["TCPCSUM_PKT_IPHDR_BAD"]) == api.PKT_IPHDR_BAD
    assert int(consts["TCPCSUM_PKT_CSUM_PARTIAL"]) == api.PKT_CSUM_PARTIAL
    assert int(consts["TCPCSUM_IPV4_IPHDR"]) == api.IPV4_IPHDR
    assert int(consts["TCPCSUM_ABI_VERSION"]) == tcp_amd.lib().tcpcsum_abi_version()
    assert api.DESC_DTYPE.itemsize == 16


def test_library_is_a_product_build_of_this_tree():
    """the loaded library says which sources it was compiled from (sha256 over the
    Makefile's HASH_SRCS) and that no measurement knob was set; a stale or measurement build fails."""
    from tcp_amd import provenance
    info = provenance.check_product_build()
    assert info["abi"] == api.lib().tcpcsum_abi_version() and info["arch"] == "gfx950"
    assert info["knobs"] == {"TCPCSUM_MEASUREMENT_BUILD": 0, "TCPCSUM_TUNING_VARIANTS": 0, "TCPCSUM_TX_KNOCKOUT": 0,
                             "TCPCSUM_WIRE_WAVES": 1, "TCPCSUM_TX_WAVES": 1, "TCPCSUM_LINE_CPOL": 17,
                             "TCPCSUM_LOAD_CPOL": -1, "TCPCSUM_XCD_REMAP": 1,
                             "TCPCSUM_XCD_CHUNK": 0, "TCPCSUM_UNIFORM_WPB": 4,
                             "TCPCSUM_DESC_LB_WAVES": 1, "TCPCSUM_SS_LOAD": 2, "TCPCSUM_LB_VARIANT": 0, "TCPCSUM_LB_HEAD": 1,
                             "TCPCSUM_LB_HDR_X4": 1}
    # the only environment a product context reads
    assert info["runtime_knobs"] == ["TCPCSUM_HOST_THREADS", "TCPCSUM_HOST_NUMA", "TCPCSUM_HOST_SPIN_US",
                                     "LOCAL_WORLD_SIZE"]
    # the Makefile hashes the same files in the same order
    mk = open(os.path.join(REPO, "Makefile")).read()
    listed = re.search(r"HASH_SRCS := (.*?)\nSRC_HASH", mk, re.S).group(1).replace("\\", " ").split()
    assert tuple(listed) == provenance.HASH_SRCS


def test_product_library_does_not_contain_retired_knobs():
    """the host pipeline's A/B switches (measured and rejected, or kept for A/B runs)
    are read by measurement builds only — the product library's binary does not even hold their
    names, so no application environment can change the product path through them."""
    blob = open(api.lib_path(), "rb").read()
    for name in ("STAGE_BLOCKS", "STAGE_PASSES", "WIRE_NT", "DMA", "SLOT_SLEEP", "SLOTS", "CHUNK_MB",
                 "DMA_CHUNK_MB", "WIRE_THREADS", "BULK_THREADS", "NT", "POLL_US", "PINNED_DMA"):
        assert b"TCPCSUM_HOST_" + name.encode() not in blob, name
    for kept in (b"TCPCSUM_HOST_THREADS", b"TCPCSUM_HOST_NUMA", b"TCPCSUM_HOST_SPIN_US", b"LOCAL_WORLD_SIZE"):
        assert kept in blob


def test_product_build_refuses_measurement_knobs(tmp_path):
    """A knock-out or register-budget knob without -DTCPCSUM_MEASUREMENT_BUILD=1 is a compile error."""
    src = tmp_path / "k.hip"
    src.write_text('#include "tcpcsum_internal.h"\nint main() { return 0; }\n')
    base = ["/opt/rocm/bin/hipcc", "-fsyntax-only", "--offload-arch=gfx950", "-std=c++17", "-I", os.path.join(REPO, "include"),
            "-I", os.path.join(REPO, "tcp_amd", "csrc"), str(src)]
    if not os.path.exists(base[0]):
        pytest.skip("no hipcc")
    ok = subprocess.run(base, capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr
    for knob in ("-DTCPCSUM_TX_KNOCKOUT=8", "-DTCPCSUM_WIRE_WAVES=5", "-DTCPCSUM_TUNING_VARIANTS=1", "-DTCPCSUM_LINE_CPOL=2"):
        bad = subprocess.run(base + [knob], capture_output=True, text=True)
        assert bad.returncode != 0 and "measurement builds only" in bad.stderr, knob
        meas = subprocess.run(base + [knob, "-DTCPCSUM_MEASUREMENT_BUILD=1"], capture_output=True, text=True)
        assert meas.returncode == 0, meas.stderr


def test_library_never_page_locks_foreign_memory():
    """ABI v4: the library has no registration entry point and its code calls
    hipHostRegister / hipHostUnregister nowhere — the only page-locked memory it touches is its own
    hipHostMalloc or memory its owner locked."""
    L = tcp_amd.lib()
    for gone in ("tcpcsum_ctx_register_host", "tcpcsum_ctx_unregister_host", "tcpcsum_ctx_registered"):
        assert not hasattr(L, gone), gone
    und = subprocess.run(["nm", "-D", "--undefined-only", tcp_amd.lib_path()], capture_output=True, text=True,
                         check=True).stdout
    assert "hipHostRegister" not in und and "hipHostUnregister" not in und
    assert L.tcpcsum_ctx_set_flags(None, 0) == api.EINVAL


def test_scalar_dropins_equal_oracle():
    rng = random.Random(99)
    for _ in range(300):
        n = rng.randrange(0, 3000)
        p = bytes(rng.getrandbits(8) for _ in range(n))
        ss = rng.choice([0, 393210, rng.getrandbits(32), rng.getrandbits(48)])
        nb = rng.choice([n, max(n - 1, 0), -1])
        assert tcp_amd.csum_continue(ss, p, nb if nb >= 0 else 0) == oracle.csum_continue(ss, p, nb if nb >= 0 else 0)
        sa, da, ln = rng.getrandbits(32), rng.getrandbits(32), rng.getrandbits(16)
        assert tcp_amd.getPseudoHeaderSum(sa, da, ln) == oracle.pseudo(sa, da, ln)
    # negative nbytes is a no-op loop in the reference
    assert tcp_amd.lib().tcpcsum_continue(5, b"abc", -3) == oracle.csum_continue(5, b"abc", -3)


def test_scalar_kats(golden):
    for k in golden["kat_csum_continue"]:
        assert tcp_amd.csum_continue(k["sum_start"], bytes.fromhex(k["bytes"]), k["nbytes"]) == int(k["out"], 16)
    for k in golden["kat_pseudo"]:
        sa = socket.htonl(int(k["saddr_host"], 16))
        da = socket.htonl(int(k["daddr_host"], 16))
        assert tcp_amd.getPseudoHeaderSum(sa, da, socket.htons(k["len_host"] & 0xFFFF)) == k["out"]


def test_argument_errors_need_no_device():
    L = tcp_amd.lib()
    assert L.tcpcsum_batch_uniform_dev(None, 0, 0, None, 0, None, 0, None, None) == api.OK      # n == 0
    assert L.tcpcsum_batch_uniform_dev(None, 0, 10, None, 0, None, 5, None, None) == api.EINVAL
    assert L.tcpcsum_batch_uniform_dev(1 << 20, 0, 2**31, None, 0, 1 << 20, 5, None, None) == api.EINVAL
    assert L.tcpcsum_batch_desc_dev(1 << 20, (1 << 20) + 8, 5, 64, 1 << 20, None, None) == api.EINVAL   # unaligned
    assert L.tcpcsum_ipv4_batch_dev(1 << 20, 1 << 20, 1 << 20, 5, 1500, 7, None, None, None, None) == api.EINVAL
    assert L.tcpcsum_ipv4_batch_dev(1 << 20, 1 << 20, 1 << 20, 5, 1500, 4, None, None, None, None) == api.EINVAL
    assert L.tcpcsum_ipv4_batch_dev(1 << 20, 0, 1 << 20, 5, 1500, 0, None, None, None, None) == api.EINVAL
    assert L.tcpcsum_ipv4_batch_ptrs_dev(None, 1 << 20, 5, 1500, 0, 0, None, None, None, None) == api.EINVAL
    assert L.tcpcsum_ipv4_batch_ptrs_dev((1 << 20) + 4, 1 << 20, 5, 1500, 0, 0, None, None, None, None) == api.EINVAL
    assert L.tcpcsum_ipv4_batch_ptrs_dev(1 << 20, 1 << 20, 5, 1500, 0, 8, None, None, None, None) == api.EINVAL
    assert L.tcpcsum_ipv4_batch_ptrs_host(None, 1 << 20, 1 << 20, 5, 0, None, None) == api.EINVAL
    assert L.tcpcsum_ctx_set_tuning(None, None) == api.EINVAL
    assert L.tcpcsum_ctx_set_flags(None, 0) == api.EINVAL
    assert L.tcpcsum_ctx_get_stats(None, None) == api.EINVAL
    ng = ctypes.c_int()
    assert L.tcpcsum_stream_probe_dev(1 << 20, 17, 1 << 20, ctypes.byref(ng), None, None) == api.EINVAL
    T = api.Tuning
    for bad in (T(-1, 0, -1, 0), T(0, 3, -1, 0), T(0, 0, 15, 0), T(0, 0, -2, 0),
                T(0, 0, -1, 3),      # PIPE_ON | PIPE_OFF
                T(0, 0, -1, 12),     # NT_ON | NT_OFF
                T(0, 0, -1, 8192)):   # past the last TCPCSUM_TUNE_* bit
        assert L.tcpcsum_tuning_check(ctypes.byref(bad)) == api.EINVAL
        # every entry point rejects it before touching anything else (n == 0 included)
        assert L.tcpcsum_batch_uniform_dev(None, 0, 0, None, 0, None, 0, None, ctypes.byref(bad)) == api.EINVAL
        assert L.tcpcsum_ipv4_batch_dev(None, 0, None, 0, 0, 0, None, None, None, ctypes.byref(bad)) == api.EINVAL
        assert L.tcpcsum_plan_uniform(0, 1500, 1500, 10, ctypes.byref(bad), ctypes.byref(ng), ctypes.byref(ng),
                                      ctypes.byref(ng), ctypes.byref(ng)) == api.EINVAL
    assert L.tcpcsum_tuning_check(ctypes.byref(T(0, 0, -1, 0))) == api.OK
    assert L.tcpcsum_tuning_check(None) == api.OK
    assert L.tcpcsum_batch_uniform_host(None, None, 0, 0, None, 0, None, 0) == api.EINVAL
    assert L.tcpcsum_strerror(api.EHIP) == b"HIP runtime error"


def test_no_device_is_reported_not_faked():
    """On a box without a gfx950 GPU every device entry point fails loudly."""
    rc, arch = tcp_amd.device_check()
    if rc == api.OK:
        pytest.skip(f"a {arch} GPU is present")
    assert rc == api.ENODEV
    L = tcp_amd.lib()
    assert L.tcpcsum_batch_uniform_dev(1 << 20, 1500, 1500, None, 0, 1 << 20, 4, None, None) == api.ENODEV
    with pytest.raises(tcp_amd.TcpCsumError):
        tcp_amd.HostContext(0)


@pytest.mark.parametrize("base,stride,length,n,expect", [
    (0, 1500, 1500, 1 << 20, (1, 5)),       # 1M x 1500: 4-B aligned, 95 chunks -> 32 lanes x 3
    (0, 64, 64, 1 << 20, (0, 0)),           # 1M x 64: 16-B aligned, 4 lanes
    (0, 65536, 65536, 1 << 18, (0, 14)),    # 16 GiB of 64 KiB: a workgroup per segment, 4 KiB per wave
    (0, 65536, 65536, 1 << 14, (0, 14)),    # 1 GiB of 64 KiB: the same
    (4, 131072, 131072, 1 << 12, (1, 14)),  # 128 KiB, dword aligned (8193 chunks): the same
    (0, 32768, 32768, 1 << 14, (0, 13)),    # 32 KiB: four waves per segment (split)
    (0, 262144, 262144, 1 << 14, (0, 9)),   # 4 GiB of 256 KiB: resident one-wave-per-segment grid
    (0, 9000, 9000, 1 << 17, (1, 13)),      # jumbo, dword aligned: split
    (3, 1501, 1501, 100, (2, 5)),           # byte-granular
    (0, 1500, 1500, 1, (1, 5)),
    (12, 64, 64, 8, (1, 1)),                # misaligned 64 B touches 5 chunks
    (0, 8192, 8192, 10, (0, 13)),            # exactly 512 chunks: split
    (0, 8208, 8193, 10, (2, 9)),            # 514 chunks, byte-granular -> one wave per segment
])
def test_plan_uniform(base, stride, length, n, expect):
    mode, shape, unroll, blocks = api.plan_uniform(base, stride, length, n)
    assert (mode, shape) == expect
    # small tiles launch one tile per wave: the grid cap is then 1 << 24 (uncapped)
    assert unroll in (1, 2, 4, 8) and (1 <= blocks <= 32768 or blocks == 1 << 24)


@pytest.mark.parametrize("stride,length,unroll", [
    (1500, 1500, 1),    # 32-lane groups, two segments per wave: 3000 B
    (64, 64, 4),        # 4-lane groups, 16 per instruction x 4: 4096 B
    (128, 128, 4), (256, 256, 4), (512, 512, 4), (1024, 1024, 4),
    (2048, 2048, 2),    # 64-lane groups, one per instruction x 2: 4096 B
    (3000, 3000, 1), (4096, 4096, 1), (6000, 6000, 1),
    (1536, 1500, 1),    # the span is the stride
    (576, 576, 8),      # 64-lane groups, one per instruction x 8: 4608 B, the limit
])
def test_plan_tile_of_at_most_4608_bytes(stride, length, unroll):
    """The lane-group plan (profiles/r05_tile_sweep_xcd.jsonl): one wave tile per wave
    (grid cap 1 << 24, tiles in XCD order) of the most segments in flight whose span fits 4608 B."""
    mode, shape, u, blocks = api.plan_uniform(0, stride, length, 1 << 20)
    assert mode in (0, 1) and shape <= 8
    assert (u, blocks) == (unroll, 1 << 24)


def test_plan_byte_granular_keeps_its_grid():
    """Byte-granular batches keep 16384 looping workgroups and at most 4 in flight: the tile plan in
    XCD order measured 1-11 % slower for them (profiles/r05_plan_ab.jsonl)."""
    for length in (99, 577, 1499, 3001):
        mode, shape, u, blocks = api.plan_uniform(1, length, length, 1 << 20)
        assert mode == 2 and shape <= 8 and u <= 4 and blocks == 16384


def test_plan_respects_overrides():
    try:
        api.set_tuning(100, 1, -1, 0)
        assert api.plan_uniform(0, 1500, 1500, 1000)[2:] == (1, 100)
        api.set_tuning(0, 0, 6)                       # G=64 x C=2 covers 95 chunks: honoured
        assert api.plan_uniform(0, 1500, 1500, 1000)[1] == 6
        api.set_tuning(0, 0, 0)                       # 4 chunks cannot cover 1500 B: ignored
        assert api.plan_uniform(0, 1500, 1500, 1000)[1] == 5
    finally:
        api.set_tuning(0, 0, -1, 0)


def test_tuning_is_per_call_not_global():
    """The library keeps no tuning state: a tuned call never reshapes a later untuned one,
    and the Python default set by set_tuning() is per thread."""
    import threading
    t = api.make_tuning(0, 0, 6)
    assert api.plan_uniform(0, 1500, 1500, 1000, tune=t)[1] == 6
    assert api.plan_uniform(0, 1500, 1500, 1000)[1] == 5        # nothing stuck in the library
    seen = {}
    try:
        api.set_tuning(0, 0, 6)

        def other():
            seen["other"] = api.plan_uniform(0, 1500, 1500, 1000)[1]

        th = threading.Thread(target=other)
        th.start()
        th.join()
        seen["mine"] = api.plan_uniform(0, 1500, 1500, 1000)[1]
    finally:
        api.set_tuning(0, 0, -1, 0)
    assert seen == {"other": 5, "mine": 6}
    with pytest.raises(tcp_amd.TcpCsumError):
        api.make_tuning(0, 3)


def test_c_program_links_the_abi():
    exe = os.path.join(REPO, "tests", "c", "abi_smoke")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", REPO, "tests/c/abi_smoke"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
