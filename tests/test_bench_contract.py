"""bench.py's output contract (the driver parses its one JSON line): a short run on the GPU,
in a child process, every field the contract names present and consistent."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_contract():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--no-other-configs", "--host-steps", "1"],
                       cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["digest_check"] is True
    # value = whole-job bytes / wall time, GiB/s; the kernel's rate bounds it from above
    assert 0 < d["value"] < 7451
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert "workload" in d["config"]
    hp = d["host_path"]
    assert set(hp) == {"pageable", "pinned"} and all(hp[m]["digest_check"] is True for m in hp)
    assert d["host_path_order"] == "after the device configs"
    for m in hp:   # every rank's throttling and copy-thread budget
        assert len(hp[m]["cgroup_throttled_ms_per_rank"]) == 1 and len(hp[m]["copy_threads_per_rank"]) == 1
    assert d["stream_probe"]["avg_ms"] > 0


def test_bench_other_configs_carry_their_ceilings():
    """the 64-B config carries the read probe over its own rotation, and the wire
    leg the read and write-back probes over its own region; the wire FILL / VERIFY self-check holds
    after the write-back probe rewrote the lines it read."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--no-host-path", "--other", "64,wire"],
                       cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    oc = d["other_configs"]
    assert set(oc) == {"64", "wire_1500"}
    assert oc["64"]["digest_check"] is True and oc["64"]["stream_probe"]["kernel_over_probe"] > 0
    w = oc["wire_1500"]
    assert w["check"] is True
    for k in ("fill", "verify"):
        assert w[k]["kernel_avg_ms"] > 0
    assert w["copy_probe"]["bytes_moved_per_launch"] == (1 << 20) * (1536 + 128)
    assert w["fill_over_copy_probe"] > 0 and w["verify_over_read_probe"] > 0
