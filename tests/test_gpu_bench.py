"""The bench.py contract the driver reads: ONE strict-JSON line on stdout with
the metric, the whole-job value, the roofline of the dominant kernel and the
CPU baseline (N = 1), for the default run and the other workloads.  Short
runs (a few steps) in a child process; the numbers themselves are not checked
here, only that they are present, finite and consistent with each other."""
import json
import math
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
METRIC = "GiB/s fp32 gradient encode+decode (device-resident); 1/2/4/8-GPU compressed all-reduce GiB/s"


def run_bench(*args, timeout=150):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                         text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, f"stdout must be one JSON line, got {len(lines)}: {out.stdout[:500]}"
    return json.loads(lines[0])


def check_common(d, steps, warmup):
    assert d["metric"] == METRIC and d["unit"] == "GiB/s"
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert math.isfinite(d["value"]) and d["value"] > 0 and d["ms_per_step"] > 0
    assert "workload" in d["config"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    # achieved = algorithmic bytes per launch / the launch's measured duration
    assert abs(r["achieved"] - r["alg_bytes_per_launch"] / (r["avg_launch_us"] * 1e-6) / 1e9) < 0.01 * r["achieved"]


@pytest.fixture(scope="module")
def default_line():
    return run_bench("--steps", "20", "--warmup", "3", "--cpu-seconds", "0.5")


@pytest.fixture(scope="module")
def allreduce_line():
    return run_bench("--workload", "allreduce", "--steps", "20", "--warmup", "3", "--cpu-seconds", "0.5",
                     "--no-decentralized", timeout=200)


def test_default_run_is_config2_with_cpu_baseline(default_line):
    d = default_line
    check_common(d, 20, 3)
    assert d["config"]["config_index"] == 2 and d["config"]["bucket_elements"] == 1 << 26
    # value = 256 MiB of fp32 gradient per step
    assert abs(d["value"] - 256 / 1024 / (d["ms_per_step"] * 1e-3)) < 0.01 * d["value"]
    assert d["roofline"]["kernel"] == "minmax_resident_encode_kernel"
    assert d["roofline"]["traffic"] and d["roofline"]["traffic"] > 0  # committed PMC summary
    src = d["roofline"]["traffic_source"]  # labelled as a committed record, not a live count
    assert src.startswith("profiles/") and "not live" in src and os.path.exists(os.path.join(ROOT, src.split()[0]))
    check_cpu(d)
    # the CPU leg runs on the same 256 MiB bucket, and its bytes equal the GPU's
    assert "256 MiB bucket" in d["cpu_baseline"]["sample"] and d["cpu_baseline"]["matches_gpu_bytes"] is True


def check_cpu(d):
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0 and c["sample"]
    h = c["host"]
    assert h["os_cpu_count"] >= 1 and h["affinity_cpus"] >= 1 and "cpu_model" in h
    assert d["hw_queues"]["effective"] == d["hw_queues"]["inherited"]  # N = 1 leaves the setting alone


def test_onebit_run():
    d = run_bench("--workload", "onebit", "--steps", "5", "--warmup", "2", "--cpu-seconds", "0.5")
    check_common(d, 5, 2)
    assert d["config"]["config_index"] == 3
    assert d["roofline"]["kernel"] == "onebit_encode_kernel"
    check_cpu(d)
    assert d["cpu_baseline"]["matches_gpu_bytes"] is True


def test_allreduce_run_single_rank(allreduce_line):
    d = allreduce_line
    check_common(d, 20, 3)
    check_cpu(d)
    assert d["config"]["config_index"] == 4 and d["config"]["parallelism"] == "dp1"
    assert d["fp32_allreduce_gib_s"] > 0 and d["onebit_allreduce"]["ms_per_step"] > 0
    small = d["bucket_25mib"]
    assert small["elements_per_rank"] == (25 << 20) // 4 - ((25 << 20) // 4) % 128
    assert small["ms_per_step"] > 0 and small["fp32_ms_per_step"] > 0 and small["gib_s_total"] > 0
    assert "side_errors" not in d


def test_default_line_carries_config4_point(default_line, allreduce_line):
    """The default N = 1 line also times config 4 at one rank (allreduce_p1), so the driver's
    1 -> 8 GPU curve has a same-workload N = 1 point; it agrees with --workload allreduce."""
    a = default_line["allreduce_p1"]
    assert a["config_index"] == 4 and a["n_ranks"] == 1
    assert a["ms_per_step"] > 0 and a["fp32_allreduce_ms_per_step"] > 0 and a["ratio_vs_fp32"] > 0
    assert abs(a["gib_s"] - 1.0 / (a["ms_per_step"] * 1e-3)) < 0.01 * a["gib_s"]  # 1 GiB per step
    # every kernel of the op was timed by its own events, and the dominant one carries a roofline
    ks = a["op_kernels_us"]
    assert ks and all(v > 0 for v in ks.values())
    r = a["roofline"]
    assert r and r["kernel"] in {k.split(":", 1)[1] for k in ks}
    # algorithmic bytes above peak are possible only for the one-launch encode, whose SURVEY
    # figure counts a second read it serves on chip; every other kernel's algorithmic bytes
    # are its compulsory bytes, so a frac of 1 or more there would mean skipped work
    assert 0 < r["frac"] < (1.2 if r["kernel"] == "minmax_resident_encode_kernel" else 1.0), r
    ref = allreduce_line["ms_per_step"]
    assert abs(a["ms_per_step"] - ref) <= 0.05 * ref, (a["ms_per_step"], ref)
    # and config 5 (2^27 bf16 ring op) at one rank
    assert a["ring_bf16_config5_ms_per_step"] > 0
    assert abs(a["ring_bf16_config5_gib_s"] * a["ring_bf16_config5_ms_per_step"] * 1e-3 - 0.25) < 0.01
