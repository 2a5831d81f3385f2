"""CPU tests of bench.py's host-side legs: the cpu_baseline functions (the
reference algorithm = the C oracle on the host cores) and the
host description every line carries.  No GPU: small tensors on the CPU."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _args(**kw):
    a = argparse.Namespace(cpu_seconds=0.05)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_host_info_fields():
    h = bench.host_info()
    assert h["os_cpu_count"] >= 1 and h["affinity_cpus"] >= 1
    assert "cpu_model" in h and "cpu_quota" in h and "omp_num_threads_env" in h
    assert 1 <= h["threads_allowed"] <= h["affinity_cpus"]


def test_cpu_baseline_threads_follow_the_host_rules(monkeypatch, oracle_c):
    """cores = min(cgroup quota, affinity, OMP_NUM_THREADS): what the box allows, stated"""
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: 2.5)
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    n, lim = bench.cpu_baseline_threads()
    assert n == min(2, lim["affinity_cpus"]) and lim["cpu_quota"] == 2.5
    x = torch.randn(1 << 14) * 1e-3
    c = bench.cpu_codec_baseline(_args(), x, None)
    assert c["cores"] == n
    monkeypatch.undo()
    bench._oracle_threads(oracle_c)  # later tests: the host's own rule again


def test_cpu_codec_baseline_same_bucket(oracle_c):
    x = torch.randn(1 << 16) * 1e-3
    comp = torch.from_numpy(oracle_c.compress_minmax_u8(x.numpy(), 0, 1))
    c = bench.cpu_codec_baseline(_args(), x, comp)
    assert c["kind"] == "port" and c["value"] > 0 and c["cores"] >= 1
    assert c["matches_gpu_bytes"] is True  # the given bytes are the oracle's own here
    assert "0 MiB bucket" in c["sample"] or "MiB bucket" in c["sample"]
    bad = comp.clone()
    bad[40] ^= 1
    assert bench.cpu_codec_baseline(_args(), x, bad)["matches_gpu_bytes"] is False


def test_cpu_codec_baseline_onebit_and_bf16(oracle_c):
    x = (torch.randn(1 << 15) * 1e-3).to(torch.bfloat16)
    c = bench.cpu_codec_baseline(_args(), x, None, onebit=True)
    assert c["value"] > 0 and c["matches_gpu_bytes"] is None and "1-bit" in c["sample"]


def test_cpu_allreduce_baseline_all_ranks(oracle_c):
    c = bench.cpu_allreduce_baseline(_args(), 4, 1 << 14, torch.device("cpu"), sample_elems=1 << 12)
    assert c["value"] > 0 and "4 ranks" in c["sample"] and c["host"]["os_cpu_count"] >= 1


def _fake_rank(tmp_path, body):
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time, json\nr = int(os.environ['RANK'])\nw = int(os.environ['WORLD_SIZE'])\n"
                      + body)
    return [sys.executable, str(script)]


def test_launch_ranks_forwards_rank0_line(tmp_path, capsys):
    """`python3 bench.py --gpus N` with no launcher: N rank processes with the
    torch.distributed env contract, rank 0's one line forwarded, exit 0."""
    cmd = _fake_rank(tmp_path, "assert os.environ['MASTER_ADDR'] == '127.0.0.1' and int(os.environ['MASTER_PORT'])\n"
                               "assert os.environ['LOCAL_RANK'] == str(r)\n"
                               "if r == 0: print(json.dumps({'n_gpus': w}))\n")
    assert bench.launch_ranks(4, [], child_cmd=cmd) == 0
    out = capsys.readouterr().out.strip().splitlines()
    assert out == ['{"n_gpus": 4}']


def test_launch_ranks_stops_every_rank_when_one_fails(tmp_path, capsys):
    """a rank that dies leaves the others waiting in a collective: the launcher stops
    them and fails with the dead rank's code (no line printed)."""
    import time
    cmd = _fake_rank(tmp_path, "if r == 1: sys.exit(3)\ntime.sleep(600)\n")
    t0 = time.time()
    assert bench.launch_ranks(3, [], child_cmd=cmd) == 3
    assert time.time() - t0 < 60
    assert capsys.readouterr().out == ""


def test_side_line_budget_rules():
    """The N > 1 line's budget rules (bench.py side_skipped / side_limit_s / side_steps):
    required lines always run with the full side limit; others are skipped below
    MIN_SIDE_S left, aborted at what is left, and sized to a fifth of it."""
    import bench
    m, lim = bench.MIN_SIDE_S, bench.SIDE_TIMEOUT_S
    assert not bench.side_skipped(-100.0, True) and bench.side_limit_s(-100.0, True) == lim
    assert bench.side_skipped(m - 0.1, False) and not bench.side_skipped(m, False)
    assert bench.side_limit_s(1000.0, False) == lim and bench.side_limit_s(30.0, False) == 30.0
    assert bench.side_limit_s(m + 1, False) == m + 1 and bench.side_limit_s(1.0, False) == m
    assert bench.side_steps(1000.0, 0.001, 25) == 25  # plenty of budget: the nominal count
    assert bench.side_steps(100.0, 2.0, 25) == 10  # 0.2 * 100 s / 2 s
    assert bench.side_steps(0.0, 2.0, 25) == 2 and bench.side_steps(-5.0, 0.0, 25) == 2  # never below 2


def test_budget_helpers_not_shadowed():
    """no assignment in bench.py rebinds a budget helper's name (a local dict of that name
    once turned every N > 1 side line into a caught TypeError)"""
    import ast
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "bench.py")) as f:
        tree = ast.parse(f.read())
    helpers = {"side_skipped", "side_limit_s", "side_steps"}
    bound = [(n.id, n.lineno) for n in ast.walk(tree) if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Store)
             and n.id in helpers]
    assert not bound, bound
