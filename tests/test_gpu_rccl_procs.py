"""Multi-process RCCL tests on the box's one MI355X (tests/rccl_worker.py).

Every rank is its own process with its own RCCL communicator; the ranks share
the GPU and RCCL carries their bytes over its socket transport (each worker
sets a distinct NCCL_HOSTID, see rccl_worker.py).  This runs the comm ops —
the pipelined centralized op (MinMax and 1-bit), the pipelined ring op incl.
the multipath exchange from 6 ranks, hierarchical mode, the native scheduler —
through real RCCL grouped send/recv, alltoall and allgather across processes,
which the in-process loopback transport (test_gpu_multirank.py) only emulates
and the gloo rehearsals (test_distributed_sim.py) run without RCCL.  Every
rank's bytes must equal the oracle simulation of the reference op sequence.
Nothing here measures speed: the socket transport is not the xGMI path.
"""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle_np as NP
from oracle import simulate

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "rccl_worker.py")
F32, F16, BF16 = 0, 1, 2
TIMEOUT_S = 90


def run_procs(tmp_path, scenario: str, world: int, inputs: dict, **kw) -> list[dict]:
    np.savez(tmp_path / "inputs.npz", **inputs)
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update({"NCCL_HOSTID": f"bagua-test-rank-{r}", "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                    "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
        log = open(tmp_path / f"rank{r}.log", "w")
        procs.append((subprocess.Popen([sys.executable, "-u", WORKER, scenario, str(r), str(world), str(tmp_path)] +
                                       [f"{k}={v}" for k, v in kw.items()],
                                       stdout=log, stderr=subprocess.STDOUT, env=env, cwd=ROOT), log))
    failed = []
    for r, (p, log) in enumerate(procs):
        try:
            rc = p.wait(timeout=TIMEOUT_S)
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            rc = "timeout"
        log.close()
        if rc != 0:
            failed.append(r)
    if failed:
        tails = "\n".join(f"--- rank {r}:\n" + (tmp_path / f"rank{r}.log").read_text()[-1500:] for r in failed)
        pytest.fail(f"{scenario} ranks {failed} failed:\n{tails}")
    outs = []
    for r in range(world):
        with np.load(tmp_path / f"out{r}.npz", allow_pickle=False) as z:
            outs.append({k: z[k] for k in z.files})
    return outs


@pytest.mark.parametrize("world", [2, 3])
def test_collectives(tmp_path, world):
    rng = np.random.default_rng(world)
    n = 6 * 1000 + 6
    xs = [rng.integers(-100, 100, n).astype(np.float32) for _ in range(world)]  # exact sums in any order
    outs = run_procs(tmp_path, "collectives", world, {f"x{r}": x for r, x in enumerate(xs)})
    m = n // world * world
    cnt = m // world
    total = sum(xs)
    for r, o in enumerate(outs):
        assert np.array_equal(o["allreduce"].view(np.float32), total), r
        want_g = np.concatenate([xs[j][j * cnt:(j + 1) * cnt] for j in range(world)])
        assert np.array_equal(o["allgather"].view(np.float32), want_g), r
        want_t = np.concatenate([xs[j][r * cnt:(r + 1) * cnt] for j in range(world)])
        assert np.array_equal(o["alltoall"].view(np.float32), want_t), r
        assert np.array_equal(o["broadcast"].view(np.float32), xs[world - 1]), r
    assert np.array_equal(outs[0]["reduce"].view(np.float32), total)


def test_tapered_pieces_over_rccl(tmp_path, oracle_c, monkeypatch):
    """BAGUA_PIPELINE_TAPER (first and last piece half size) in every rank process: the
    pipelined MinMax op over real RCCL still equals the reference sequence."""
    monkeypatch.setenv("BAGUA_PIPELINE_TAPER", "1")
    world, cs = 4, 4 * 16384
    rng = np.random.default_rng(77)
    xs = [(rng.standard_normal(world * cs) * 1e-3).astype(np.float32) for _ in range(world)]
    want = simulate.centralized_low_precision(oracle_c, xs, F32, True)
    outs = run_procs(tmp_path, "centralized", world, {f"x{r}": x for r, x in enumerate(xs)},
                     method="MinMaxUInt8", dtype=F32, pieces=5, repeat=2, average=1)
    for r, o in enumerate(outs):
        for rep in ("t0", "t1"):
            assert np.array_equal(o[rep], want[r].view(np.uint8)), (r, rep)


@pytest.mark.parametrize("world,method,dtype,cs,pieces,average", [
    (2, "MinMaxUInt8", F32, 3 * 65536, 3, 1),  # pipelined, 3 pieces per chunk
    (4, "MinMaxUInt8", F16, 4 * 4096, 2, 0),   # reduce_sum (average = False)
    (3, "OneBit", F32, 3 * 4096, 2, 0),
    (4, "MinMaxUInt8", F32, 40960, 0, 1),      # automatic pieces
    (3, "MinMaxUInt8", BF16, 3 * 8192, 4, 1),
    (2, "MinMaxUInt8", F32, 12288, -1, 1),     # the reference's unfused sequence
    (2, "OneBit", F32, 5 * 4096, 3, 1),
    (4, "OneBit", BF16, 2 * 4096 + 7, 2, 1),   # ragged last tile
    (8, "MinMaxUInt8", F32, 8 * 4096, 0, 1),   # the driver's N = 8 shape (smaller bucket)
    (8, "OneBit", F32, 8 * 4096, 0, 1),
])
def test_centralized_ops(tmp_path, oracle_c, world, method, dtype, cs, pieces, average):
    rng = np.random.default_rng(world * 31 + cs)
    xs = [NP.from_f32((rng.standard_normal(world * cs) * 1e-3 + 2e-4 * r).astype(np.float32), dtype)
          for r in range(world)]
    if method == "MinMaxUInt8" and oracle_c.minmax_compressed_size(world, cs, dtype) % world:
        pytest.skip("reference alltoall requires S % nranks == 0")
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, bool(average),
                                              method="MinMaxUInt8" if method == "MinMaxUInt8" else "OneBitSignScale")
    outs = run_procs(tmp_path, "centralized", world, {f"x{r}": x for r, x in enumerate(xs)},
                     method=method, dtype=dtype, pieces=pieces, repeat=2, average=average)
    for r, o in enumerate(outs):
        for rep in ("t0", "t1"):  # the op twice on one communicator: same bytes
            assert np.array_equal(o[rep], want[r].view(np.uint8)), (r, rep)


@pytest.mark.parametrize("world,dtype,n,pieces,multipath", [
    (2, F32, 100003, 3, 0),
    (3, BF16, 65536 * 2, 0, 0),
    (6, F32, 6 * 4096 + 100, 2, 1),            # multipath exchange: 3 direct slices + relays
    (6, BF16, 50000, 1, 1),
    (8, BF16, 8 * 8192, 0, 1),                 # config 5's rank count, multipath
])
def test_decentralized_ring_op(tmp_path, oracle_c, world, dtype, n, pieces, multipath):
    rng = np.random.default_rng(world * 7 + n)
    arrs = {k: [NP.from_f32((rng.standard_normal(n) * 1e-3).astype(np.float32), dtype) for _ in range(world)]
            for k in "twlr"}
    want = simulate.decentralized_low_precision(oracle_c, arrs["t"], arrs["w"], arrs["l"], arrs["r"], dtype)
    inputs = {f"{k}{r}": arrs[k][r] for k in "twlr" for r in range(world)}
    outs = run_procs(tmp_path, "decentralized", world, inputs, dtype=dtype, pieces=pieces, multipath=multipath)
    for r, o in enumerate(outs):
        for i, k in enumerate("twlr"):
            assert np.array_equal(o[k], want[i][r].view(np.uint8)), (r, k)


def test_hierarchical(tmp_path, oracle_c):
    """2 emulated nodes x 2 ranks: ncclReduce(AVG) into each leader, the compressed op
    between the leaders, ncclBroadcast back (comm_ops.cpp hierarchical)."""
    nodes, per_node = 2, 2
    world = nodes * per_node
    n = 4 * 8192
    rng = np.random.default_rng(5)
    xs = [(rng.standard_normal(n) * 1e-3).astype(np.float32) for _ in range(world)]
    outs = run_procs(tmp_path, "hierarchical", world, {f"x{r}": x for r, x in enumerate(xs)}, per_node=per_node)
    # two ranks per node: RCCL's AVG (pre-multiplied or post-divided) is exactly (x0 + x1) / 2
    avgs = [((xs[2 * k] + xs[2 * k + 1]) / np.float32(2)).astype(np.float32) for k in range(nodes)]
    want = simulate.centralized_low_precision(oracle_c, avgs, F32, True)
    for r, o in enumerate(outs):
        assert np.array_equal(o["t"], want[r // per_node].view(np.uint8)), r


def test_bench_side_line_timeout_recovers(tmp_path):
    """A side line past its limit (BAGUA_BENCH_FAIL_SIDE: the scheduler's lanes run, limit 0 s)
    aborts the communicator; every rank rebuilds it, the scheduler workload is rebuilt on
    the new one, and the remaining side lines (one lane, 1-bit, config 5) still measure."""
    import json
    env = dict(os.environ)
    env.update({"BAGUA_BENCH_SHARED_GPU": "1", "NCCL_IB_DISABLE": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                "BAGUA_BENCH_FAIL_SIDE": "scheduler_lanes3"})
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--elements", str(1 << 22), "--cpu-seconds", "1"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["value"] > 0 and "headline_fallback" not in d, d
    assert set(d["side_errors"]) == {"scheduler_lanes3"}, d["side_errors"]
    sc = d["scheduler_buckets"]
    assert sc["lanes_1"]["ms_per_step"] > 0, sc
    assert d["onebit_allreduce"]["ms_per_step"] > 0 and d["decentralized_bf16"]["ms_per_step"] > 0


# the N > 1 line's skippable side lines in the order they run (bench.py bench_allreduce)
SIDE_ORDER = ["onebit", "unpieced", "bucket_25mib", "bucket_25mib_fp32", "decentralized", "onebit_unpieced",
              "scheduler_buckets", "pieces_2", "pieces_8", "pieces_4_tapered", "pieces_5_tapered"]


def test_bench_line_budget(tmp_path):
    """The N > 1 line under a wall budget (--budget-s 60 from process start): the headline,
    the fp32 all-reduce and comm-only always run; the side line "unpieced" is made to take
    60 s longer (BAGUA_BENCH_SPEND), so every side line after it is skipped -- the line
    still prints its one JSON line, with the skipped lines named, in order."""
    import json
    import time
    env = dict(os.environ)
    env.update({"BAGUA_BENCH_SHARED_GPU": "1", "NCCL_IB_DISABLE": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                "BAGUA_BENCH_SPEND": "unpieced:60"})
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--elements", str(1 << 22), "--cpu-seconds", "1", "--budget-s", "60"]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    wall = time.time() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["fp32_allreduce_gib_s"] > 0 and d["ratio_vs_fp32"] > 0, d
    assert d["comm_only_ms"] > 0 and d["budget_s"] == 60 and "phase_wall_s" in d, d
    assert d["onebit_allreduce"]["ms_per_step"] > 0 and d["unpieced_ms_per_step"] > 0, d
    assert d["skipped_for_budget"] == SIDE_ORDER[2:], d["skipped_for_budget"]  # everything after "unpieced"
    assert "side_errors" not in d, d
    assert wall < 60 + 60, wall


def test_bench_line_zero_budget(tmp_path):
    """--budget-s 0: every skippable side line is skipped (decentralized and the scheduler
    blocks included), the required ones still measure."""
    import json
    env = dict(os.environ)
    env.update({"BAGUA_BENCH_SHARED_GPU": "1", "NCCL_IB_DISABLE": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--elements", str(1 << 22), "--cpu-seconds", "1", "--budget-s", "0"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["value"] > 0 and d["fp32_allreduce_gib_s"] > 0 and d["comm_only_ms"] > 0, d
    assert d["skipped_for_budget"] == SIDE_ORDER, d["skipped_for_budget"]
    assert d["decentralized_bf16"] is None and d["scheduler_buckets"] is None, d


@pytest.mark.parametrize("world,fail_headline,launcher", [(2, False, "self"), (8, False, "self"),
                                                          (2, True, "torchrun")])
def test_bench_line_multirank(tmp_path, world, fail_headline, launcher):
    """bench.py's N > 1 line (config 4 + side lines) end to end with `world` ranks on the one
    GPU (BAGUA_BENCH_SHARED_GPU), started as plain `python3 bench.py --gpus N` (bench.py
    launches its own rank processes, launcher "self") or under torch.distributed.run: the
    pipelined headline must
    not fall back, and the side measurements must not fail (8 ranks: the direct ring
    exchange and the opt-in multipath side line).  fail_headline: the headline's communicator
    is aborted (BAGUA_BENCH_FAIL_HEADLINE, ncclCommAbort on every rank), so the line must come
    from the unpieced op on a fresh RCCL communicator, with every side line still measured."""
    import json
    env = dict(os.environ)
    env.update({"BAGUA_BENCH_SHARED_GPU": "1", "NCCL_IB_DISABLE": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    if fail_headline:
        env["BAGUA_BENCH_FAIL_HEADLINE"] = "1"
    args = ["--gpus", str(world), "--steps", "3", "--warmup", "1", "--elements", str(1 << 22), "--cpu-seconds", "1"]
    if launcher == "self":
        env.pop("WORLD_SIZE", None)
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={29517 + world + 20 * fail_headline}",
               os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["value"] > 0 and d["config"]["config_index"] == 4
    assert "side_errors" not in d, d
    assert d["onebit_allreduce"]["ms_per_step"] > 0 and d["decentralized_bf16"]["ms_per_step"] > 0
    small = d["bucket_25mib"]  # Bagua's default bucket size, op and fp32 all-reduce side by side
    assert small["ms_per_step"] > 0 and small["fp32_ms_per_step"] > 0 and small["elements_per_rank"] % world == 0
    if fail_headline:
        assert d["headline_fallback"]["headline"].startswith("unpieced") and d["pieces"] == 1, d
    else:
        assert "headline_fallback" not in d, d
        assert set(d["pieces_sweep_ms_per_step"]) == {"2", "8", "4_tapered", "5_tapered"}, d
        # the headline's piece count is chosen on the node during the warmup
        tune = d["pieces_autotune_ms_per_step"]
        best = min(tune, key=tune.get)
        assert set(tune) == {"1", "2", "4", "8", "16", "4_tapered", "8_tapered"}, d
        assert d["pieces"] == int(best.split("_")[0]) and d["pieces_tapered"] == best.endswith("_tapered"), d
        assert all(v > 0 for v in d["pieces_sweep_ms_per_step"].values()), d["pieces_sweep_ms_per_step"]
    assert d["roofline"]["frac"] > 0
    sc = d["scheduler_buckets"]  # the native scheduler over this RCCL communicator, lanes and one lane
    assert sc and sc["lanes_1"]["ms_per_step"] > 0 and len([k for k in sc if k.startswith("lanes_")]) == 3, sc
    timed_lanes = {int(k[6:]): v["ms_per_step"] for k, v in sc.items() if k.startswith("lanes_") and k[6:].isdigit()}
    assert sc["lanes_chosen"] == min(timed_lanes, key=timed_lanes.get), sc
    assert d["skipped_for_budget"] == [] and d["budget_s"] == 420, d
    # the CPU path beside every N: rank 0 runs the op sequence for all ranks on the host cores
    c = d["cpu_baseline"]
    assert c and c["value"] > 0 and c["cores"] >= 1 and c["host"]["os_cpu_count"] >= 1 and str(world) in c["sample"]
    assert d["hw_queues"]["effective"] == "8", d["hw_queues"]
    ph = d["phase_wall_s"]  # where the line's wall time went, phase by phase (rank 0's clock)
    for k in ("startup", "setup", "headline", "fp32_allreduce", "scheduler_buckets", "onebit", "cpu_baseline"):
        assert ph[k] >= 0, (k, ph)
    assert abs(ph["unaccounted"]) <= 0.05 * ph["process_wall"], ph


def test_native_scheduler(tmp_path, oracle_c):
    world, nb, per = 2, 3, 2 * 16384
    rng = np.random.default_rng(9)
    xs = {(b, r): (rng.standard_normal(per) * 1e-3).astype(np.float32) for b in range(nb) for r in range(world)}
    outs = run_procs(tmp_path, "backend", world, {f"b{b}_{r}": x for (b, r), x in xs.items()}, buckets=nb)
    for b in range(nb):
        want = simulate.centralized_low_precision(oracle_c, [xs[(b, r)] for r in range(world)], F32, True)
        for r in range(world):
            assert np.array_equal(outs[r][f"b{b}"], want[r].view(np.uint8)), (b, r)


@pytest.mark.parametrize("lanes,steps,nb", [(1, 2, 7), (3, 2, 7)])
def test_native_scheduler_lanes_over_rccl(tmp_path, oracle_c, lanes, steps, nb):
    """Scheduler lanes over a real RCCL communicator: with 3 lanes, consecutive buckets'
    collectives go out on different streams of ONE ncclComm, and stay correct only because
    RCCL runs a communicator's operations in the order they are issued, whatever the stream
    (every rank's scheduler worker issues them in the same order).  7 buckets over 2 steps,
    each step's output feeding the next: every bucket's bytes equal the oracle's two
    applications of the reference op, with 3 lanes and with 1."""
    world, per = 2, 2 * 8192
    rng = np.random.default_rng(90 + lanes)
    xs = {(b, r): (rng.standard_normal(per) * 1e-3).astype(np.float32) for b in range(nb) for r in range(world)}
    outs = run_procs(tmp_path, "backend", world, {f"b{b}_{r}": x for (b, r), x in xs.items()}, buckets=nb,
                     lanes=lanes, steps=steps)
    for r in range(world):
        assert int(outs[r]["lanes"][0]) == lanes
    for b in range(nb):
        want = [xs[(b, r)] for r in range(world)]
        for _ in range(steps):
            want = simulate.centralized_low_precision(oracle_c, want, F32, True)
        for r in range(world):
            assert np.array_equal(outs[r][f"b{b}"], want[r].view(np.uint8)), (b, r)


def test_schedule_mismatch_over_rccl(tmp_path, oracle_c):
    """Rank 0's schedule switches win at creation (rank 1's own BAGUA_PIPELINE_TAPER is
    ignored, rank 0's BAGUA_CHECK_SCHEDULE reaches rank 1); with the check on, ranks asking
    for different piece counts, or one the pipelined op and the other the unfused one, all
    fail with invalid argument before posting anything, tensors untouched, and the same
    communicator then runs a matching op bit-exactly."""
    world, cs = 2, 4 * 16384
    rng = np.random.default_rng(515)
    xs = [(rng.standard_normal(world * cs) * 1e-3).astype(np.float32) for _ in range(world)]
    want = simulate.centralized_low_precision(oracle_c, xs, F32, True)
    outs = run_procs(tmp_path, "mismatch", world, {f"x{r}": x for r, x in enumerate(xs)})
    for r, o in enumerate(outs):
        assert o["rc"].tolist() == [0, 1, 1, 0], (r, o["rc"])
        assert o["cfg"].tolist() == [4, 1 << 20, -1, 0, 1], (r, o["cfg"])  # rank 0's switches on both
        assert np.array_equal(o["same"], want[r].view(np.uint8)), r
        assert np.array_equal(o["after_pieces"], xs[r].view(np.uint8)), r
        assert np.array_equal(o["after_kind"], xs[r].view(np.uint8)), r
        assert np.array_equal(o["again"], want[r].view(np.uint8)), r


def test_stuck_op_fails_over_rccl(tmp_path):
    """lib.rs:255-265 monitor: rank 1 never posts the op, so rank 0's alltoall waits for a
    peer that never comes.  After the 3 s limit the monitor aborts rank 0's communicator
    (ncclCommAbort), wait_pending_comm_ops raises within the limit plus a margin, and the
    scheduler is destroyed without hanging."""
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(2 * 65536) * 1e-3).astype(np.float32)
    outs = run_procs(tmp_path, "stuck", 2, {"x0": x}, limit=3)
    o = outs[0]
    assert bool(o["raised"][0]) and int(o["failures"][0]) == 1 and bool(o["aborted"][0]), o
    assert 3.0 <= float(o["elapsed"][0]) < 3.0 + 15.0, o["elapsed"]
