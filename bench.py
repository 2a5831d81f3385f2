#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X bagua-core gradient codec.

Metric (BASELINE.json): "GiB/s fp32 gradient encode+decode (device-resident);
1/2/4/8-GPU compressed all-reduce GiB/s".

  N = 1 (default): config 2 — one 256 MiB fp32 bucket (2^26 elements,
      n_chunks = 1), one step = MinMax-UInt8 encode (min/max pass + quantise
      pass) + decode, inputs resident in HBM.  value = 4*2^26 B / step time.
  N > 1 (torchrun, one rank per GPU): config 4 — every rank owns a 1 GiB fp32
      gradient (2^28 elements, seed 0x5EED + rank); one step = the compressed
      centralized all-reduce (compress -> RCCL alltoall -> fused dequantise +
      reduce + requantise -> RCCL allgather -> decompress).  value = the
      gradient bytes all ranks reduced / max-over-ranks step time (weak scaling:
      per-GPU bucket fixed).  The uncompressed fp32 RCCL all-reduce of the same
      bucket is timed beside it (fp32_allreduce_gib_s, ratio_vs_fp32).

Launch: `python3 bench.py --gpus N` starts its N rank processes itself (before
anything touches the GPU; launch_ranks), or runs as one rank under
torch.distributed.run (RANK / WORLD_SIZE / MASTER_* set by the launcher).

Every byte is produced by the gfx950 kernels through the C ABI
(bagua-core_amd/lib/*.so).  The oracle is used ONLY for the cpu_baseline leg
(rank 0, N = 1): the C restatement of the reference kernels timed on the
host's cores on a bounded sample.
"""
from __future__ import annotations

import time as _time

_PROCESS_T0 = _time.perf_counter()  # the N > 1 line's phase clock starts here (phase_wall_s)

import argparse
import ctypes
import json
import math
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bagua-core_amd"))
sys.path.insert(0, ROOT)


def launch_ranks(world: int, argv: list, child_cmd: list | None = None) -> int:
    """`python3 bench.py --gpus N` without a launcher: start N rank processes of this
    script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their
    environment, the way torch.distributed.run sets them; rank 0's gloo store is the
    rendezvous, as rank 0's unique id is in communicators/mod.rs:25-60), forward rank 0's
    one JSON line, and return non-zero if any rank fails (the others are then stopped,
    by PID).  Called before anything touches the GPU: this process never does."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = child_cmd or [sys.executable, os.path.abspath(__file__)] + list(argv)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      stdin=subprocess.DEVNULL, text=True))
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()

    def forward(signum, _frame):  # a launcher stopped by its caller stops its ranks too
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        sys.exit(128 + signum)

    old_handlers = {sig: signal.signal(sig, forward) for sig in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0] if bad[0] > 0 else 128 - bad[0]
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.2)
    if rc:
        for p in procs:  # a failed rank leaves the others waiting in a collective
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        print(f"bench.py: a rank failed (exit {rc}); every rank stopped", file=sys.stderr, flush=True)
    reader.join(timeout=30)
    for sig, h in old_handlers.items():
        signal.signal(sig, h)
    if rc == 0:
        sys.stdout.write("".join(out))
        sys.stdout.flush()
    return rc


def _maybe_launch() -> None:
    """--gpus N > 1 with no launcher environment: become the launcher (see launch_ranks)."""
    if "WORLD_SIZE" in os.environ:
        return
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    known, _ = ap.parse_known_args(sys.argv[1:])
    if known.gpus > 1:
        sys.exit(launch_ranks(known.gpus, sys.argv[1:]))


if __name__ == "__main__":
    _maybe_launch()

# The hardware-queue count this process inherited (the GPU box exports 4) and the
# one HIP will actually use: both go into every line ("hw_queues").
HW_QUEUES_INHERITED = os.environ.get("GPU_MAX_HW_QUEUES")
if int(os.environ.get("WORLD_SIZE", "1")) > 1:
    # N > 1: the pipelined ops overlap a side stream (RCCL pieces) with the codec
    # stream, and RCCL keeps internal streams of its own.  HIP maps streams onto
    # GPU_MAX_HW_QUEUES hardware queues round-robin (4 by default); two streams on
    # one queue serialise (profiles/r02_host_copy_ab.jsonl shows what that costs).
    # Set explicitly (not setdefault: an inherited 4 would win) before HIP
    # initialises; BAGUA_BENCH_HW_QUEUES overrides (A/B at the box's 4).
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("BAGUA_BENCH_HW_QUEUES", "8")
    if os.environ.get("BAGUA_BENCH_SHARED_GPU"):
        # rehearsal of the N > 1 line on a one-GPU box (tests/test_gpu_rccl_procs.py): every
        # rank on device 0, each its own "host" to RCCL (which refuses two ranks of one
        # communicator on one GPU of one host), so RCCL links them by its socket transport.
        # Exercises the code path, not the xGMI speed.
        os.environ["NCCL_HOSTID"] = f"bagua-bench-rank-{os.environ.get('RANK', '0')}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ["LOCAL_RANK"] = "0"

import torch  # noqa: E402

METRIC = ("GiB/s fp32 gradient encode+decode (device-resident); "
          "1/2/4/8-GPU compressed all-reduce GiB/s")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GiB = float(1 << 30)
SIDE_TIMEOUT_S = 120.0  # N > 1 side measurements: abort the communicator instead of hanging
MIN_SIDE_S = 10.0  # N > 1: a side line starts only with this much of --budget-s left
HEADLINE_TIMEOUT_S = 300.0  # N > 1 headline (pipelined op): abort, then measure the unpieced op
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06_pmc_traffic.json")
PMC_SUMMARY_ONEBIT = os.path.join(ROOT, "profiles", "r06_pmc_traffic_onebit.json")


# ---- the N > 1 line's wall budget (bench_allreduce `side`): every input is agreed
# over the ranks (the budget left is the min over ranks, a probe step's time the max), so
# every rank takes the same decisions
def side_skipped(left_s: float, required: bool) -> bool:
    """a side line that is not required is skipped once less than MIN_SIDE_S is left"""
    return not required and left_s < MIN_SIDE_S


def side_limit_s(left_s: float, required: bool) -> float:
    """abort a side line after SIDE_TIMEOUT_S, or what is left of the budget if less (never
    below MIN_SIDE_S); a required line keeps the full SIDE_TIMEOUT_S"""
    return SIDE_TIMEOUT_S if required else max(MIN_SIDE_S, min(SIDE_TIMEOUT_S, left_s))


def side_steps(left_s: float, t1_s: float, nominal: int) -> int:
    """timed steps of a side line: as many as fit in a fifth of what is left after one probe
    step of t1_s, between 2 and the nominal count"""
    return max(2, min(nominal, int(0.2 * max(0.0, left_s) / max(t1_s, 1e-9))))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["auto", "codec", "allreduce", "onebit", "host", "backend"], default="auto")
    ap.add_argument("--buckets", type=int, default=32, help="backend workload: gradient buckets per iteration")
    ap.add_argument("--bucket-mib", type=int, default=25, help="backend workload: MiB of fp32 gradient per bucket")
    ap.add_argument("--lanes", type=int, default=0,
                    help="backend workload: scheduler lanes (cross-bucket pipelining; 0 = the library default)")
    ap.add_argument("--elements", type=int, default=0, help="override bucket elements")
    ap.add_argument("--dtype", choices=["f32", "f16", "bf16"], default="f32",
                    help="codec workloads: gradient dtype (the headline is f32; bf16/f16 buckets keep 256 MiB)")
    ap.add_argument("--pieces", type=int, default=0,
                    help="pipelined all-reduce pieces per chunk (0 = automatic, 1 = unpieced)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--two-pass", action="store_true",
                    help="codec workload: force the two-kernel MinMax encode (BAGUA_RESIDENT=0) for A/B")
    ap.add_argument("--no-decentralized", action="store_true", help="skip the config-5 side measurement (N > 1)")
    ap.add_argument("--no-allreduce-p1", action="store_true",
                    help="default N = 1 line: skip the config-4 point at one rank (allreduce_p1)")
    ap.add_argument("--no-cold", action="store_true",
                    help="codec workloads: skip the two-bucket alternating side line")
    ap.add_argument("--host-buffers", type=int, default=2,
                    help="host workload: buckets in flight in the overlapped mode (device buffers per stage)")
    ap.add_argument("--copy-chunks", type=int, default=2,
                    help="host workload: pieces per H2D / D2H copy (1 = one copy each way per bucket)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="wall budget of the cpu_baseline leg")
    ap.add_argument("--budget-s", type=float, default=420.0,
                    help="N > 1: wall budget of the whole line from process start; the headline, the fp32 "
                         "all-reduce and comm-only always run, later side lines are skipped once it is spent "
                         "(skipped_for_budget)")
    ap.add_argument("--kernel-events-every", type=int, default=5,
                    help="codec workloads: the dominant kernel records start/stop events on every N-th timed step")
    ap.add_argument("--stream", choices=["own", "current"], default="own",
                    help="codec workloads: launch on a stream of their own or on torch's current (null) stream")
    return ap.parse_args()


class PhaseClock:
    """Wall seconds per phase of a line (this rank's clock), from the process start on, so a
    node run says where its time went (phase_wall_s; the phases sum to the process wall at
    the moment the line is printed)."""

    def __init__(self):
        self.t = _PROCESS_T0
        self.s = {}

    def lap(self, name: str) -> None:
        now = time.perf_counter()
        self.s[name] = self.s.get(name, 0.0) + (now - self.t)
        if int(os.environ.get("WORLD_SIZE", "1")) > 1 and os.environ.get("RANK", "0") == "0":
            # progress on stderr (stdout carries only the JSON line): a long N > 1 run is
            # visibly alive phase by phase
            print(f"bench.py: phase {name} {now - self.t:.1f} s (process {now - _PROCESS_T0:.1f} s)",
                  file=sys.stderr, flush=True)
        self.t = now

    def report(self) -> dict:
        total = time.perf_counter() - _PROCESS_T0
        out = {k: round(v, 3) for k, v in self.s.items()}
        out["unaccounted"] = round(total - sum(self.s.values()), 3)
        out["process_wall"] = round(total, 3)
        return out


PHASES = PhaseClock()


def pmc_traffic(kernel: str, summary: str = PMC_SUMMARY):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc
    summary (profiles/r04_pmc_traffic.json, produced by
    profiles/collect_pmc.py following MI355X_MICROARCH.md §HBM: FETCH_SIZE
    doubled for 16-B streaming reads, WRITE_SIZE as is), or None."""
    try:
        with open(summary) as f:
            d = json.load(f)
        return d.get("per_launch_hbm_bytes", {}).get(kernel)
    except (OSError, ValueError):
        return None


# ----------------------------------------------------------------- N = 1 ------
def bench_codec(args, onebit: bool = False):
    from bagua_core import _native as N
    K = N.K
    dcode, tdt, esz = {"f32": (0, torch.float32, 4), "f16": (1, torch.float16, 2),
                       "bf16": (2, torch.bfloat16, 2)}[args.dtype]
    n = args.elements or ((1 << 28) // esz)  # a 256 MiB bucket
    p = 1
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    x = (torch.randn(n, device=dev, generator=g) * 1e-3).to(tdt)
    y = torch.empty_like(x)
    # the codec runs on a stream of its own (a communicator's stream, as in the
    # comm ops), not on the null stream (--stream current: A/B)
    stream = torch.cuda.Stream(device=dev) if args.stream == "own" else torch.cuda.current_stream(dev)
    torch.cuda.synchronize()  # x was generated on the current stream
    sp = ctypes.c_void_p(stream.cuda_stream)
    if onebit:
        S = K.bagua_onebit_compressed_bytes(n, p)
        ws_bytes = K.bagua_onebit_workspace_bytes(n, p)
    else:
        S = K.bagua_minmax_u8_compressed_bytes(dcode, n, p)
        ws_bytes = K.bagua_minmax_u8_workspace_bytes(n, p)
    comp = torch.empty(S, dtype=torch.uint8, device=dev)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    xp, yp, cp, wp = x.data_ptr(), y.data_ptr(), comp.data_ptr(), ws.data_ptr()

    launches_for = None
    if onebit:
        # the compress call launches encode then finalize; the timing hook times its first kernel
        names = ["onebit_encode_kernel", "onebit_decode_kernel"]

        def launches_for(xq, yq, cq):
            return [lambda: K.bagua_onebit_compress(dcode, xq, n, n, p, cq, S, wp, ws_bytes, -1, sp),
                    lambda: K.bagua_onebit_decompress(dcode, cq, S, n, p, yq, sp)]

        def launches():
            return [lambda: K.bagua_onebit_compress(dcode, xp, n, n, p, cp, S, wp, ws_bytes, -1, sp),
                    lambda: K.bagua_onebit_decompress(dcode, cp, S, n, p, yp, sp)]
        alg = [esz * n + n // 8 + 4 * ((n + 1023) // 1024), n // 8 + 32 + esz * n]  # + per-tile |x| partials
    elif K.bagua_minmax_u8_resident_path(dcode, xp, n, n, p, cp, S, -1, sp) == 1:
        # one-launch encode (minmax_resident.hip): pass 1 keeps part of the bucket in
        # VGPRs/LDS across the min/max exchange (a single kernel per compress call)
        names = ["minmax_resident_encode_kernel", "minmax_dequantize_kernel"]

        def launches_for(xq, yq, cq):
            return [lambda: K.bagua_minmax_u8_compress(dcode, xq, n, n, p, cq, S, wp, ws_bytes, -1, sp),
                    lambda: K.bagua_minmax_u8_decompress(dcode, cq, S, n, p, yq, sp)]

        def launches():
            return [lambda: K.bagua_minmax_u8_compress(dcode, xp, n, n, p, cp, S, wp, ws_bytes, -1, sp),
                    lambda: K.bagua_minmax_u8_decompress(dcode, cp, S, n, p, yp, sp)]
        # algorithmic bytes per launch as SURVEY §8(d) counts them: encode 4N (min/max read) +
        # 4N (quantise read) + N + header, decode N + header read, 4N written.  This kernel
        # serves part of the second read from VGPRs/LDS; its compulsory bytes (4N + N) are
        # reported beside it (roofline.compulsory_*).
        alg = [2 * esz * n + n + 32, n + 32 + esz * n]
        compulsory = [esz * n + n + 32, n + 32 + esz * n]
    else:
        names = ["minmax_partials_kernel", "minmax_quantize_kernel", "minmax_dequantize_kernel"]

        def launches():
            return [lambda: K.bagua_minmax_u8_compress_stage(1, dcode, xp, n, n, p, cp, S, wp, ws_bytes, -1, sp),
                    lambda: K.bagua_minmax_u8_compress_stage(2, dcode, xp, n, n, p, cp, S, wp, ws_bytes, -1, sp),
                    lambda: K.bagua_minmax_u8_decompress(dcode, cp, S, n, p, yp, sp)]
        # algorithmic bytes per launch: partials read 4N; quantise read 4N + write N + header;
        # dequantise read N + header, write 4N.  Sum = 14N + 64p.
        alg = [esz * n, esz * n + n + 32, n + 32 + esz * n]
    if "compulsory" not in locals():
        compulsory = alg
    calls = launches()

    def step():
        for c in calls:
            rc = c()
            if rc:
                raise RuntimeError(f"kernel launch failed: {N.STATUS.get(rc, rc)}")

    # Kernel durations come from HIP events that the kernels themselves record
    # at their start and end (bagua_time_next_kernel -> hipExtLaunchKernel), so
    # they exclude dispatch overhead and agree with rocprofv3's kernel trace.
    def kernel_events(count):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(count)]
        for a, b in evs:  # torch creates the HIP events on first record
            a.record(stream)
            b.record(stream)
        return evs

    # warmup; the last steps time every kernel to find the dominant one
    nprof = min(5, max(1, args.warmup))
    for _ in range(max(0, args.warmup - nprof)):
        step()
    pev = [kernel_events(len(calls)) for _ in range(nprof)]
    torch.cuda.synchronize()
    for k in range(nprof):
        for i, c in enumerate(calls):
            N.check(K.bagua_time_next_kernel(pev[k][i][0].cuda_event, pev[k][i][1].cuda_event), "timing hook")
            c()
    torch.cuda.synchronize()
    per = [sum(pev[k][i][0].elapsed_time(pev[k][i][1]) for k in range(nprof)) / nprof for i in range(len(calls))]
    dom = max(range(len(calls)), key=lambda i: per[i])
    # timed region: K steps, wall clock between synchronisations; the dominant
    # kernel records its own start/stop events on every `--kernel-events-every`-th
    # step (each recorded pair costs the step ~3 us of dispatch: A/B in
    # profiles/r02_kernel_events_ab.jsonl), so its average launch duration is
    # measured live over the timed region on a sample of its steps
    every = max(1, args.kernel_events_every)
    sampled = list(range(0, args.steps, every))
    ev = kernel_events(len(sampled))
    resident = names[0] == "minmax_resident_encode_kernel"

    def give_ups():  # one-launch encode workgroups that timed out in the exchange (synchronises sp)
        c = ctypes.c_uint64(0)
        N.check(K.bagua_minmax_u8_resident_give_ups(sp, ctypes.byref(c)), "resident give-ups")
        return int(c.value)
    gu0 = give_ups() if resident else 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        for i, c in enumerate(calls):
            if i == dom and k % every == 0:
                K.bagua_time_next_kernel(ev[k // every][0].cuda_event, ev[k // every][1].cuda_event)
            rc = c()
            if rc:
                raise RuntimeError(f"kernel launch failed: {N.STATUS.get(rc, rc)}")
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gu_timed = give_ups() - gu0 if resident else None
    ms = wall * 1e3 / args.steps
    value = esz * n / (ms * 1e-3) / GiB  # gradient bytes processed (4N fp32, 2N bf16)
    dom_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    per[dom] = dom_ms
    achieved = alg[dom] / (per[dom] * 1e-3) / 1e9
    step_alg = sum(alg)
    # the committed PMC passes are of the default 256 MiB f32 bench (MinMax and 1-bit)
    traffic = (pmc_traffic(names[dom], PMC_SUMMARY_ONEBIT if onebit else PMC_SUMMARY)
               if (args.dtype == "f32" and n == (1 << 26)) else None)
    summary = PMC_SUMMARY_ONEBIT if onebit else PMC_SUMMARY
    roof = {"bound": "hbm", "kernel": names[dom], "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            # the PMC bytes are read from a committed rocprofv3 --pmc record of this command, not
            # counted during this run (counters need their own profiler passes)
            "traffic_source": (f"{os.path.relpath(summary, ROOT)} (committed rocprofv3 --pmc FETCH_SIZE / "
                               "WRITE_SIZE passes of this bench command; not live)") if traffic else None,
            "alg_bytes_per_launch": alg[dom], "avg_launch_us": round(per[dom] * 1e3, 2),
            "compulsory_bytes_per_launch": compulsory[dom],
            "compulsory_frac": round(compulsory[dom] / (per[dom] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    extra = {
        "per_kernel_us": {nm: round(t * 1e3, 2) for nm, t in zip(names, per)},
        "per_kernel_gbs": {nm: round(a / (t * 1e-3) / 1e9, 1) for nm, a, t in zip(names, alg, per)},
        # whole step by wall clock (launch gaps included): 14N + 64p algorithmic bytes
        "step_roofline": {"alg_bytes": step_alg, "compulsory_bytes": sum(compulsory),
                          "wall_us": round(ms * 1e3, 2),
                          "achieved_gbs": round(step_alg / (ms * 1e-3) / 1e9, 1),
                          "frac": round(step_alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "per_kernel_note": "kernel-recorded HIP events (hipExtLaunchKernel); dominant kernel over the timed region "
                           f"(every {every}th step: {len(sampled)} of {args.steps}), others over the last warmup steps",
        # workgroups of the one-launch encode that gave up waiting in its exchange over the
        # timed steps (0 unless something else held CUs; each give-up re-reads its slices)
        "resident_give_ups_timed": gu_timed,
        "encode_gib_s": round(esz * n / (sum(per[:-1]) * 1e-3) / GiB, 1),
        "decode_gib_s": round(esz * n / (per[-1] * 1e-3) / GiB, 1),
    }
    # Side line: the same steps alternating between two buckets, so each step's bucket
    # was last touched a whole other bucket ago (>= 2 x 256 MiB of traffic since: no
    # Infinity-Cache reuse across steps, which the one-bucket loop may enjoy)
    if not args.no_cold:
        x2 = (torch.randn(n, device=dev, generator=g) * 1e-3).to(tdt)
        y2, comp2 = torch.empty_like(y), torch.empty_like(comp)
        torch.cuda.synchronize()  # x2 was generated on the current stream
        calls2 = launches_for(x2.data_ptr(), y2.data_ptr(), comp2.data_ptr()) if launches_for else None
        if calls2 is not None:
            pairs = [calls, calls2]
            for k in range(4):
                for c in pairs[k % 2]:
                    c()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.steps):
                for c in pairs[k % 2]:
                    rc = c()
                    if rc:
                        raise RuntimeError(f"kernel launch failed: {N.STATUS.get(rc, rc)}")
            torch.cuda.synchronize()
            cms = (time.perf_counter() - t0) * 1e3 / args.steps
            extra["two_bucket_alternating"] = {"ms_per_step": round(cms, 4),
                                               "gib_s": round(esz * n / (cms * 1e-3) / GiB, 2)}
        del x2, y2, comp2
    cfg = {"workload": ("onebit_sign_scale" if onebit else "minmax_uint8") +
           f"_encode_decode_{esz * n >> 20}MiB_{args.dtype}_bucket", "bucket_elements": n, "n_chunks": p,
           "compressed_bytes": S, "config_index": 3 if onebit else 2}
    return value, ms, roof, cfg, extra, (x, comp)


def bench_host(args):
    """Host-resident rate: the bucket starts and ends in pinned
    host memory — H2D fp32 -> encode -> decode -> D2H fp32.  `serial` runs the
    four steps back to back per bucket; `overlapped` keeps two buckets in
    flight on three streams (H2D of bucket i+1 and D2H of bucket i-1 overlap
    the codec of bucket i), the steady state of a stream of buckets."""
    from bagua_core import _native as N
    K = N.K
    n = args.elements or (1 << 26)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator().manual_seed(0x5EED)
    src = (torch.randn(n, generator=g) * 1e-3).pin_memory()
    nb = max(2, args.host_buffers)
    dst = [torch.empty(n, pin_memory=True) for _ in range(nb)]
    x = [torch.empty(n, device=dev) for _ in range(nb)]
    y = [torch.empty(n, device=dev) for _ in range(nb)]
    S = K.bagua_minmax_u8_compressed_bytes(0, n, 1)
    wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
    comp = [torch.empty(S, dtype=torch.uint8, device=dev) for _ in range(nb)]
    ws = [torch.empty(wsb, dtype=torch.uint8, device=dev) for _ in range(nb)]
    s_in, s_cmp, s_out = (torch.cuda.Stream(device=dev) for _ in range(3))

    def codec(b, st):
        sp = ctypes.c_void_p(st.cuda_stream)
        N.check(K.bagua_minmax_u8_compress(0, x[b].data_ptr(), n, n, 1, comp[b].data_ptr(), S, ws[b].data_ptr(), wsb,
                                           -1, sp), "compress")
        N.check(K.bagua_minmax_u8_decompress(0, comp[b].data_ptr(), S, n, 1, y[b].data_ptr(), sp), "decompress")

    def serial(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            with torch.cuda.stream(s_cmp):
                x[0].copy_(src, non_blocking=True)
                codec(0, s_cmp)
                dst[0].copy_(y[0], non_blocking=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    ev_in = [torch.cuda.Event() for _ in range(nb)]
    ev_cmp = [torch.cuda.Event() for _ in range(nb)]
    ev_out = [torch.cuda.Event() for _ in range(nb)]

    chunks = max(1, args.copy_chunks)

    def h2d(b):
        # the copies go in `chunks` pieces: one 256 MiB H2D next to one D2H sometimes
        # does not overlap at all (9.4 ms for the pair vs 4.7 ms each), two pieces per
        # copy overlap every time (5.6 ms; tools/pcie_probe.py,
        # profiles/r02_host_copy_ab.jsonl)
        step = (n + chunks - 1) // chunks
        for lo in range(0, n, step):
            x[b][lo:lo + step].copy_(src[lo:lo + step], non_blocking=True)

    def d2h(b):
        step = (n + chunks - 1) // chunks
        for lo in range(0, n, step):
            dst[b][lo:lo + step].copy_(y[b][lo:lo + step], non_blocking=True)

    def overlapped(steps):
        torch.cuda.synchronize()
        for b in range(nb):  # start with every buffer free
            ev_cmp[b].record(s_cmp)
            ev_out[b].record(s_out)
        t0 = time.perf_counter()
        for i in range(steps):
            b = i % nb
            s_in.wait_event(ev_cmp[b])       # x[b] consumed by the codec of bucket i-2
            with torch.cuda.stream(s_in):
                h2d(b)
            ev_in[b].record(s_in)
            s_cmp.wait_event(ev_in[b])
            s_cmp.wait_event(ev_out[b])      # y[b] drained by the D2H of bucket i-2
            codec(b, s_cmp)
            ev_cmp[b].record(s_cmp)
            s_out.wait_event(ev_cmp[b])
            with torch.cuda.stream(s_out):
                d2h(b)
            ev_out[b].record(s_out)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    def copy_rate(to_dev: bool, steps: int):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s_in):
            for _ in range(steps):
                (x[0].copy_(src, non_blocking=True) if to_dev else dst[0].copy_(y[0], non_blocking=True))
        torch.cuda.synchronize()
        return 4.0 * n / ((time.perf_counter() - t0) / steps) / GiB

    serial(max(1, args.warmup))
    overlapped(max(2, args.warmup))
    t_ser = serial(args.steps)
    t_ovl = overlapped(args.steps)
    torch.cuda.synchronize()
    ok = torch.equal(dst[(args.steps - 1) % nb], y[(args.steps - 1) % nb].cpu())
    value = 4.0 * n / t_ovl / GiB
    cfg = {"workload": f"minmax_uint8_encode_decode_{4 * n >> 20}MiB_fp32_bucket_host_resident", "bucket_elements": n,
           "n_chunks": 1, "config_index": 2, "buffers": "pinned host fp32 in/out", "copy_pieces": chunks,
           "buckets_in_flight": nb}
    extra = {"serial_gib_s": round(4.0 * n / t_ser / GiB, 2), "serial_ms_per_bucket": round(t_ser * 1e3, 3),
             "overlapped_gib_s": round(value, 2), "h2d_gib_s": round(copy_rate(True, 5), 2),
             "d2h_gib_s": round(copy_rate(False, 5), 2), "result_copied_back_intact": bool(ok)}
    x[0].copy_(src)
    codec(0, torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    return value, t_ovl * 1e3, None, cfg, extra, (x[0], comp[0])


def cgroup_cpu_quota():
    """CPUs the cgroup lets this process use (cgroup v2 cpu.max "quota period", v1
    cfs_quota_us / cfs_period_us), or None when unlimited / unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_baseline_threads() -> tuple:
    """Threads the CPU baseline runs with: min(cgroup CPU quota, affinity, OMP_NUM_THREADS
    when the box sets one -- its stated CPU share), and the inputs of that choice."""
    quota = cgroup_cpu_quota()
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    omp_env = os.environ.get("OMP_NUM_THREADS")
    limits = [affinity]
    if quota is not None:
        limits.append(max(1, int(quota)))
    if omp_env and omp_env.strip().isdigit() and int(omp_env) > 0:
        limits.append(int(omp_env))
    return min(limits), {"cpu_quota": quota, "omp_num_threads_env": omp_env, "affinity_cpus": affinity}


def host_info() -> dict:
    """The host cores the CPU baseline ran on: the machine's CPU count, this
    process's affinity mask, the cgroup CPU quota, OMP_NUM_THREADS and the CPU model."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    threads, lim = cpu_baseline_threads()
    return {"os_cpu_count": os.cpu_count(), "affinity_cpus": lim["affinity_cpus"], "cpu_quota": lim["cpu_quota"],
            "omp_num_threads_env": lim["omp_num_threads_env"], "threads_rule": "min(cpu_quota, affinity, "
            "OMP_NUM_THREADS)", "threads_allowed": threads, "cpu_model": model}


def _oracle_threads(oracle_c) -> int:
    """the oracle's OpenMP team = the threads the host rules allow (cpu_baseline_threads)"""
    return oracle_c.set_num_threads(cpu_baseline_threads()[0])


def _cpu_timed(fn, budget_s: float, max_reps: int = 100000):
    fn()  # warm (page faults, OpenMP pool)
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= max_reps:
            return reps, el


def cpu_codec_baseline(args, xdev, comp_dev, onebit: bool = False):
    """The reference's algorithm (C restatement, oracle/bagua_oracle.c; the
    reference has no CPU path) on the host cores, on the SAME bucket
    the GPU encoded: encode+decode of x.cpu(), timed for about
    --cpu-seconds.  As a by-product the GPU's compressed bytes of that bucket
    are compared with the CPU's (`matches_gpu_bytes`)."""
    import numpy as np
    from oracle import oracle_c
    threads = _oracle_threads(oracle_c)
    dcode, npdt = {torch.float32: (0, np.float32), torch.float16: (1, np.float16),
                   torch.bfloat16: (2, np.uint16)}[xdev.dtype]
    x = (xdev.view(torch.int16) if xdev.dtype == torch.bfloat16 else xdev).cpu().numpy().view(npdt)
    out = np.empty_like(x)
    comp = oracle_c.compress_onebit(x, dcode, 1) if onebit else oracle_c.compress_minmax_u8(x, dcode, 1)
    same = bool(np.array_equal(comp, comp_dev.cpu().numpy())) if comp_dev is not None else None

    def step():
        if onebit:
            oracle_c.compress_onebit(x, dcode, 1, out=comp)
            oracle_c.decompress_onebit(comp, 1, out, dcode)
        else:
            oracle_c.compress_minmax_u8(x, dcode, 1, out=comp)
            oracle_c.decompress_minmax_u8(comp, 1, out, dcode)

    reps, el = _cpu_timed(step, args.cpu_seconds)
    # config 1: 4 MiB fp32, the whole centralized op sequence (compress -> alltoall ->
    # decompress -> reduce -> compress -> allgather -> decompress) at p = 1 on the CPU path
    from oracle import simulate
    rng = np.random.default_rng(0x5EED)
    x1 = [(rng.standard_normal(1 << 20) * 1e-3).astype(np.float32)]
    r1, e1 = _cpu_timed(lambda: simulate.centralized_low_precision(oracle_c, x1, 0, True), 1.0)
    codec = "1-bit sign+scale" if onebit else "MinMax-UInt8"
    return {"value": round(x.nbytes * reps / el / GiB, 3), "unit": "GiB/s", "cores": threads,
            "kind": "port", "host": host_info(), "matches_gpu_bytes": same,
            "config1_loopback_op_gib_s": round(4.0 * (1 << 20) * r1 / e1 / GiB, 3),
            "sample": f"the same {x.nbytes >> 20} MiB bucket the GPU encoded (x.cpu()), {codec} encode+decode "
                      f"x{reps} ({el:.1f} s wall, {threads} OpenMP threads, oracle/bagua_oracle.c)"}


def cpu_allreduce_baseline(args, world: int, n: int, dev, sample_elems: int = 1 << 22):
    """The compressed centralized all-reduce (centralized_low_precision_synchronous.rs:30-71)
    on the host cores: oracle/simulate.py composes the C restatement in the
    reference's op order for all `world` ranks (collectives = array moves).
    Inputs: the first `sample_elems` elements of every rank's own bucket
    (torch.randn, seed 0x5EED + r, regenerated here), a bounded sample of the
    same workload.  value = gradient bytes of all ranks / wall time."""
    import numpy as np
    from oracle import oracle_c, simulate
    threads = _oracle_threads(oracle_c)
    m = min(n, sample_elems)
    m -= m % world
    xs = []
    for r in range(world):
        g = torch.Generator(device=dev).manual_seed(0x5EED + r)
        xs.append((torch.randn(n, device=dev, generator=g) * 1e-3)[:m].cpu().numpy())
    torch.cuda.empty_cache()
    reps, el = _cpu_timed(lambda: simulate.centralized_low_precision(oracle_c, xs, 0, True),
                          args.cpu_seconds, max_reps=10000)
    return {"value": round(world * 4.0 * m * reps / el / GiB, 3), "unit": "GiB/s", "cores": threads,
            "kind": "port", "host": host_info(),
            "sample": f"{world} ranks x the first {4 * m >> 20} MiB of each rank's fp32 bucket (seed 0x5EED + r), "
                      f"the whole MinMax-UInt8 op sequence for all ranks x{reps} ({el:.1f} s wall, {threads} OpenMP "
                      "threads, oracle/simulate.py over oracle/bagua_oracle.c; rank 0 after the timed region)"}


# algorithmic bytes per launch of the op's kernels at one rank (SURVEY §8(d) counting;
# n elements of fp32, p = 1): DESIGN.md §6
def _op_kernel_alg_bytes(name: str, n: int):
    return {"minmax_resident_encode_kernel": 9 * n + 32, "minmax_partials_kernel": 4 * n,
            "minmax_quantize_kernel": 5 * n + 32,
            "dequant_reduce_kernel": n + 32,            # partials-only pass: the received payload
            "dequant_reduce_quantize_kernel": 5 * n + 32,  # payload read + final values written (no segment)
            "minmax_dequantize_kernel": 5 * n + 32,
            "minmax_one_rank_kernel": 8 * n}.get(name)  # the one-rank op's table pass: x read, result written


def allreduce_p1(args, n: int = 1 << 28):
    """Config 4 at one rank, beside the N = 1 codec headline: the same workload the N > 1
    lines time (1 GiB fp32, the compressed centralized op,
    centralized_low_precision_synchronous.rs:16-73, p = 1), the fp32 all-reduce of the same
    bucket, and every kernel of the op timed by the kernel library's own events
    (bagua_time_next_kernels), so the driver's 1 -> 8 GPU curve has a same-workload N = 1
    point.  Steps and warmup as the headline's."""
    from bagua_core import BaguaSingleCommunicatorPy, BaguaTensorPy
    from bagua_core import _native as N
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.Stream(device=dev)
    comm = BaguaSingleCommunicatorPy(0, 1, 0, stream.cuda_stream,
                                     BaguaSingleCommunicatorPy.generate_nccl_unique_id_str())
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    torch.cuda.synchronize()
    raw = BaguaTensorPy(x, "gradient_bucket").raw()

    def op():
        N.check(N.C.bagua_centralized_low_precision_pipelined(comm.handle, ctypes.byref(raw), 1,
                                                              N.COMPRESSION_MINMAX_UINT8, 0), "compressed allreduce")

    def fp32():
        N.check(N.C.bagua_centralized_full_precision_synchronous(comm.handle, ctypes.byref(raw), 1), "fp32 allreduce")

    def onebit():  # the same op with the 1-bit codec (at one rank: bagua_onebit_centralized_one_rank)
        N.check(N.C.bagua_centralized_low_precision_pipelined(comm.handle, ctypes.byref(raw), 1,
                                                              N.COMPRESSION_ONEBIT, 0), "1-bit allreduce")

    def timed(fn, steps, warm):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    t_op = timed(op, args.steps, args.warmup)
    t_f = timed(fp32, max(3, args.steps // 2), max(1, args.warmup // 2))
    t_ob = timed(onebit, max(3, args.steps // 2), max(1, args.warmup // 2))
    # config 5 at one rank: 2^27 bf16, the decentralized ring op
    # (decentralized_low_precision_synchronous.rs:42-152; at one rank its own left and right
    # peer: bagua_ring_one_rank_minmax, two passes)
    nb = 1 << 27
    ring = [(torch.randn(nb, device=dev, generator=g) * 1e-3).to(torch.bfloat16) for _ in range(4)]
    rraws = [BaguaTensorPy(b, k).raw() for b, k in zip(ring, "twlr")]

    def ring_op():
        N.check(N.C.bagua_decentralized_low_precision_synchronous(comm.handle, *[ctypes.byref(r) for r in rraws],
                                                                  N.COMPRESSION_MINMAX_UINT8), "ring op")
    t_ring = timed(ring_op, max(3, args.steps // 2), max(1, args.warmup // 2))
    del ring, rraws
    # every kernel of the op, a few times (the op syncs its stream before returning)
    reps, per, names = 5, {}, []
    for _ in range(reps):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(8)]
        for a, b in ev:
            a.record(stream)
            b.record(stream)
        N.time_next_kernels(ev)
        op()
        names = N.timed_kernel_names()
        N.check(N.K.bagua_time_next_kernels(None, None, 0), "disarm")
        torch.cuda.synchronize()
        for i, nm in enumerate(names):
            per.setdefault(f"{i}:{nm}", []).append(ev[i][0].elapsed_time(ev[i][1]))
    kern = {k: sum(v) / len(v) * 1e3 for k, v in per.items()}  # us
    dom = max(kern, key=kern.get)
    dname = dom.split(":", 1)[1]
    alg = _op_kernel_alg_bytes(dname, n)
    roof = None
    if alg:
        ach = alg / (kern[dom] * 1e-6) / 1e9
        roof = {"bound": "hbm", "kernel": dname, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": alg,
                "avg_launch_us": round(kern[dom], 2)}
    res = {"config_index": 4, "workload": f"minmax_uint8_compressed_allreduce_{4 * n >> 20}MiB_fp32_per_rank",
           "n_ranks": 1, "ms_per_step": round(t_op * 1e3, 4), "gib_s": round(4.0 * n / t_op / GiB, 2),
           "fp32_allreduce_ms_per_step": round(t_f * 1e3, 4), "fp32_allreduce_gib_s": round(4.0 * n / t_f / GiB, 2),
           "ratio_vs_fp32": round(t_f / t_op, 3),
           "onebit_ms_per_step": round(t_ob * 1e3, 4), "onebit_gib_s": round(4.0 * n / t_ob / GiB, 2),
           "ring_bf16_config5_ms_per_step": round(t_ring * 1e3, 4),
           "ring_bf16_config5_gib_s": round(2.0 * nb / t_ring / GiB, 2),
           "op_kernels_us": {k: round(v, 2) for k, v in kern.items()}, "roofline": roof,
           "note": "the N > 1 lines' workload (--workload allreduce) at one rank; kernel times are the "
                   "kernels' own HIP events inside the op (bagua_time_next_kernels)",
           "ratio_note": "at one rank RCCL's fp32 all-reduce is its single-rank reduce-copy (oneRankReduce, "
                         "~0.19 of HBM peak): ratio_vs_fp32 here is not the multi-GPU ratio the >= 6x target "
                         "is about"}
    del comm, x
    torch.cuda.empty_cache()
    return res


# ----------------------------------------------------------------- N > 1 ------
def bench_allreduce(args, world: int, rank: int, local_rank: int):
    PHASES.lap("startup")  # interpreter, torch import, argument parsing
    import torch.distributed as dist
    from bagua_core import BaguaSingleCommunicatorPy, BaguaTensorPy
    from bagua_core import _native as N
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("gloo", rank=rank, world_size=world)
    comm_stream = torch.cuda.Stream(device=dev)

    def make_comm():
        # communicators/mod.rs:25-60: rank 0's base64 ncclUniqueId, shared over gloo
        uid = [BaguaSingleCommunicatorPy.generate_nccl_unique_id_str() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        return BaguaSingleCommunicatorPy(rank, world, local_rank, comm_stream.cuda_stream, uid[0])

    comm = make_comm()
    n = args.elements or (1 << 28)
    n -= n % world
    g = torch.Generator(device=dev).manual_seed(0x5EED + rank)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    torch.cuda.synchronize()
    raw = BaguaTensorPy(x, "gradient_bucket").raw()
    PHASES.lap("setup")  # process group, RCCL communicator, 1 GiB bucket

    headline_taper = [False]  # the autotune may pick tapered pieces (N.PIECES_TAPERED) for the headline

    def compressed_step(pieces=None, taper=None):
        # a tapered schedule goes in the op's `pieces` argument (N.PIECES_TAPERED): the
        # process environment is never changed while ops run
        taper = headline_taper[0] if (taper is None and pieces is None) else bool(taper)
        q = args.pieces if pieces is None else pieces
        N.check(N.C.bagua_centralized_low_precision_pipelined(comm.handle, ctypes.byref(raw), 1,
                                                              N.COMPRESSION_MINMAX_UINT8,
                                                              q | (N.PIECES_TAPERED if taper else 0)),
                "compressed allreduce")

    def fp32_step():
        N.check(N.C.bagua_centralized_full_precision_synchronous(comm.handle, ctypes.byref(raw), 1), "fp32 allreduce")

    def barrier():
        if world > 1:
            dist.barrier()

    def timed(fn, steps, warm):
        for _ in range(warm):
            fn()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()) / steps

    side_errors = {}
    skipped = []  # side lines not started because the line's wall budget was spent
    sized_steps = {}  # side lines timed over fewer steps than usual to fit the budget

    def remaining_s() -> float:
        # the line's wall budget left, the same on every rank (min over ranks, gloo), so
        # every rank skips the same side lines
        left = torch.tensor([args.budget_s - (time.perf_counter() - _PROCESS_T0)], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(left, op=dist.ReduceOp.MIN)
        return float(left.item())

    def side(name, fn, required=False):
        # side measurements must not cost the headline line: an error that every rank
        # raises alike (argument checks, an unsupported shape) is recorded instead, and a
        # measurement that has not finished after its limit aborts the communicator
        # (ncclCommAbort: pending collectives return) so the line is still printed; the
        # ranks then agree (gloo) to rebuild it, so the later side lines still measure.
        # The limit is SIDE_TIMEOUT_S or what is left of --budget-s, whichever is less; a
        # line that is not `required` is skipped (skipped_for_budget) once less than
        # MIN_SIDE_S is left.
        nonlocal comm
        expired = []
        left = remaining_s()
        if side_skipped(left, required):
            skipped.append(name)
            return float("nan")

        # test hook (BAGUA_BENCH_FAIL_SIDE=<side line>): that line's limit is 0 s, so its
        # communicator is aborted at once and the recovery below runs
        limit = side_limit_s(left, required)
        if os.environ.get("BAGUA_BENCH_FAIL_SIDE") == name:
            limit = 0.0

        def expire():
            expired.append(True)
            side_errors[name] = f"timed out after {limit:.0f} s; communicator aborted and rebuilt"
            comm.abort()

        timer = threading.Timer(limit, expire)
        timer.daemon = True
        timer.start()
        res = float("nan")
        try:
            for _ in range(max(1, args.warmup // 2)):
                fn()
            # one timed call sizes the line: as many steps as fit in a fifth of what is left
            # (t1 is the max over ranks and `left` the min, so every rank runs the same count)
            nominal = max(3, args.steps // 2)
            t1 = timed(fn, 1, 0)
            steps = side_steps(left, t1, nominal)
            if steps < nominal:
                sized_steps[name] = steps
            res = timed(fn, steps, 0)
        except Exception as e:  # noqa: BLE001
            side_errors.setdefault(name, str(e)[:200])
        finally:
            timer.cancel()
        spend = os.environ.get("BAGUA_BENCH_SPEND", "")  # test hook "<side line>:<s>": that line takes s longer
        if spend.partition(":")[0] == name:
            time.sleep(float(spend.partition(":")[2] or 0))
        flag = torch.tensor([1.0 if expired else 0.0])
        if world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if flag.item():
            if not expired:
                comm.abort()  # another rank's timer fired: every rank leaves the old communicator
            comm = make_comm()
            return float("nan")
        return res

    def budget_allows(name) -> bool:
        """a block of side lines with set-up of its own starts only with MIN_SIDE_S left"""
        if remaining_s() >= MIN_SIDE_S:
            return True
        skipped.append(name)
        return False

    # The headline: the pipelined op.  Its multi-group RCCL schedule has run over the
    # loopback transport, gloo and single-rank RCCL only; should it not
    # finish on this node within its limit (HEADLINE_TIMEOUT_S, at most half the line's
    # budget), the communicator is aborted and the headline falls back to the unpieced
    # op (the reference's one alltoall + one allgather) on a fresh communicator,
    # recorded in headline_fallback.
    headline_fallback = None
    aborted = []
    autotune = {}  # pieces -> s per step during the untimed choice (N > 1, --pieces 0)
    user_pieces = args.pieces  # the other ops keep the library's own choice unless --pieces is given

    def expire_headline():
        aborted.append(True)
        comm.abort()

    timer = threading.Timer(max(30.0, min(HEADLINE_TIMEOUT_S, 0.5 * args.budget_s)), expire_headline)
    timer.daemon = True
    timer.start()
    try:
        if os.environ.get("BAGUA_BENCH_FAIL_HEADLINE"):  # test hook: exercise the fallback below
            comm.abort()
        if world > 1 and args.pieces == 0:
            # runtime piece-count choice for this node (part of the warmup, untimed): a few
            # steps at each count, the fastest max-over-ranks time wins on every rank alike
            for q in (1, 2, 4, 8, 16):
                autotune[str(q)] = timed(lambda q=q: compressed_step(q), 2, 1)
            for q in (4, 8):  # first and last piece half size: shorter prefix and suffix
                autotune[f"{q}_tapered"] = timed(lambda q=q: compressed_step(q, taper=True), 2, 1)
            best = min(autotune, key=lambda q: autotune[q])
            args.pieces = int(best.split("_")[0])
            headline_taper[0] = best.endswith("_tapered")
            PHASES.lap("autotune")
        t_c = timed(compressed_step, args.steps, args.warmup)
        err = "timed out; communicator aborted" if aborted else None
    except Exception as e:  # noqa: BLE001 - an op error on every rank alike
        err = str(e)[:200]
    finally:
        timer.cancel()
    if world > 1:  # every rank takes the same branch (gloo all-reduce of the failure flag)
        flag = torch.tensor([1.0 if err else 0.0])
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if flag.item() and not err:
            err = "another rank failed"
    if err:
        if world == 1 and not os.environ.get("BAGUA_BENCH_FAIL_HEADLINE"):
            raise RuntimeError(f"compressed all-reduce failed: {err}")
        headline_fallback = {"pipelined_error": err, "headline": "unpieced op (pieces = 1)"}
        comm = make_comm()
        args.pieces = 1
        t_c = timed(lambda: compressed_step(1), args.steps, args.warmup)
    PHASES.lap("headline")
    # What the north star compares the headline with, measured right after it (never
    # skipped for the budget): the uncompressed fp32 RCCL all-reduce of the same bucket,
    # and the op's two collectives alone on its compressed bytes (RCCL alltoall of S
    # bytes, in-place allgather of S bytes), so the codec time the op did not hide is
    # ms_per_step - comm_only_ms
    t_f = side("fp32_allreduce", fp32_step, required=True)
    PHASES.lap("fp32_allreduce")
    S_c = N.K.bagua_minmax_u8_compressed_bytes(0, n // world, world)
    cbuf = [torch.zeros(S_c, dtype=torch.uint8, device=dev) for _ in range(2)]
    craw = [N.bagua_tensor_t(b.data_ptr(), S_c, S_c, 3, local_rank) for b in cbuf]

    def comm_only():
        N.check(N.C.bagua_comm_alltoall(comm.handle, ctypes.byref(craw[0]), ctypes.byref(craw[1])), "alltoall")
        N.check(N.C.bagua_comm_allgather_inplace(comm.handle, ctypes.byref(craw[1])), "allgather")
        N.check(N.C.bagua_comm_synchronize(comm.handle), "sync")

    t_comm = side("comm_only", comm_only, required=True)
    del cbuf, craw
    PHASES.lap("comm_only")
    # the same all-reduce with the 1-bit sign+scale codec (this repo's extension:
    # N/8 wire bytes per phase instead of N), fused middle step
    def onebit_step(pieces=user_pieces):
        N.check(N.C.bagua_centralized_low_precision_pipelined(comm.handle, ctypes.byref(raw), 1,
                                                              N.COMPRESSION_ONEBIT, pieces), "1-bit allreduce")

    t_o = side("onebit", onebit_step)
    PHASES.lap("onebit")
    t_u = side("unpieced", lambda: compressed_step(1))
    PHASES.lap("unpieced")
    # Bagua's default bucket size (25 MiB of fp32): the same op and the fp32 all-reduce on the
    # first 25 MiB of the bucket, where latency, not bandwidth, sets the step
    m = min(n, (25 << 20) // 4)
    m -= m % (4 * 32 * world)
    small = BaguaTensorPy(x[:m], "bucket_25mib").raw()
    t_s = side("bucket_25mib", lambda: N.check(N.C.bagua_centralized_low_precision_pipelined(
        comm.handle, ctypes.byref(small), 1, N.COMPRESSION_MINMAX_UINT8, user_pieces), "25 MiB op"))
    t_sf = side("bucket_25mib_fp32", lambda: N.check(N.C.bagua_centralized_full_precision_synchronous(
        comm.handle, ctypes.byref(small), 1), "25 MiB fp32 allreduce"))
    PHASES.lap("bucket_25mib")
    decentralized = None
    if not args.no_decentralized and budget_allows("decentralized"):
        # config 5: bf16 bucket, decentralized ring exchange with the uint8 codec
        # (decentralized_low_precision_synchronous.rs:42-152), 2^27 elements per rank
        try:
            nb = args.elements or (1 << 27)  # config 5: 2^27 bf16 (256 MiB) per rank
            bufs = [(torch.randn(nb, device=dev, generator=g) * 1e-3).to(torch.bfloat16) for _ in range(4)]
            draws = [BaguaTensorPy(b, k).raw() for b, k in zip(bufs, "twlr")]

            def dec_step(pieces=user_pieces, multipath=False):
                # the opt-in relayed exchange (comm_ops.cpp ring_ops: 3/p of each piece direct, the
                # rest through the other ranks) goes in the op's `pieces` argument; the default is
                # the reference's direct exchange
                N.check(N.C.bagua_decentralized_low_precision_pipelined(
                    comm.handle, *[ctypes.byref(r) for r in draws], N.COMPRESSION_MINMAX_UINT8,
                    pieces | (N.PIECES_MULTIPATH if multipath else 0)), "decentralized")

            multipath = world >= 6  # comm_ops.cpp kRingMinMultipath
            t_d = side("decentralized", dec_step)
            t_du = side("decentralized_unpieced", lambda: dec_step(1))
            t_dm = side("decentralized_multipath", lambda: dec_step(multipath=True)) if multipath else float("nan")
            decentralized = {"config_index": 5, "elements_per_rank": nb, "dtype": "bf16",
                             "exchange": "direct (the reference's; multipath is opt-in)",
                             "ms_per_step": round(t_d * 1e3, 3), "unpieced_ms_per_step": round(t_du * 1e3, 3),
                             "multipath_exchange_ms_per_step": round(t_dm * 1e3, 3) if multipath else None,
                             "gib_s_per_rank": round(2.0 * nb / t_d / GiB, 2),
                             "gib_s_total": round(world * 2.0 * nb / t_d / GiB, 2)}
            del bufs, draws
        except Exception as e:  # noqa: BLE001 - a failed side measurement must not lose the headline line
            decentralized = {"error": str(e)[:200]}
        PHASES.lap("decentralized_bf16")
    t_ou = side("onebit_unpieced", lambda: onebit_step(1))
    PHASES.lap("onebit_unpieced")
    # the scheduler workload (32 x 25 MiB buckets, Bagua's default bucket size) through the native
    # scheduler on this communicator: cross-bucket lanes (the library default, 3) and one lane;
    # the faster of the two on this node is recorded as lanes_chosen (the library
    # default stays 3 only while a node line shows lanes paying at p > 1)
    sched = {}
    nbk, mib = (32, 25) if not args.elements else (8, max(1, (4 * n >> 20) // 8))  # --elements: a rehearsal
    if world > 1 and budget_allows("scheduler_buckets"):
        try:
            wl = SchedulerWorkload(comm, world, rank, local_rank, nbk, mib)
            sched["buckets"], sched["bucket_mib"] = nbk, mib
            for ln in (wl.backend.lanes(), 1):
                if wl.comm is not comm:  # a timed-out side line rebuilt the communicator
                    wl.close()
                    wl = SchedulerWorkload(comm, world, rank, local_rank, nbk, mib)
                wl.backend.set_lanes(ln)
                t_sc = side(f"scheduler_lanes{ln}", wl.iteration)
                if math.isfinite(t_sc):
                    sched[f"lanes_{ln}"] = {"ms_per_step": round(t_sc * 1e3, 4),
                                            "per_bucket_us": round(t_sc * 1e6 / nbk, 2),
                                            "gib_s_total": round(world * 4.0 * wl.per * nbk / t_sc / GiB, 2)}
            timed_lanes = {int(k[6:]): v["ms_per_step"] for k, v in sched.items() if k.startswith("lanes_")}
            if timed_lanes:
                sched["lanes_chosen"] = min(timed_lanes, key=timed_lanes.get)
            wl.close()
            del wl
        except Exception as e:  # noqa: BLE001 - a failed side measurement must not lose the headline line
            side_errors.setdefault("scheduler", str(e)[:200])
        PHASES.lap("scheduler_buckets")
    # piece counts either side of the automatic choice (the autotune already timed them
    # briefly), so the node's own run says which count hides the codec best behind its links
    sweep = {}
    if world > 1 and not headline_fallback:
        for q in (2, 8):
            sweep[str(q)] = side(f"pieces_{q}", lambda q=q: compressed_step(q))

        def tapered(q):
            # first and last piece half size (N.PIECES_TAPERED, minmax_u8.hip piece_range)
            compressed_step(q, taper=True)

        for q in (4, 5):
            sweep[f"{q}_tapered"] = side(f"pieces_{q}_tapered", lambda q=q: tapered(q))
        sweep = {q: v for q, v in sweep.items() if math.isfinite(v)}
        PHASES.lap("pieces_sweep")
    value = world * 4.0 * n / t_c / GiB
    per_rank = 4.0 * n / t_c / GiB
    fp32 = 4.0 * n / t_f / GiB
    # roofline of the dominant codec kernel on this bucket (p = world chunks), HIP events on its stream
    K = N.K
    S = K.bagua_minmax_u8_compressed_bytes(0, n // world, world)
    comp = torch.empty(S, dtype=torch.uint8, device=dev)
    wsb = K.bagua_minmax_u8_workspace_bytes(n // world, world)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    y = torch.empty_like(x)
    calls = [lambda: K.bagua_minmax_u8_compress_stage(1, 0, x.data_ptr(), n, n // world, world, comp.data_ptr(), S,
                                                       ws.data_ptr(), wsb, -1, sp),
             lambda: K.bagua_minmax_u8_compress_stage(2, 0, x.data_ptr(), n, n // world, world, comp.data_ptr(), S,
                                                       ws.data_ptr(), wsb, -1, sp),
             lambda: K.bagua_minmax_u8_decompress(0, comp.data_ptr(), S, n // world, world, y.data_ptr(), sp)]
    names = ["minmax_partials_kernel", "minmax_quantize_kernel", "minmax_dequantize_kernel"]
    alg = [4 * n, 5 * n + 32 * world, 5 * n + 32 * world]
    reps = 5
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
          for _ in range(reps)]
    for row in ev:  # torch creates the HIP events on first record
        for a, b in row:
            a.record(st)
            b.record(st)
    for c in calls:
        c()
    for k in range(reps):
        for i, c in enumerate(calls):  # kernel-recorded start/stop events (hipExtLaunchKernel)
            N.check(K.bagua_time_next_kernel(ev[k][i][0].cuda_event, ev[k][i][1].cuda_event), "timing hook")
            c()
    torch.cuda.synchronize()
    per = [sum(ev[k][i][0].elapsed_time(ev[k][i][1]) for k in range(reps)) / reps for i in range(3)]
    dom = max(range(3), key=lambda i: per[i])
    achieved = alg[dom] / (per[dom] * 1e-3) / 1e9
    roof = {"bound": "hbm", "kernel": names[dom], "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            # the committed PMC pass is of the 256 MiB codec launch; at this size: unmeasured
            "traffic": pmc_traffic(names[dom]) if n == (1 << 26) and world == 1 else None,
            "alg_bytes_per_launch": alg[dom], "avg_launch_us": round(per[dom] * 1e3, 2)}
    PHASES.lap("roofline")
    cfg = {"workload": f"minmax_uint8_compressed_allreduce_{4 * n >> 20}MiB_fp32_per_rank", "bucket_elements": n,
           "n_chunks": world, "collectives": "rccl alltoall + allgather (uint8)", "parallelism": f"dp{world}",
           "config_index": 4}
    extra = {"per_rank_gib_s": round(per_rank, 2), "fp32_allreduce_gib_s": round(fp32, 2),
             "ratio_vs_fp32": round(per_rank / fp32, 3), "fp32_ms_per_step": round(t_f * 1e3, 3),
             "pieces": args.pieces or "auto",
             "pieces_tapered": headline_taper[0],
             "pieces_autotune_ms_per_step": {q: round(v * 1e3, 3) for q, v in autotune.items()} or None,
             "unpieced_ms_per_step": round(t_u * 1e3, 3),
             "pieces_sweep_ms_per_step": {q: round(v * 1e3, 3) for q, v in sweep.items()} or None,
             "comm_only_ms": round(t_comm * 1e3, 3),
             "comm_only_note": "RCCL alltoall + in-place allgather of the op's S compressed bytes, nothing else",
             "bucket_25mib": {"elements_per_rank": m, "ms_per_step": round(t_s * 1e3, 4),
                              "fp32_ms_per_step": round(t_sf * 1e3, 4),
                              "gib_s_total": round(world * 4.0 * m / t_s / GiB, 2),
                              "ratio_vs_fp32": round(t_sf / t_s, 3)},
             "decentralized_bf16": decentralized,
             "scheduler_buckets": sched or None,
             "onebit_allreduce": {"ms_per_step": round(t_o * 1e3, 3), "unpieced_ms_per_step": round(t_ou * 1e3, 3),
                                  "per_rank_gib_s": round(4.0 * n / t_o / GiB, 2),
                                  "ratio_vs_fp32": round((4.0 * n / t_o) / (4.0 * n / t_f), 3)},
             "per_kernel_us": {nm: round(t * 1e3, 2) for nm, t in zip(names, per)}}
    if side_errors:
        extra["side_errors"] = side_errors
    extra["budget_s"] = args.budget_s
    extra["skipped_for_budget"] = skipped
    if sized_steps:
        extra["side_steps_for_budget"] = sized_steps
    if headline_fallback:
        extra["headline_fallback"] = headline_fallback
    del comm
    return value, t_c * 1e3, roof, cfg, extra


class SchedulerWorkload:
    """The scheduler (BaguaCommBackendPy, bagua-core-internal/src/lib.rs:176-338) driving a
    model-sized gradient: `buckets` buckets of `bucket_mib` MiB fp32 (4 tensors each,
    contiguous), each with the compressed centralized op on `comm`.  One iteration =
    every tensor marked ready in reverse bucket order (as backward produces them, each
    bucket with a ready event) + wait_pending_comm_ops."""

    def __init__(self, comm, world: int, rank: int, local_rank: int, buckets: int, bucket_mib: int):
        import bagua_core
        dev = torch.device("cuda", local_rank)
        self.comm, self.world, self.nb = comm, world, buckets
        per = (bucket_mib << 20) // 4
        per -= per % (4 * 32 * world)
        self.per = per
        g = torch.Generator(device=dev).manual_seed(0x5EED + rank)
        self.flats = [torch.randn(per, device=dev, generator=g) * 1e-3 for _ in range(buckets)]
        self.buckets, self.tensors = [], []
        for b, flat in enumerate(self.flats):
            ts = [bagua_core.BaguaTensorPy(v, f"b{b}.t{i}") for i, v in enumerate(flat.view(4, -1).unbind(0))]
            bk = bagua_core.BaguaBucketPy(f"bucket{b}", ts)
            bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
            self.buckets.append(bk)
            self.tensors.append(ts)
        self.backend = bagua_core.BaguaCommBackendPy(buckets, local_rank)
        # backward produces the last layers' gradients first: the registration order is the
        # order buckets become ready
        self.backend.register_ordered_buckets(list(reversed(self.buckets)))
        self.events = [torch.cuda.Event() for _ in range(buckets)]
        # where backward's ready events are recorded: the current (default) stream, as a
        # training loop does, or a stream of their own (BAGUA_BENCH_READY_STREAM=own, A/B)
        self.ready_mode = os.environ.get("BAGUA_BENCH_READY_STREAM", "default")  # default / own / none
        self.ready_stream = torch.cuda.Stream(device=dev) if self.ready_mode == "own" else None
        self.mark_s = []
        torch.cuda.synchronize()

    def iteration(self):
        t0 = time.perf_counter()
        for b in reversed(range(self.nb)):
            if self.ready_mode != "none":
                self.events[b].record(self.ready_stream)
            ev = self.events[b].cuda_event if self.ready_mode != "none" else 0
            for t in self.tensors[b]:
                self.backend.mark_communication_ready(t, ev)
        self.mark_s.append(time.perf_counter() - t0)
        done = self.backend.wait_pending_comm_ops()
        assert done == self.nb, done

    def time(self, steps: int, warmup: int, lanes: int, barrier=None) -> float:
        """ms per iteration (max over ranks when `barrier` reduces)"""
        self.backend.set_lanes(lanes)
        for _ in range(max(1, warmup)):
            self.iteration()
        torch.cuda.synchronize()
        if barrier:
            barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.iteration()
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        if self.world > 1:
            import torch.distributed as dist
            tt = torch.tensor([t], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
        return t / steps * 1e3

    def close(self):
        del self.backend, self.buckets


def bench_backend(args, world: int, rank: int, local_rank: int):
    """The scheduler workload (SchedulerWorkload): `--buckets` x `--bucket-mib` MiB fp32
    buckets through the native scheduler, with cross-bucket lanes (backend.cpp; the
    default 3) and, beside it, one lane (every bucket on the communicator's stream).
    value = GiB of gradient per second (all ranks)."""
    import torch.distributed as dist
    import bagua_core
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("gloo", rank=rank, world_size=world)
    uid = [bagua_core.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0)
    comm_stream = torch.cuda.Stream(device=dev)
    comm = bagua_core.BaguaSingleCommunicatorPy(rank, world, local_rank, comm_stream.cuda_stream, uid[0])
    wl = SchedulerWorkload(comm, world, rank, local_rank, args.buckets, args.bucket_mib)
    barrier = (lambda: dist.barrier()) if world > 1 else None
    lanes = args.lanes or wl.backend.lanes()
    # one lane first, the configured lanes last (a kernel trace's tail is the headline's)
    ms1 = wl.time(args.steps, args.warmup, 1, barrier) if lanes != 1 else None
    wl.mark_s.clear()
    ms = wl.time(args.steps, args.warmup, lanes, barrier)
    mark = sorted(wl.mark_s)[len(wl.mark_s) // 2]
    ms1 = ms if ms1 is None else ms1
    grad_bytes = 4.0 * wl.per * args.buckets
    value = world * grad_bytes / (ms * 1e-3) / GiB
    cfg = {"workload": f"comm_backend_{args.buckets}x{args.bucket_mib}MiB_fp32_buckets_minmax_uint8",
           "bucket_elements": wl.per, "buckets": args.buckets, "tensors_per_bucket": 4,
           "parallelism": f"dp{world}", "scheduler": "bagua_core.backend.BaguaCommBackendPy", "lanes": lanes}
    extra = {"per_bucket_us": round(ms * 1e3 / args.buckets, 2), "per_rank_gib_s": round(value / world, 2),
             # host time of the Python side per bucket (a ready event + one mark per tensor): the
             # scheduler cannot run a bucket before its last tensor is marked
             "mark_us_per_bucket": round(mark * 1e6 / args.buckets, 2),
             "one_lane": {"ms_per_step": round(ms1, 4), "per_bucket_us": round(ms1 * 1e3 / args.buckets, 2),
                          "gib_s_total": round(world * grad_bytes / (ms1 * 1e-3) / GiB, 2)}}
    wl.close()
    del comm
    return value, ms, None, cfg, extra


def _finite(o):
    """NaN / inf (a failed side measurement) -> null: the line stays strict JSON."""
    if isinstance(o, float):
        return o if math.isfinite(o) else None
    if isinstance(o, dict):
        return {k: _finite(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_finite(v) for v in o]
    return o


def main():
    # Native libraries (RCCL's version banner) write to fd 1; the contract is ONE
    # JSON line on stdout, so everything else goes to stderr.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    args = parse()
    if args.two_pass:
        os.environ["BAGUA_RESIDENT"] = "0"  # read by the kernel library on every compress call
    world = int(os.environ.get("WORLD_SIZE", args.gpus))
    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    workload = args.workload
    if workload == "auto":
        workload = "codec" if world == 1 else "allreduce"
    cpu = None
    if workload in ("codec", "onebit"):
        value, ms, roof, cfg, extra, (xb, cb) = bench_codec(args, onebit=(workload == "onebit"))
        if rank == 0 and not args.no_cpu_baseline:
            try:
                cpu = cpu_codec_baseline(args, xb, cb, onebit=(workload == "onebit"))
            except Exception as e:  # noqa: BLE001 - a failed baseline must not lose the headline line
                cpu = {"error": str(e)[:200]}
        del xb, cb
        if args.workload == "auto" and world == 1 and not args.no_allreduce_p1 and not args.elements:
            # the default line: config 2 (headline) + config 4 at one rank (the 1 -> 8 GPU curve's N = 1 point)
            try:
                extra["allreduce_p1"] = allreduce_p1(args)
            except Exception as e:  # noqa: BLE001 - a failed side measurement must not lose the headline line
                extra["allreduce_p1"] = {"error": str(e)[:200]}
        dtype = f"{args.dtype} -> u8" if workload == "codec" else f"{args.dtype} -> 1bit"
    elif workload == "host":
        value, ms, roof, cfg, extra, (xb, cb) = bench_host(args)
        if rank == 0 and not args.no_cpu_baseline:
            try:
                cpu = cpu_codec_baseline(args, xb, cb)
            except Exception as e:  # noqa: BLE001 - a failed baseline must not lose the headline line
                cpu = {"error": str(e)[:200]}
        del xb, cb
        dtype = "f32 -> u8"
    else:
        if workload == "backend":
            value, ms, roof, cfg, extra = bench_backend(args, world, rank, local_rank)
            n_cpu = cfg["bucket_elements"]
        else:
            value, ms, roof, cfg, extra = bench_allreduce(args, world, rank, local_rank)
            n_cpu = cfg["bucket_elements"]
        # after every rank's timed region: rank 0 times the op on the host cores while
        # the others wait at the closing barrier
        if rank == 0 and not args.no_cpu_baseline:
            if workload == "allreduce" and world > 1:  # inside the line's wall budget too
                left = args.budget_s - (time.perf_counter() - _PROCESS_T0)
                args.cpu_seconds = max(0.5, min(args.cpu_seconds, left - 10.0))
            try:
                cpu = cpu_allreduce_baseline(args, world, n_cpu, torch.device("cuda", local_rank))
            except Exception as e:  # noqa: BLE001 - a failed baseline must not lose the headline line
                cpu = {"error": str(e)[:200]}
            PHASES.lap("cpu_baseline")
        if workload == "allreduce":
            extra["phase_wall_s"] = PHASES.report()
        dtype = "f32 -> u8"
    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": dtype,
                "data": "synthetic fp32 gradients N(0, 1e-3^2) (torch.randn, seed 0x5EED + rank), " +
                        ("in pinned host memory (H2D + D2H timed)" if workload == "host" else "resident in HBM"),
                "config": cfg, "roofline": roof, "cpu_baseline": cpu,
                "hw_queues": {"inherited": HW_QUEUES_INHERITED, "effective": os.environ.get("GPU_MAX_HW_QUEUES")}}
        line.update(extra)
        print(json.dumps(_finite(line)), file=json_out, flush=True)
    if world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
