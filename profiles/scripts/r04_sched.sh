#!/usr/bin/env bash
# Round 4: the scheduler workload (32 x 25 MiB, p = 1) with cross-bucket lanes and the
# one-rank op, A/B against one lane and the four-kernel op; kernel traces for the
# GPU idle-gap analysis (profiles/trace_gaps.py).  Raw output: gpurun_out/r04s
set -u
OUT=gpurun_out/r04s
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "[sched] $name $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[sched] $name failed rc=$rc" >&2; exit $rc; fi
}
step be 200 python3 bench.py --workload backend --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/b_backend.json"
BAGUA_ONE_RANK_FUSED=0 step be_4k 200 python3 bench.py --workload backend --steps 20 --warmup 3 --no-cpu-baseline \
  > "$OUT/b_backend_fourkernel.json"
step ar1 200 python3 bench.py --workload allreduce --steps 20 --warmup 3 --no-cpu-baseline --no-decentralized \
  > "$OUT/b_ar1.json"
BAGUA_ONE_RANK_FUSED=0 step ar1_4k 200 python3 bench.py --workload allreduce --steps 20 --warmup 3 --no-cpu-baseline \
  --no-decentralized > "$OUT/b_ar1_fourkernel.json"
for ln in 2 1; do
  step trace_l$ln 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_l$ln" -o be -- \
    python3 bench.py --workload backend --steps 8 --warmup 2 --no-cpu-baseline --lanes $ln
  python3 profiles/trace_gaps.py "$OUT/trace_l$ln" --window 0.4 --out "$OUT/gaps_l$ln.json" > /dev/null || true
done
echo "[sched] done $(date +%T)" >&2
