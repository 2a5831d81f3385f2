#!/usr/bin/env bash
# Round 4: the bf16 codec line's one-off 0.32 ms step (resident encode 893 us average,
# gpurun_out/r04k/b_codec_bf16.json): repeat the bf16 and f32 lines with the timed
# region's give-up count, then a kernel trace of a bf16 run.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04p11
mkdir -p "$OUT"
step() {
  local name=$1 to=$2; shift 2
  echo "[probe11] $name $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[probe11] $name failed rc=$rc" >&2; exit $rc; fi
}
for r in 1 2 3; do
  step bf16_$r 150 python3 bench.py --dtype bf16 --no-cpu-baseline --no-allreduce-p1 > "$OUT/bf16_$r.json"
  step f32_$r 150 python3 bench.py --no-cpu-baseline --no-allreduce-p1 > "$OUT/f32_$r.json"
done
step trace_bf16 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_bf16" -o t -- \
  python3 bench.py --dtype bf16 --no-cpu-baseline --no-allreduce-p1 > "$OUT/bf16_traced.json"
echo "[probe11] done $(date +%T)" >&2
