#!/usr/bin/env bash
# Round 4: VALU instruction counts of the codec kernels (f32 vs bf16 vs f16, 256 MiB),
# one --pmc pass per dtype, kernel trace only.  Raw output: gpurun_out/r04p9
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04p9
mkdir -p "$OUT"
for dt in f32 bf16 f16; do
  echo "[probe9] $dt $(date +%T)" >&2
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/$dt" -o p -- python3 bench.py --dtype $dt --steps 5 --warmup 2 --no-cpu-baseline \
    --no-allreduce-p1 --no-cold > "$OUT/$dt.json" 2> "$OUT/$dt.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "[probe9] $dt failed rc=$rc" >&2; exit $rc; fi
done
echo "[probe9] done" >&2
