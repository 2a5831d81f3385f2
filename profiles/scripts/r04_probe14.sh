#!/usr/bin/env bash
# Round 4: one-launch encode configuration 11 vs 12 for bf16 and f16 buckets (256 MiB),
# rounds interleaved.  Raw output: gpurun_out/r04p14
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04p14
mkdir -p "$OUT"
for r in 1 2 3; do
  for dt in bf16 f16; do
    for c in 11 12; do
      echo "[probe14] $dt cfg $c round $r $(date +%T)" >&2
      BAGUA_RESIDENT_CFG=$c timeout -k 10 150 python3 bench.py --dtype $dt --no-cpu-baseline --no-allreduce-p1 > "$OUT/${dt}_c${c}_r$r.json" || exit $?
    done
  done
done
echo "[probe14] done" >&2
