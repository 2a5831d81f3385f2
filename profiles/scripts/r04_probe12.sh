#!/usr/bin/env bash
# Round 4: scheduler lanes 1..4 after the mark fast path and deferred completion events
# (32 x 25 MiB, p = 1), two interleaved rounds.  Raw output: gpurun_out/r04p12
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04p12
mkdir -p "$OUT"
for r in 3 4 5; do
  for l in 2 3; do
    echo "[probe12] lanes $l round $r $(date +%T)" >&2
    timeout -k 10 150 python3 bench.py --workload backend --steps 20 --no-cpu-baseline --lanes $l > "$OUT/l${l}_r$r.json" || exit $?
  done
done
echo "[probe12] done" >&2
