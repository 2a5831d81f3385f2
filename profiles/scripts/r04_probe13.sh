#!/usr/bin/env bash
# Round 4: one-launch encode with the on-chip part of pass 1 loaded non-temporally
# (BAGUA_RESIDENT_CFG 12 / 13) against the default 11; config-2 line, rounds interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04p13
mkdir -p "$OUT"
for r in 1 2 3; do
  for c in 11 12 13; do
    echo "[probe13] cfg $c round $r $(date +%T)" >&2
    BAGUA_RESIDENT_CFG=$c timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-allreduce-p1 > "$OUT/c${c}_r$r.json" || exit $?
  done
done
echo "[probe13] done" >&2
