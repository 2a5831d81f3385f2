#!/usr/bin/env bash
# Round-3 batch 3: the resident-encode tests after the ticket/drain lane change,
# then ring_apply variants (contiguous family) and the mix pass A/B.
set -u
O=gpurun_out/r03
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "[r03] $name" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[r03] $name failed rc=$rc" >&2; exit $rc; fi
}
step apply_sweep 500 python3 tools/ring_apply_sweep.py --cfgs 0,14,16,17,18,19,20,21,22 --rounds 4 \
  > "$O/ring_apply_sweep3.jsonl"
echo "[r03] done" >&2
