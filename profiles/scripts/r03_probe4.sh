#!/usr/bin/env bash
# Round-3 batch 4: launch-shape sweep of the codec kernels; ring tests with the new apply default.
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
step grid_sweep 400 python3 tools/grid_sweep.py --rounds 4 --steps 30 > "$O/grid_sweep.jsonl"
step ring_tests 400 python3 -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_fullsize.py -k "decentralized" -x -q \
  --timeout 120 --timeout-method thread
echo "[r03] done" >&2
