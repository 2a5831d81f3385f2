#!/usr/bin/env bash
# Round-3 batch 6: comm-op tests after the one-rank exchange changes, N=1 all-reduce / backend lines.
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
step comm_tests 500 python3 -u -m pytest tests/test_gpu_comm.py tests/test_gpu_backend.py tests/test_gpu_multirank.py \
  tests/test_gpu_c_abi.py tests/test_gpu_bench.py -x -q --timeout 200 --timeout-method thread
step b_ar1 300 python3 bench.py --workload allreduce > "$O/b_ar1_v2.json"
step b_backend 300 python3 bench.py --workload backend --steps 10 > "$O/b_backend_v2.json"
step ring 120 python3 tools/ring_probe.py --steps 20
echo "[r03] done" >&2
