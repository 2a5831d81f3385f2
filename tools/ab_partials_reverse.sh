#!/usr/bin/env bash
# A/B of the pipelined op's backwards min/max sweep (BAGUA_PARTIALS_FORWARD=1: the old forward
# sweep): parity of the pipelined tests, op time at p = 1 with 4 pieces, and the first quantise
# piece's duration from a kernel trace
set -euo pipefail
mkdir -p gpurun_out/rev
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_codec.py -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "pipelined or stage or range" > gpurun_out/rev/tests.log 2>&1
for r in 1 2 3; do
  for f in 1 0; do
    BAGUA_PARTIALS_FORWARD=$f timeout -k 10 200 python3 bench.py --workload allreduce --pieces 4 --no-decentralized \
      --steps 30 > gpurun_out/rev/ar_f${f}_$r.json
  done
done
export TMPDIR=/tmp
for f in 1 0; do
  BAGUA_PARTIALS_FORWARD=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rev/trace_f$f \
    -o run -- python3 bench.py --workload allreduce --pieces 4 --no-decentralized --steps 10 --warmup 2 > /dev/null
done
