#!/usr/bin/env bash
# A/B: kernel-recorded timing events on every timed step vs every 4th vs every 50th (config 2 / 3)
set -euo pipefail
mkdir -p gpurun_out/kev
for r in 1 2 3; do
  for e in 1 4 50; do
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --kernel-events-every $e > gpurun_out/kev/codec_e${e}_$r.json
    timeout -k 10 120 python3 bench.py --workload onebit --no-cpu-baseline --kernel-events-every $e > gpurun_out/kev/onebit_e${e}_$r.json
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/kev/tests.log 2>&1
