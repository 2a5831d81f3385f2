#!/usr/bin/env bash
# A/B of the 1-bit fused middle step: table-driven (default) vs per-element tree (BAGUA_ONEBIT_LUT=0)
set -euo pipefail
mkdir -p gpurun_out/lut
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "onebit or OneBit or rccl_procs" > gpurun_out/lut/tests.log 2>&1
for r in 1 2; do
  BAGUA_ONEBIT_LUT=0 timeout -k 10 200 python3 tools/onebit_reduce_probe.py > gpurun_out/lut/probe_off_$r.json
  timeout -k 10 200 python3 tools/onebit_reduce_probe.py > gpurun_out/lut/probe_on_$r.json
done
timeout -k 10 200 python3 tools/onebit_reduce_probe.py --dtype bf16 > gpurun_out/lut/probe_on_bf16.json
for r in 1 2; do
  BAGUA_ONEBIT_LUT=0 timeout -k 10 200 python3 bench.py --workload allreduce --no-decentralized > gpurun_out/lut/ar1_off_$r.json
  timeout -k 10 200 python3 bench.py --workload allreduce --no-decentralized > gpurun_out/lut/ar1_on_$r.json
done
