#!/bin/bash
# round 6: the 1-bit streaming kernels' tile tree with permlane swaps and DPP row shifts
# (wave_tree_sum_lane0) -- parity tests, then the pipeline probe (1-bit only)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06obd
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "onebit" > $O/tests.txt 2>&1
for u in 1 2; do
  for b in 2048 4096; do
    BAGUA_OB_MIDDLE_U=$u BAGUA_TUNE_OB_MIDDLE_BLOCKS=$b timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 --onebit-only > $O/u${u}_b$b.json
  done
done
timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 --onebit-only > $O/default.json
