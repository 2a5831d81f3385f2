#!/bin/bash
# round 6: the 1-bit middle step's pair table at 2 < p <= 4 -- parity tests, then the
# pipeline probe with one and two tiles per wave iteration
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06obp
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "onebit" > $O/tests.txt 2>&1
for u in 1 2 4; do
  BAGUA_OB_MIDDLE_U=$u timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/u$u.json
done
BAGUA_OB_MIDDLE_U=1 BAGUA_TUNE_OB_MIDDLE_BLOCKS=4096 timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/u1_b4096.json
