#!/bin/bash
# round 6: the storing reduce piece with half the vectors per lane per step
# (BAGUA_TUNE_REDUCE_QD=2, fewer accumulators -> fewer VGPRs) against the default
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06rqd
mkdir -p $O
cd $R
BAGUA_TUNE_REDUCE_QD=2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or piece" > $O/tests.txt 2>&1
BAGUA_TUNE_REDUCE_QD=2 timeout -k 10 150 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/qd2.json
timeout -k 10 150 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/qd1.json
