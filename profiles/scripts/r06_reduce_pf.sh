#!/bin/bash
# round 6: the fused reduce kernels with a 32-bit uniform tile counter and compile-time p
# (p = 2 recompute reduce + requantise, p = 4 / 8 storing reduce) -- parity tests, then the
# pipeline probe with BAGUA_REDUCE_PF=1 (default) and 0
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06rpf
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_multirank.py tests/test_gpu_op_goldens.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 150 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/pf1.json
BAGUA_REDUCE_PF=0 timeout -k 10 150 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/pf0.json
