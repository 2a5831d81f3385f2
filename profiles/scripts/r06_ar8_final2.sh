#!/bin/bash
# round 6: the N > 1 line at full size, 8 ranks on one GPU (RCCL socket transport), with the
# final kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06ar8
BAGUA_BENCH_SHARED_GPU=1 timeout -k 20 700 python3 -u bench.py --gpus 8 > gpurun_out/r06ar8/b_ar8.json 2> gpurun_out/r06ar8/b_ar8.err
