#!/bin/bash
# round 6: grids of the fused reduce pieces (BAGUA_TUNE_FUSED_BLOCKS) and of the
# recompute requantise (BAGUA_TUNE_RRQ_BLOCKS), pipeline probe with 4 pieces
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06mgrid
mkdir -p $O
cd $R
for b in 1024 2048 4096; do
  BAGUA_TUNE_FUSED_BLOCKS=$b timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/fb$b.json
done
for b in 256 1024 2048 4096; do
  BAGUA_TUNE_RRQ_BLOCKS=$b timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/rrq$b.json
done
