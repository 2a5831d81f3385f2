#!/bin/bash
# round 6: the 1-bit fused middle step at p <= 2: tiles per wave iteration (BAGUA_OB_MIDDLE_U)
# x grid (BAGUA_TUNE_OB_MIDDLE_BLOCKS), pipeline probe with 4 pieces
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06obm
mkdir -p $O
cd $R
for u in 2 4 8; do
  for b in 1024 2048 4096; do
    BAGUA_OB_MIDDLE_U=$u BAGUA_TUNE_OB_MIDDLE_BLOCKS=$b timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/u${u}_b$b.json
  done
done
