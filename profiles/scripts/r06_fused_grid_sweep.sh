#!/bin/bash
# round 6: workgroups of the fused reduce pieces (contiguous shares), pipeline probe per grid cap
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06grid
mkdir -p $O
cd $R
for b in 1024 1536 1792 2048 3072 4096; do
  BAGUA_TUNE_FUSED_BLOCKS=$b timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/probe_p4_b$b.json
done
