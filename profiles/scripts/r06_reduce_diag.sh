#!/bin/bash
# round 6: where the partials-only fused reduce piece spends its time (timing diagnostics:
# BAGUA_REDUCE_DIAG=1 skips the table build, =2 the table lookups; results wrong by design)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06diag
mkdir -p $O
cd $R
for d in 0 1 2; do
  BAGUA_REDUCE_DIAG=$d timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/probe_p4_d$d.json
done
