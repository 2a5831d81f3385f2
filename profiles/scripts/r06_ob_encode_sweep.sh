#!/bin/bash
# round 6: the 1-bit encode's grid and tiles per iteration with the DPP tile tree (config 3 line)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06obe
mkdir -p $O
for tpi in 1 2; do
  for b in 2048 4096 8192 65536; do
    BAGUA_TUNE_OB_ENCODE_TPI=$tpi BAGUA_TUNE_OB_ENCODE_BLOCKS=$b timeout -k 10 120 python3 -u bench.py --workload onebit --steps 30 --no-cpu-baseline --no-cold > $O/t${tpi}_b$b.json 2> $O/t${tpi}_b$b.err || exit 1
  done
done
