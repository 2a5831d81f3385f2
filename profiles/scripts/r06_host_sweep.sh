#!/bin/bash
# round 6: host-resident rate (pinned H2D + codec + D2H) by buckets in flight and copy pieces
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06host
mkdir -p $O
cd $R
for nb in 2 3 4; do
  for ch in 1 2 4; do
    timeout -k 10 120 python3 bench.py --workload host --steps 10 --no-cpu-baseline --host-buffers $nb --copy-chunks $ch > $O/nb${nb}_ch$ch.json
  done
done
