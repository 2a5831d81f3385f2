#!/bin/bash
# round 6, final tree: the default N = 1 line three times on one box, then the 1-bit line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06fs
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py > $O/b_default_$i.json 2> $O/b_default_$i.err || exit 1
done
timeout -k 10 300 python3 -u bench.py --workload onebit > $O/b_onebit.json 2> $O/b_onebit.err || exit 1
