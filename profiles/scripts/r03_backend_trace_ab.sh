#!/bin/bash
# kernel timeline of the 32 x 25 MiB scheduler workload with the middle step
# stored + re-read (BAGUA_REDUCE_RECOMPUTE=0) vs recomputed with the final values
set -e
export TMPDIR=/tmp
for rc in 0 1; do
  BAGUA_REDUCE_RECOMPUTE=$rc timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_be_rc$rc -o be -- \
    python3 bench.py --workload backend --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_be_rc$rc.log 2>&1
done
