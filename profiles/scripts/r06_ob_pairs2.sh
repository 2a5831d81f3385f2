#!/bin/bash
# round 6: where the 1-bit middle step's time goes -- its duration against the bucket size
# (a fixed part?), then one SQ counter pass over the 1-bit kernels at 1 GiB
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06obp2
mkdir -p $O
cd $R
for l in 24 26 27 28 29; do
  BAGUA_OB_MIDDLE_U=2 timeout -k 10 120 python3 tools/pipeline_kernels_probe.py --pieces 4 --onebit-only --log2n $l > $O/n$l.json
done
cd /tmp && export TMPDIR=/tmp
BAGUA_OB_MIDDLE_U=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc -o run -- python3 $R/tools/pipeline_kernels_probe.py --pieces 4 --reps 1 --onebit-only > $O/pmc_probe.json
