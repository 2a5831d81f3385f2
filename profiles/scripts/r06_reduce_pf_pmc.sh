#!/bin/bash
# round 6: SQ counters of the pipelined MinMax op's kernels with the p = 2 recompute pair
# built with p known
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06rpfpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/pmc -o run -- python3 $R/tools/pipeline_kernels_probe.py --pieces 4 --reps 1 > $O/probe.json
