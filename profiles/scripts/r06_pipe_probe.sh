#!/bin/bash
# round 6: pipelined MinMax middle step, storing pair vs recompute (tools/pipeline_kernels_probe.py),
# then one PMC pass (SQ occupancy / VALU / LDS counters) over the same probe
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06pipe
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/pipeline_kernels_probe.py --pieces 4 > $O/probe_p4.json
timeout -k 10 300 python3 tools/pipeline_kernels_probe.py --pieces 8 > $O/probe_p8.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/pmc_sq -o run -- python3 $R/tools/pipeline_kernels_probe.py --pieces 4 --reps 1 > $O/pmc_sq_probe.json
