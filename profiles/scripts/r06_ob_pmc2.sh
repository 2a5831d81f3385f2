#!/bin/bash
# round 6: SQ counters of the 1-bit middle-step kernels after the DPP tile tree
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06obpmc2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc -o run -- python3 $R/tools/pipeline_kernels_probe.py --pieces 4 --reps 1 --onebit-only > $O/probe.json
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR --output-format csv -d $O/pmc2 -o run -- python3 $R/tools/pipeline_kernels_probe.py --pieces 4 --reps 1 --onebit-only > $O/probe2.json
