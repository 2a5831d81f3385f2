#!/bin/bash
# round 6: the 1-bit finalize's ragged batch with clamped loads -- parity tests, then a
# kernel trace of the 1-bit probe (per-dispatch durations of the finalize and middle kernels)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06obf
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "onebit" > $O/tests.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/pipeline_kernels_probe.py --pieces 4 --onebit-only --reps 5 > $O/probe.json
