#!/usr/bin/env bash
# Round-3 batch 8: the remaining GPU test modules, then the profile set.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_comm.py tests/test_gpu_rccl_procs.py tests/test_gpu_resident.py \
  tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gputest3.log 2>&1
rc=$?
tail -3 gpurun_out/r03_gputest3.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/run_profiles.sh r03
