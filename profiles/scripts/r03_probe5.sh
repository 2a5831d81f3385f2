#!/usr/bin/env bash
# Round-3 batch 5: the whole GPU suite, then the profile set (profiles/run_profiles.sh r03).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gputest2.log 2>&1
rc=$?
tail -3 gpurun_out/r03_gputest2.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/run_profiles.sh r03
