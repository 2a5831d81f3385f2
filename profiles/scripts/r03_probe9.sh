#!/usr/bin/env bash
# Round-3 batch 9: phase stamps of the one-launch encode at HEAD (bench step order).
set -u
mkdir -p gpurun_out/r03
timeout -k 10 240 python3 -u tools/resident_trace.py --cfgs 11,9,10 --runs 20 --decode \
  --dump gpurun_out/r03/trace_stamps.npy > gpurun_out/r03/resident_trace_head.jsonl 2>&1
rc=$?
cat gpurun_out/r03/resident_trace_head.jsonl
exit $rc
