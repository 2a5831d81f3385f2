#!/usr/bin/env bash
# Round 4: VALU counters of the config-5 kernels (2^27 bf16, distinct payloads), one --pmc pass
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04p10
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/ring" -o p -- python3 tools/ring_kernels_probe.py --steps 5 > "$OUT/ring.json" 2> "$OUT/ring.err"
echo "rc=$?"
