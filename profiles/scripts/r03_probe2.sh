#!/usr/bin/env bash
# Round-3 measurement batch 2: ring_apply variants (config 5) and the 1-bit codec A/B
# between the round-1 and current kernel libraries.
set -u
O=gpurun_out/r03
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "[r03] $name" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[r03] $name failed rc=$rc" >&2; exit $rc; fi
}
step encode_ab 300 python3 tools/resident_ab.py --lib r01=ab_libs/r01/libbagua_kernels.so \
  --lib ac2efa0=ab_libs/ac2efa0/libbagua_kernels.so --lib r03a=ab_libs/r03a/libbagua_kernels.so \
  --lib lanes=bagua-core_amd/lib/libbagua_kernels.so --rounds 8 --steps 40 --trace > "$O/encode_lanes_ab.jsonl"
step apply_sweep 400 python3 tools/ring_apply_sweep.py --rounds 4 > "$O/ring_apply_sweep.jsonl"
step onebit_ab 200 python3 tools/resident_ab.py --onebit --lib r01=ab_libs/r01/libbagua_kernels.so \
  --lib f832131=ab_libs/f832131/libbagua_kernels.so --lib head=bagua-core_amd/lib/libbagua_kernels.so \
  --rounds 6 --steps 40 > "$O/onebit_ab.jsonl"
echo "[r03] done" >&2
