#!/usr/bin/env bash
# Round 4: 1-bit encode/decode launch shapes at 1 GiB and 256 MiB (grid, tiles per wave
# iteration), interleaved rounds.  Raw output: gpurun_out/r04p4
set -u
OUT=gpurun_out/r04p4
mkdir -p "$OUT"
step() {
  local name=$1 to=$2; shift 2
  echo "[probe4] $name $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[probe4] $name failed rc=$rc" >&2; exit $rc; fi
}
for r in 1 2; do
  for el in 268435456 67108864; do
    for cfg in "16384 1 16384" "65536 1 16384" "16384 2 16384" "32768 2 16384" "16384 1 65536" "65536 1 65536"; do
      set -- $cfg
      BAGUA_TUNE_OB_ENCODE_BLOCKS=$1 BAGUA_TUNE_OB_ENCODE_TPI=$2 BAGUA_TUNE_OB_DECODE_BLOCKS=$3 \
        step "ob_${el}_$1_$2_$3_r$r" 120 python3 bench.py --workload onebit --no-cpu-baseline --no-cold \
        --elements $el --steps 30 > "$OUT/ob_${el}_e$1_t$2_d$3_r$r.json"
    done
  done
done
echo "[probe4] done $(date +%T)" >&2
