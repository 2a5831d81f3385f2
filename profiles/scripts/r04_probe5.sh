#!/usr/bin/env bash
# Round 4: MinMax quantise / dequantise grids at 1 GiB (two-pass codec, the pipelined op's
# per-piece kernels) and 256 MiB, interleaved rounds.  Raw output: gpurun_out/r04p5
set -u
OUT=gpurun_out/r04p5
mkdir -p "$OUT"
T=tools
step() {
  local name=$1 to=$2; shift 2
  echo "[probe5] $name $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[probe5] $name failed rc=$rc" >&2; exit $rc; fi
}
for r in 1 2; do
  for cfg in "8192 16384" "32768 16384" "65536 16384" "8192 65536" "65536 65536"; do
    set -- $cfg
    BAGUA_TUNE_QUANT_BLOCKS=$1 BAGUA_TUNE_DEQUANT_BLOCKS=$2 step "c1g_$1_$2_r$r" 120 python3 bench.py --two-pass \
      --no-cpu-baseline --no-cold --no-allreduce-p1 --elements 268435456 --steps 30 > "$OUT/c1g_q$1_d$2_r$r.json"
    BAGUA_TUNE_QUANT_BLOCKS=$1 BAGUA_TUNE_DEQUANT_BLOCKS=$2 step "c256_$1_$2_r$r" 120 python3 bench.py \
      --no-cpu-baseline --no-cold --no-allreduce-p1 --steps 30 > "$OUT/c256_q$1_d$2_r$r.json"
    BAGUA_TUNE_QUANT_BLOCKS=$1 BAGUA_TUNE_DEQUANT_BLOCKS=$2 step "op_$1_$2_r$r" 120 python3 $T/op_probe.py --ranks 1 \
      --method minmax --pieces 4 --iters 4 --json "$OUT/op_q$1_d$2_r$r.json" > /dev/null
  done
done
echo "[probe5] done $(date +%T)" >&2
