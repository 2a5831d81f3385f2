#!/usr/bin/env bash
# Round 4: the pipelined op's backward min/max pass with the chunks' beginnings (the
# last BAGUA_PARTIALS_KEEP_MIB of the sweep) loaded with the default policy, the rest
# non-temporally; tools/op_probe.py p = 1, 4 pieces, 1 GiB, rounds interleaved.
set -u
OUT=gpurun_out/r04p8
mkdir -p "$OUT"
T=tools
step() {
  local name=$1 to=$2; shift 2
  echo "[probe8] $name $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[probe8] $name failed rc=$rc" >&2; exit $rc; fi
}
for r in 1 2 3; do
  for keep in 0 128 256 384; do
    BAGUA_PARTIALS_KEEP_MIB=$keep step op1_k${keep}_r$r 150 python3 $T/op_probe.py --ranks 1 --method minmax --pieces 4 \
      --iters 5 --json "$OUT/op1_k${keep}_r$r.json" > /dev/null
  done
done
echo "[probe8] done $(date +%T)" >&2
