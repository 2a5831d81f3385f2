#!/usr/bin/env bash
# Round 4: the one-rank op's table-pass grid at 1 GiB and 25 MiB buckets, interleaved.
set -u
OUT=gpurun_out/r04p6
mkdir -p "$OUT"
step() {
  local name=$1 to=$2; shift 2
  echo "[probe6] $name $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[probe6] $name failed rc=$rc" >&2; exit $rc; fi
}
for r in 1 2; do
  for g in 8192 16384 32768 65536; do
    BAGUA_TUNE_ONE_RANK_BLOCKS=$g step "ar1_${g}_r$r" 150 python3 bench.py --workload allreduce --steps 30 --warmup 3 \
      --no-cpu-baseline --no-decentralized > "$OUT/ar1_g${g}_r$r.json"
    BAGUA_TUNE_ONE_RANK_BLOCKS=$g step "be_${g}_r$r" 150 python3 bench.py --workload backend --steps 20 --warmup 3 \
      --no-cpu-baseline > "$OUT/be_g${g}_r$r.json"
  done
done
echo "[probe6] done $(date +%T)" >&2
