#!/usr/bin/env bash
# Round 4: min/max pass with non-temporal loads (BAGUA_PARTIALS_NT) at 1 GiB, interleaved
# A/B: the one-rank op (bench --workload allreduce) and the pipelined op's prefix
# (tools/op_probe.py, p = 1, 4 pieces).  Raw output: gpurun_out/r04p3
set -u
OUT=gpurun_out/r04p3
mkdir -p "$OUT"
T=tools
step() {
  local name=$1 to=$2; shift 2
  echo "[probe3] $name $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[probe3] $name failed rc=$rc" >&2; exit $rc; fi
}
for r in 1 2; do
  for nt in 0 1; do
    BAGUA_PARTIALS_NT=$nt step ar1_nt${nt}_r$r 150 python3 bench.py --workload allreduce --steps 30 --warmup 3 \
      --no-cpu-baseline --no-decentralized > "$OUT/ar1_nt${nt}_r$r.json"
    BAGUA_PARTIALS_NT=$nt step op1_nt${nt}_r$r 150 python3 $T/op_probe.py --ranks 1 --method minmax --pieces 4 \
      --iters 5 --json "$OUT/op1_nt${nt}_r$r.json" > /dev/null
    BAGUA_PARTIALS_NT=$nt step be_nt${nt}_r$r 150 python3 bench.py --workload backend --steps 20 --warmup 3 \
      --no-cpu-baseline --bucket-mib 256 --buckets 8 > "$OUT/be256_nt${nt}_r$r.json"
  done
done
echo "[probe3] done $(date +%T)" >&2
