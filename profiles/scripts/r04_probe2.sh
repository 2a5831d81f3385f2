#!/usr/bin/env bash
# Round 4: 1 GiB streaming ceilings (tools/stream_probe), the 1-bit decode store policy A/B
# at 256 MiB and 1 GiB, the scheduler workload after the completed-ready-event change, and
# the round's headline profiles (profiles/run_profiles.sh r04).  Raw output: gpurun_out/r04p2
set -u
OUT=gpurun_out/r04p2
mkdir -p "$OUT"
export TMPDIR=/tmp
T=tools
step() {
  local name=$1 to=$2; shift 2
  echo "[probe2] $name $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[probe2] $name failed rc=$rc" >&2; exit $rc; fi
}
step stream_1g 200 $T/stream_probe 268435456 5 > "$OUT/stream_probe_1gib.txt"
BAGUA_OB_DECODE_NT=1 step cache_obnt 300 python3 $T/cache_state_probe.py --out "$OUT/cache_state_ob_nt.jsonl"
step b_onebit 150 python3 bench.py --workload onebit --no-cpu-baseline > "$OUT/b_onebit.json"
BAGUA_OB_DECODE_NT=1 step b_onebit_nt 150 python3 bench.py --workload onebit --no-cpu-baseline > "$OUT/b_onebit_nt.json"
step b_onebit_1g 150 python3 bench.py --workload onebit --no-cpu-baseline --elements 268435456 --no-cold > "$OUT/b_onebit_1g.json"
BAGUA_OB_DECODE_NT=1 step b_onebit_1g_nt 150 python3 bench.py --workload onebit --no-cpu-baseline --elements 268435456 --no-cold > "$OUT/b_onebit_1g_nt.json"
step b_backend 200 python3 bench.py --workload backend --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/b_backend.json"
step profiles 900 bash profiles/run_profiles.sh r04
echo "[probe2] done $(date +%T)" >&2
