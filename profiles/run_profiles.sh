#!/usr/bin/env bash
# Regenerates the committed profiles on a GPU box (gpurun), e.g.
#   bash profiles/run_profiles.sh r03
# 1. kernel trace + stats of the default bench (config 2) and of the 1-bit bench (config 3)
# 2. two SEPARATE counter passes (FETCH_SIZE, WRITE_SIZE) of each (MI355X_MICROARCH.md:
#    never combined with tracing), summarised locally by profiles/collect_pmc.py
# 3. plain bench lines of every workload, and the config-5 ring op's kernel split
# Raw output under gpurun_out/prof_<round>; summaries are copied to profiles/ locally:
#   python3 profiles/collect_pmc.py gpurun_out/prof_r03/fetch gpurun_out/prof_r03/write profiles/r03_pmc_traffic.json
set -u
R=${1:-r03}
OUT=gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...: stop at the first failure (fault, abort, time limit)
  local name=$1 to=$2; shift 2
  echo "[prof] $name" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[prof] $name failed rc=$rc" >&2; exit $rc; fi
}
B=(bench.py --steps 30 --warmup 5 --no-cpu-baseline)
step trace_codec 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o codec -- \
  python3 "${B[@]}" --no-cold > "$OUT/codec_under_rocprof.json"
step trace_onebit 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_ob" -o onebit -- \
  python3 "${B[@]}" --no-cold --workload onebit > "$OUT/onebit_under_rocprof.json"
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-cold
step write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-cold
step fetch_ob 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_ob" -o run -- \
  python3 bench.py --workload onebit --steps 5 --warmup 1 --no-cpu-baseline --no-cold
step write_ob 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_ob" -o run -- \
  python3 bench.py --workload onebit --steps 5 --warmup 1 --no-cpu-baseline --no-cold
step trace_ar1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_ar1" -o ar1 -- \
  python3 bench.py --workload allreduce --steps 20 --warmup 3 --no-cpu-baseline --no-decentralized \
  > "$OUT/ar1_under_rocprof.json"
step ring_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ring_trace" -o ring -- \
  python3 tools/ring_probe.py --steps 10
step b_codec 200 python3 bench.py > "$OUT/b_codec.json"
step b_onebit 200 python3 bench.py --workload onebit > "$OUT/b_onebit.json"
step b_bf16 200 python3 bench.py --dtype bf16 > "$OUT/b_codec_bf16.json"
step b_ar1 300 python3 bench.py --workload allreduce > "$OUT/b_ar1.json"
step b_host 300 python3 bench.py --workload host --steps 10 > "$OUT/b_host.json"
step b_backend 300 python3 bench.py --workload backend --steps 10 > "$OUT/b_backend.json"
echo "[prof] profiles written for $R" >&2
