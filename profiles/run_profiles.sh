#!/usr/bin/env bash
# Regenerates the committed profiles on a GPU box (gpurun):
#   bash profiles/run_profiles.sh r01
# 1. kernel trace + stats of the default bench (config 2) and of the 1-bit bench
# 2. two SEPARATE counter passes (FETCH_SIZE, WRITE_SIZE) of the same bench
#    (MI355X_MICROARCH.md: never combined with tracing), summarised by
#    collect_pmc.py into <round>_pmc_traffic.json
# Raw output stays under gpurun_out/prof; the summaries are copied to profiles/.
set -euo pipefail
R=${1:-r02}
OUT=gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(bench.py --steps 30 --warmup 5 --no-cpu-baseline)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o codec -- \
    python3 "${BENCH[@]}" > "$OUT/codec_under_rocprof.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_ob" -o onebit -- \
    python3 "${BENCH[@]}" --workload onebit > "$OUT/onebit_under_rocprof.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > /dev/null
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > /dev/null
# the same two counter passes of the 1-bit bench (config 3)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_ob" -o run -- \
    python3 bench.py --workload onebit --steps 5 --warmup 1 --no-cpu-baseline > /dev/null
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_ob" -o run -- \
    python3 bench.py --workload onebit --steps 5 --warmup 1 --no-cpu-baseline > /dev/null
# the two-pass encode (BAGUA_RESIDENT=0) for comparison
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_2p" -o twopass -- \
    python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --two-pass > "$OUT/twopass_under_rocprof.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_2p" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --two-pass > /dev/null
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_2p" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --two-pass > /dev/null
# plain bench lines (no profiler) for the committed r*_b_*.json
timeout -k 10 200 python3 bench.py > "$OUT/b_codec.json"
timeout -k 10 120 python3 bench.py --workload onebit --no-cpu-baseline > "$OUT/b_onebit.json"
timeout -k 10 120 python3 bench.py --dtype bf16 --no-cpu-baseline > "$OUT/b_codec_bf16.json"
timeout -k 10 120 python3 bench.py --workload allreduce > "$OUT/b_ar1.json"
timeout -k 10 200 python3 bench.py --workload host --steps 10 > "$OUT/b_host.json"
# python3 profiles/collect_pmc.py "$OUT/fetch" "$OUT/write" "profiles/${R}_pmc_traffic.json"
# python3 profiles/collect_pmc.py "$OUT/fetch_ob" "$OUT/write_ob" "profiles/${R}_pmc_traffic_onebit.json"
# (run locally on the merged gpurun_out/: only gpurun_out/ returns from the box)
# cp "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)" "profiles/${R}_bench_n1_kernel_stats.csv"
# (run locally on the merged gpurun_out/: only gpurun_out/ returns from the box)
# cp "$(find "$OUT/trace_ob" -name '*kernel_stats.csv' | head -1)" "profiles/${R}_onebit_kernel_stats.csv"
# cp "$OUT/codec_under_rocprof.json" "profiles/${R}_bench_n1_under_rocprof.json"
echo "profiles written for $R"
# small buckets through the whole op at p = 1 (host/launch overhead per op)
for e in 1048576 6553600 26214400; do
  timeout -k 10 120 python3 bench.py --workload allreduce --elements $e --steps 50 --no-decentralized > "$OUT/b_ar1_small_$e.json"
done
# the 1-bit op's fused middle step at p = 1..16 (table-driven kernel), 1 GiB bucket
timeout -k 10 200 python3 bagua-core_amd/tools/onebit_reduce_probe.py > "$OUT/onebit_reduce_probe.json"
# the N > 1 line rehearsed with 8 ranks on this one GPU over RCCL's socket transport
# (code path only; times are socket-bound)
BAGUA_BENCH_SHARED_GPU=1 NCCL_IB_DISABLE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29641 bench.py --gpus 8 --steps 3 --warmup 1 \
  --elements 4194304 > "$OUT/b_ar8_shared.json"
