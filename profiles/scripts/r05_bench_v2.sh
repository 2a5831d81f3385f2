set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r05_b_n1_v2.json 2> gpurun_out/r05_b_n1_v2.err || exit 1
timeout -k 10 400 python -u bench.py --workload allreduce > gpurun_out/r05_b_ar1_v2.json 2> gpurun_out/r05_b_ar1_v2.err || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_bench.py > gpurun_out/r05_bench_t.log 2>&1
