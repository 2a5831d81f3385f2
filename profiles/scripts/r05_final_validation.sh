set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05final
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05final/gputests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05final/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r05final/b_default.json 2> gpurun_out/r05final/b_default.err || exit 1
timeout -k 10 400 python -u bench.py --workload allreduce > gpurun_out/r05final/b_ar1.json 2> gpurun_out/r05final/b_ar1.err || exit 1
timeout -k 10 400 python -u bench.py --workload onebit > gpurun_out/r05final/b_onebit.json 2> gpurun_out/r05final/b_onebit.err || exit 1
timeout -k 10 400 python -u bench.py --workload backend > gpurun_out/r05final/b_backend.json 2> gpurun_out/r05final/b_backend.err
