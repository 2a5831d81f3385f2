set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/r04_gputests1.log 2>&1 && \
timeout -k 10 240 python -u bench.py > gpurun_out/r04_bench_default1.json 2> gpurun_out/r04_bench_default1.err
