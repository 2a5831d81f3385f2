set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04s2
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04s2/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r04s2/b_default.json 2> gpurun_out/r04s2/b_default.err
echo "done rc=$?"
