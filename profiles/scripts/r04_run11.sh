set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04l
timeout -k 10 300 python -u -m pytest tests/test_gpu_backend.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r04l/tests.log 2>&1
echo "done rc=$?"
