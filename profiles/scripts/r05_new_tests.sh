set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_backend.py -k "lanes_mixed_ops" > gpurun_out/r05_new_tests.log 2>&1
