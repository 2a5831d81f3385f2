set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_backend.py -q -rf --timeout 200 --timeout-method thread > gpurun_out/r04_backend_tests4.log 2>&1 && \
BAGUA_SCHED_PROFILE=1 BAGUA_OP_PROFILE=1 timeout -k 10 200 python -u bench.py --workload backend --steps 20 --no-cpu-baseline \
  > gpurun_out/r04_b_backend4.json 2> gpurun_out/r04_b_backend4.err
