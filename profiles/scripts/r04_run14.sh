set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04o
timeout -k 10 500 python -u -m pytest tests/test_gpu_backend.py tests/test_gpu_comm.py tests/test_gpu_streams.py tests/test_gpu_rccl_procs.py tests/test_bucket_host.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r04o/tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --workload backend --steps 20 > gpurun_out/r04o/b_backend.json 2>/dev/null && \
BAGUA_SCHED_PROFILE=1 timeout -k 10 200 python -u bench.py --workload backend --steps 20 --no-cpu-baseline > gpurun_out/r04o/b_backend_prof.json 2> gpurun_out/r04o/b_backend_prof.err
echo "done rc=$?"
