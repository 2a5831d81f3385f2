set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04g
timeout -k 10 400 python -u -m pytest tests/test_gpu_backend.py tests/test_gpu_comm.py tests/test_gpu_hierarchical.py tests/test_gpu_streams.py tests/test_bucket_host.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r04g/tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --workload backend --steps 20 > gpurun_out/r04g/b_backend.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --workload backend --steps 20 > gpurun_out/r04g/b_backend2.json 2>/dev/null && \
BAGUA_SCHED_PROFILE=1 BAGUA_OP_PROFILE=1 timeout -k 10 200 python -u bench.py --workload backend --steps 20 > gpurun_out/r04g/b_backend_prof.json 2> gpurun_out/r04g/b_backend_prof.err
echo "done rc=$?"
