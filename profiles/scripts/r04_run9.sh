set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04j
timeout -k 10 500 python -u -m pytest tests/test_gpu_backend.py tests/test_gpu_comm.py tests/test_gpu_hierarchical.py tests/test_gpu_streams.py tests/test_gpu_rccl_procs.py tests/test_bucket_host.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r04j/tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --workload backend --steps 20 > gpurun_out/r04j/b_backend.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --workload backend --steps 20 > gpurun_out/r04j/b_backend2.json 2>/dev/null && \
BAGUA_SCHED_PROFILE=1 timeout -k 10 200 python -u bench.py --workload backend --steps 20 > gpurun_out/r04j/b_backend_prof.json 2> gpurun_out/r04j/b_backend_prof.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04j/trace_l2 -o be -- \
  python3 bench.py --workload backend --steps 8 --warmup 2 --no-cpu-baseline --lanes 2 > gpurun_out/r04j/be_traced.json 2>/dev/null && \
python3 profiles/trace_gaps.py gpurun_out/r04j/trace_l2 --window 0.4 --out gpurun_out/r04j/gaps_l2.json > /dev/null
echo "done rc=$?"
