set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04n
timeout -k 10 300 python -u -m pytest tests/test_gpu_backend.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r04n/tests.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04n/trace_l3 -o be -- \
  python3 bench.py --workload backend --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r04n/be_traced.json 2>/dev/null && \
python3 profiles/trace_gaps.py gpurun_out/r04n/trace_l3 --window 0.4 --out gpurun_out/r04n/gaps_l3.json > /dev/null
echo "done rc=$?"
