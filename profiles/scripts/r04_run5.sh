set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04s5/trace_l2 -o be -- \
  python3 bench.py --workload backend --steps 8 --warmup 2 --no-cpu-baseline --lanes 2 > gpurun_out/r04s5_be_traced.json 2>/dev/null && \
python3 profiles/trace_gaps.py gpurun_out/r04s5/trace_l2 --window 0.4 --out gpurun_out/r04s5_gaps_l2.json > /dev/null
