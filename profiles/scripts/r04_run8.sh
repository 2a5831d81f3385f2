set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04i
timeout -k 10 720 python -u -m pytest tests -m gpu --maxfail=10 -q -rf --timeout 300 --timeout-method thread > gpurun_out/r04i/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r04i/gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04i/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r04i/b_default.json 2> gpurun_out/r04i/b_default.err && \
timeout -k 10 200 python -u bench.py --workload onebit > gpurun_out/r04i/b_onebit.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --dtype bf16 > gpurun_out/r04i/b_codec_bf16.json 2>/dev/null && \
timeout -k 10 300 python -u bench.py --workload allreduce > gpurun_out/r04i/b_ar1.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --workload backend --steps 20 > gpurun_out/r04i/b_backend.json 2>/dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04i/prof_default -o b -- \
  python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/r04i/b_default_traced.json 2>/dev/null
echo "done rc=$?"
