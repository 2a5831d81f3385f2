set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 720 python -u -m pytest tests -m gpu --maxfail=10 -q -rf --timeout 300 --timeout-method thread > gpurun_out/r04_gputests3.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r04_gputests3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u bench.py > gpurun_out/r04_bench_default3.json 2> gpurun_out/r04_bench_default3.err && \
timeout -k 10 200 python -u bench.py --workload onebit > gpurun_out/r04_b_onebit3.json 2>/dev/null && \
timeout -k 10 300 python -u bench.py --workload allreduce > gpurun_out/r04_b_ar1_3.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --workload backend --steps 20 > gpurun_out/r04_b_backend3.json 2>/dev/null
