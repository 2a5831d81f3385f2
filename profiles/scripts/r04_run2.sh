set -o pipefail
cd "$GRAFT_REPO_ROOT"
BAGUA_SEGV_TRACE=1 timeout -k 10 720 python -u -m pytest tests -m gpu --maxfail=10 -q -rf --timeout 300 --timeout-method thread > gpurun_out/r04_gputests2.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r04_gputests2.log
# a test failure (rc 1) still lets the bench run; a crash, abort or time limit ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u bench.py > gpurun_out/r04_bench_default2.json 2> gpurun_out/r04_bench_default2.err && \
bash tools/r04_sched.sh > gpurun_out/r04_sched.log 2>&1
