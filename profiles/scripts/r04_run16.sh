set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04q
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_resident.py tests/test_gpu_bench.py tests/test_gpu_op_goldens.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04q/tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04q/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r04q/b_default.json 2> gpurun_out/r04q/b_default.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04q/prof_default -o b -- \
  python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/r04q/b_default_traced.json 2>/dev/null
rc=$?; echo "done rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04q/pmc_fetch -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-allreduce-p1 --no-cold > /dev/null 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r04q/pmc_write -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-allreduce-p1 --no-cold > /dev/null 2>&1 && \
python3 profiles/collect_pmc.py gpurun_out/r04q/pmc_fetch gpurun_out/r04q/pmc_write gpurun_out/r04q/pmc_traffic.json
echo "pmc rc=$?"
