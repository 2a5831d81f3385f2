set -o pipefail
cd "$GRAFT_REPO_ROOT"
BAGUA_SEGV_TRACE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_op_goldens.py -v -s --timeout 120 --timeout-method thread > gpurun_out/r04_dbg_opgoldens.log 2>&1
echo "op_goldens rc=$?" >> gpurun_out/r04_dbg_opgoldens.log
