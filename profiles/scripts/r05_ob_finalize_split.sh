set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05obs
BAGUA_OB_FINALIZE_SPLIT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_codec.py tests/test_gpu_onebit_edges.py tests/test_gpu_op_goldens.py -k "onebit or OneBit or one_bit" > gpurun_out/r05obs/t1.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload onebit --no-allreduce-p1 --cpu-seconds 0.5 > gpurun_out/r05obs/b0_$i.json 2>/dev/null || exit 1
  BAGUA_OB_FINALIZE_SPLIT=1 timeout -k 10 300 python -u bench.py --workload onebit --no-allreduce-p1 --cpu-seconds 0.5 > gpurun_out/r05obs/b1_$i.json 2>/dev/null || exit 1
done
cd /tmp && export TMPDIR=/tmp
BAGUA_OB_FINALIZE_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05obs/prof1" -o b -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload onebit --no-allreduce-p1 --cpu-seconds 0.5 > /dev/null 2>&1
