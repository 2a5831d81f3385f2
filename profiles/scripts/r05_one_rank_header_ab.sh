set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "one_rank" > gpurun_out/r05_hdr_t.log 2>&1 || exit 1
BAGUA_ONE_RANK_HEADER=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "one_rank" > gpurun_out/r05_hdr_t1.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05_hdr" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only one_rank_minmax_25m,one_rank_minmax_1g --rounds 6 --variants '[{},{"BAGUA_ONE_RANK_HEADER":"1"}]' > "$GRAFT_REPO_ROOT/gpurun_out/r05_hdr.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05_hdr.err"
