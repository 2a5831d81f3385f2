set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_ring_one_rank.py tests/test_gpu_comm.py tests/test_gpu_op_goldens.py tests/test_gpu_multirank.py -k "decentral or ring or dec_ or Ring" > gpurun_out/r05_oner_t5.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_fullsize.py -k decentral > gpurun_out/r05_oner_t5b.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_final" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only op_ring_bf16_p1 --rounds 6 --variants '[{"BAGUA_ONE_RANK_FUSED":"0","BAGUA_RING_MIX_TILES":"0"},{"BAGUA_ONE_RANK_FUSED":"0"},{}]' > "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_final.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_final.err"
