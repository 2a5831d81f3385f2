set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_ring_one_rank.py "tests/test_gpu_comm.py::test_decentralized_low_precision_p1" "tests/test_gpu_comm.py::test_decentralized_p1_reads_its_own_bytes" > gpurun_out/r05_oner_t4.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace4" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only op_ring_bf16_p1 --rounds 6 --variants '[{"BAGUA_ONE_RANK_FUSED":"0"},{"BAGUA_ONE_RANK_FUSED":"0","BAGUA_RING_MIX_TILES":"1"},{"BAGUA_ONE_RANK_FUSED":"0","BAGUA_RING_MIX_TILES":"1","BAGUA_RING_MIX_NTS":"1"},{}]' > "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace4.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace4.err"
