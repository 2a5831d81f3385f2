set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ring_one_rank.py "tests/test_gpu_comm.py::test_decentralized_low_precision_p1" "tests/test_gpu_comm.py::test_decentralized_p1_reads_its_own_bytes" > gpurun_out/r05_oner_t2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace2" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only op_ring_bf16_p1 --rounds 6 --variants '[{"BAGUA_ONE_RANK_FUSED":"0"},{},{"BAGUA_RING_ONE_RANK_KEEP_MIB":"0"},{"BAGUA_RING_ONE_RANK_KEEP_MIB":"256"},{"BAGUA_RING_ONE_RANK_KEEP_MIB":"128"},{"BAGUA_RING_ONE_RANK_RECOMPUTE":"0"},{"BAGUA_RING_ONE_RANK_CFG":"4"},{"BAGUA_RING_ONE_RANK_CFG":"6"}]' > "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace2.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace2.err"
