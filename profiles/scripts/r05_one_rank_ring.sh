set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ring_one_rank.py "tests/test_gpu_comm.py::test_decentralized_low_precision_p1" "tests/test_gpu_comm.py::test_decentralized_p1_reads_its_own_bytes" tests/test_gpu_op_goldens.py > gpurun_out/r05_oner_t.log 2>&1 && \
timeout -k 10 300 python -u tools/kernel_ab.py --only op_ring_bf16_p1 --rounds 6 --variants '[{"BAGUA_ONE_RANK_FUSED":"0"},{},{"BAGUA_RING_ONE_RANK_CFG":"1"},{"BAGUA_RING_ONE_RANK_CFG":"2"},{"BAGUA_RING_ONE_RANK_CFG":"3"},{"BAGUA_RING_ONE_RANK_CFG":"4"}]' > gpurun_out/r05_oner_ab.json 2> gpurun_out/r05_oner_ab.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only op_ring_bf16_p1 --rounds 2 > "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_prof.log" 2>&1
