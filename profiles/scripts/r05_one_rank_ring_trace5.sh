set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace5" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only op_ring_bf16_p1 --rounds 6 --variants '[{},{"BAGUA_RING_ONE_RANK_MIX_BLOCKS":"512"},{"BAGUA_RING_ONE_RANK_MIX_BLOCKS":"2048"},{"BAGUA_RING_ONE_RANK_MIX_BLOCKS":"2048","BAGUA_RING_ONE_RANK_MIX_CFG":"2"},{"BAGUA_RING_ONE_RANK_MIX_BLOCKS":"768"}]' > "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace5.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace5.err"
