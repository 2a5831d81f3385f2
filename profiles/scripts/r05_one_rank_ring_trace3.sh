set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace3" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only op_ring_bf16_p1 --rounds 6 --variants '[{"BAGUA_ONE_RANK_FUSED":"0"},{},{"BAGUA_RING_ONE_RANK_MIX_CFG":"1"},{"BAGUA_RING_ONE_RANK_MIX_CFG":"2"},{"BAGUA_RING_ONE_RANK_MIX_CFG":"3"},{"BAGUA_RING_ONE_RANK_MIX_CFG":"4"}]' > "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace3.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05_oner_trace3.err"
