set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05_mixu" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only op_ring_bf16_p1 --rounds 6 --variants '[{"BAGUA_ONE_RANK_FUSED":"0"},{"BAGUA_ONE_RANK_FUSED":"0","BAGUA_RING_MIX_TILE_U":"2"},{"BAGUA_ONE_RANK_FUSED":"0","BAGUA_RING_MIX_TILE_U":"8"},{"BAGUA_ONE_RANK_FUSED":"0","BAGUA_RING_MIX_NTS":"1"}]' > "$GRAFT_REPO_ROOT/gpurun_out/r05_mixu.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05_mixu.err"
