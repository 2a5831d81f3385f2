set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/kernel_ab.py --only op_ring_bf16_p1 --rounds 8 --variants '[{"BAGUA_ONE_RANK_FUSED":"0"},{},{"BAGUA_RING_ONE_RANK_CFG":"1"},{"BAGUA_RING_ONE_RANK_CFG":"4"},{"BAGUA_RING_ONE_RANK_CFG":"5"},{"BAGUA_RING_ONE_RANK_CFG":"6"},{"BAGUA_RING_ONE_RANK_CFG":"7"},{"BAGUA_RING_ONE_RANK_CFG":"8"},{"BAGUA_RING_ONE_RANK_CFG":"4","BAGUA_RING_MIX_NTS":"1"},{"BAGUA_RING_ONE_RANK_CFG":"6","BAGUA_RING_MIX_NTS":"1"}]' > gpurun_out/r05_oner_sweep.json 2> gpurun_out/r05_oner_sweep.err
