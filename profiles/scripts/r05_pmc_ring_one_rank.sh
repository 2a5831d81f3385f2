set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05pr
cd /tmp && export TMPDIR=/tmp
V='[{},{"BAGUA_ONE_RANK_FUSED":"0"}]'
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05pr/fetch" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only op_ring_bf16_p1 --rounds 1 --reps 3 --variants "$V" > /dev/null 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05pr/write" -o run -- python3 "$GRAFT_REPO_ROOT/tools/kernel_ab.py" --only op_ring_bf16_p1 --rounds 1 --reps 3 --variants "$V" > /dev/null 2>&1 && \
cd "$GRAFT_REPO_ROOT" && python3 profiles/collect_pmc_dispatch.py gpurun_out/r05pr/fetch gpurun_out/r05pr/write gpurun_out/r05pr/pmc.json
