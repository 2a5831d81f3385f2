set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05spread
timeout -k 10 400 python -u bench.py > gpurun_out/r05spread/b_default_$1.json 2>/dev/null
