set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BAGUA_BENCH_SHARED_GPU=1 timeout -k 20 700 python3 -u bench.py --gpus 4 > gpurun_out/r05_b_ar4_v2.json 2> gpurun_out/r05_b_ar4_v2.err
