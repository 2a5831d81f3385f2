set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05nts
BAGUA_ONE_RANK_NTS=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "one_rank" > gpurun_out/r05nts/t0.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/kernel_ab.py --only one_rank_minmax_25m,one_rank_minmax_1g --rounds 6 --variants '[{},{"BAGUA_ONE_RANK_NTS":"0"}]' > gpurun_out/r05nts/ab.json 2> gpurun_out/r05nts/ab.err || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload backend > gpurun_out/r05nts/backend_nts1_$i.json 2>/dev/null || exit 1
  BAGUA_ONE_RANK_NTS=0 timeout -k 10 300 python -u bench.py --workload backend > gpurun_out/r05nts/backend_nts0_$i.json 2>/dev/null || exit 1
done
