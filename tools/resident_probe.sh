set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread > gpurun_out/res_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/res_tests.log; exit 1; }
for c in 0 1 2 3 4 5; do
  BAGUA_RESIDENT_CFG=$c timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/res_cfg$c.json 2>gpurun_out/res_cfg$c.err || exit 1
done
BAGUA_RESIDENT=0 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/res_off.json 2>gpurun_out/res_off.err
