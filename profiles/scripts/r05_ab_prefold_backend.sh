set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_codec.py tests/test_gpu_multirank.py tests/test_gpu_op_goldens.py > gpurun_out/r05_t6.log 2>&1 || exit 1
V='[{"BAGUA_QUANT_PREFOLD":"0"}, {"BAGUA_QUANT_PREFOLD":"1"}]'
timeout -k 10 400 python3 tools/kernel_ab.py --only op_ring_bf16_p1,quant_f32_256m,quant_bf16_ring --rounds 4 --reps 8 --variants "$V" > gpurun_out/r05_prefold.json 2> gpurun_out/r05_prefold.err || exit 1
for i in 1 2 3; do
  (cd ab_libs/r04 && timeout -k 10 200 python3 bench.py --workload backend --steps 20 --no-cpu-baseline > ../../gpurun_out/r05_ab_backend_r04_$i.json 2>/dev/null) || exit 1
  timeout -k 10 200 python3 bench.py --workload backend --steps 20 --no-cpu-baseline > gpurun_out/r05_ab_backend_r05_$i.json 2>/dev/null || exit 1
done
V2='[{}, {"BAGUA_RING_MIX_U":"2"}, {"BAGUA_RING_MIX_U":"8"}]'
timeout -k 10 400 python3 tools/kernel_ab.py --only mix_bf16,op_ring_bf16_p1 --rounds 3 --reps 6 --variants "$V2" > gpurun_out/r05_mixu.json 2> gpurun_out/r05_mixu.err || exit 1
