# Bench the config-2 step for each one-launch encode configuration ($@), one process each.
set -o pipefail
mkdir -p gpurun_out
for c in "$@"; do
  BAGUA_RESIDENT_CFG=$c timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/sweep_cfg$c.json 2>gpurun_out/sweep_cfg$c.err || exit 1
done
