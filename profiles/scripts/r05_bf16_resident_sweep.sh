# the bf16 codec line under each one-launch encode configuration, two rounds, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05bf
for r in 1 2; do
  for c in 12 11 9 2 0 1 5 6 10 13; do
    BAGUA_RESIDENT_CFG=$c timeout -k 10 120 python -u bench.py --dtype bf16 --no-cpu-baseline --no-allreduce-p1 --steps 40 > gpurun_out/r05bf/cfg${c}_r$r.json 2>/dev/null || exit 1
  done
done
