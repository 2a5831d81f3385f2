set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05twice
for i in 1 2; do
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05twice/suite_$i.log 2>&1 || exit 1
done
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05twice/smoke.log 2>&1
