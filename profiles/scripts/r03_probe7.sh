#!/usr/bin/env bash
# Round-3 batch 7: scheduler bucket graphs (BAGUA_BACKEND_GRAPHS) -- tests, then an A/B
# of the 32 x 25 MiB scheduler workload, interleaved.
set -u
O=gpurun_out/r03
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "[r03] $name" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[r03] $name failed rc=$rc" >&2; exit $rc; fi
}
step backend_tests 300 python3 -u -m pytest tests/test_gpu_backend.py -x -q --timeout 120 --timeout-method thread
rm -f "$O/backend_graphs_ab.jsonl"
for r in 1 2 3; do
  for g in 0 1; do
    BAGUA_BACKEND_GRAPHS=$g PYTHONFAULTHANDLER=1 step "backend_g$g" 200 python3 -X faulthandler bench.py --workload backend --steps 10 --no-cpu-baseline \
      > "$O/b_backend_g$g.json" 2> "$O/b_backend_g$g.r$r.err" || { tail -40 "$O/b_backend_g$g.r$r.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_backend_g$g.json'));print(json.dumps({'round':$r,'BAGUA_BACKEND_GRAPHS':$g,'gib_s':d['value'],'per_bucket_us':d['per_bucket_us']}))" >> "$O/backend_graphs_ab.jsonl"
  done
done
echo "[r03] done" >&2
