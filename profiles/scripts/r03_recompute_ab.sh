#!/bin/bash
# A/B of the centralized op's middle step: the reduced own chunk stored and read
# back (BAGUA_REDUCE_RECOMPUTE=0) vs recomputed from the received segments (=1),
# N = 1 all-reduce (1 GiB) and the 32 x 25 MiB scheduler workload, interleaved.
set -e
out=gpurun_out/r03_recompute_ab.jsonl
mkdir -p gpurun_out
: > $out
for round in 1 2; do
  for rc in 0 1; do
    BAGUA_REDUCE_RECOMPUTE=$rc timeout -k 10 150 python bench.py --workload allreduce --steps 30 --warmup 5 \
      --no-cpu-baseline --no-decentralized > gpurun_out/ab.log 2>&1
    python - "$rc" "$round" allreduce >> $out <<'PY'
import json, sys
l = [x for x in open("gpurun_out/ab.log") if x.startswith("{")][-1]
d = json.loads(l)
print(json.dumps({"recompute": int(sys.argv[1]), "round": int(sys.argv[2]), "workload": sys.argv[3],
                  "ms_per_step": d["ms_per_step"], "gib_s": d["value"], "per_kernel_us": d.get("per_kernel_us")}))
PY
    BAGUA_REDUCE_RECOMPUTE=$rc timeout -k 10 150 python bench.py --workload backend --steps 10 --warmup 5 \
      --no-cpu-baseline > gpurun_out/ab.log 2>&1
    python - "$rc" "$round" backend >> $out <<'PY'
import json, sys
l = [x for x in open("gpurun_out/ab.log") if x.startswith("{")][-1]
d = json.loads(l)
print(json.dumps({"recompute": int(sys.argv[1]), "round": int(sys.argv[2]), "workload": sys.argv[3],
                  "ms_per_step": d["ms_per_step"], "gib_s": d["value"], "per_bucket_us": d.get("per_bucket_us")}))
PY
  done
done
cat $out
