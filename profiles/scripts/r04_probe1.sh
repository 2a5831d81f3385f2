#!/usr/bin/env bash
# Round 4 probes (gpurun): config-5 ring kernels with distinct payloads; codec kernels at
# 256 MiB vs 1 GiB in three cache states; the pipelined op's kernels at 1 GiB inside the
# op (p = 1 durations, p = 1 and loopback p = 8 counters).  Raw output: gpurun_out/r04p1
set -u
OUT=gpurun_out/r04p1
mkdir -p "$OUT"
export TMPDIR=/tmp
T=tools
step() {  # name timeout cmd...: stop at the first failure (fault, abort, time limit)
  local name=$1 to=$2; shift 2
  echo "[probe] $name $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[probe] $name failed rc=$rc" >&2; exit $rc; fi
}
step ring_plain 150 python3 $T/ring_kernels_probe.py --json "$OUT/ring_kernels.json"
step ring_trace 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ring_trace" -o ring -- \
  python3 $T/ring_kernels_probe.py --steps 10
step ring_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/ring_fetch" -o run -- \
  python3 $T/ring_kernels_probe.py --steps 3
step ring_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/ring_write" -o run -- \
  python3 $T/ring_kernels_probe.py --steps 3
step cache 300 python3 $T/cache_state_probe.py --out "$OUT/cache_state.jsonl"
for m in minmax onebit; do
  step op1_${m}_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/op1_${m}_trace" -o op -- \
    python3 $T/op_probe.py --ranks 1 --method $m --pieces 4 --iters 6 --json "$OUT/op1_${m}.json"
  step op1_${m}_fetch 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/op1_${m}_fetch" -o run -- \
    python3 $T/op_probe.py --ranks 1 --method $m --pieces 4 --iters 2
  step op1_${m}_write 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/op1_${m}_write" -o run -- \
    python3 $T/op_probe.py --ranks 1 --method $m --pieces 4 --iters 2
  step op8_${m}_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/op8_${m}_fetch" -o run -- \
    python3 $T/op_probe.py --ranks 8 --method $m --pieces 4 --iters 2
  step op8_${m}_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/op8_${m}_write" -o run -- \
    python3 $T/op_probe.py --ranks 8 --method $m --pieces 4 --iters 2
done
echo "[probe] done $(date +%T)" >&2
