#!/usr/bin/env bash
# Round-3 measurement batch 1 (gpurun): encode A/B across kernel-library builds,
# the encode under a concurrent GEMM stream, config-5 ring kernel counters,
# and the pipelined op's queue mapping at 4 and 8 hardware queues.
set -u
O=gpurun_out/r03
mkdir -p "$O"
export TMPDIR=/tmp
L=bagua-core_amd/lib/libbagua_kernels.so
step() {  # name timeout cmd...: stop the batch at the first failure (fault, abort, timeout)
  local name=$1 to=$2; shift 2
  echo "[r03] $name" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[r03] $name failed rc=$rc" >&2; exit $rc; fi
}
step resident_ab 300 python3 tools/resident_ab.py --lib r01=ab_libs/r01/libbagua_kernels.so \
  --lib ac2efa0=ab_libs/ac2efa0/libbagua_kernels.so --lib f832131=ab_libs/f832131/libbagua_kernels.so \
  --lib 376ae00=ab_libs/376ae00/libbagua_kernels.so --lib head=$L --rounds 6 --steps 40 --trace \
  > "$O/resident_ab.jsonl"
step contention 300 python3 tools/contention_probe.py > "$O/contention.jsonl"
step ring_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ring_trace" -o ring -- \
  python3 tools/ring_probe.py --steps 10
step ring_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/ring_fetch" -o run -- \
  python3 tools/ring_probe.py --steps 3
step ring_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/ring_write" -o run -- \
  python3 tools/ring_probe.py --steps 3
# calibration of the counters on known byte counts with the ring kernels' access widths:
# the bf16 two-pass codec (16-B/lane loads; 8-B payload loads and stores)
step cal_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/cal_fetch" -o run -- \
  python3 bench.py --dtype bf16 --two-pass --steps 5 --warmup 1 --no-cpu-baseline --no-cold
step cal_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/cal_write" -o run -- \
  python3 bench.py --dtype bf16 --two-pass --steps 5 --warmup 1 --no-cpu-baseline --no-cold
for q in 4 8; do
  rm -rf /tmp/qp$q
  GPU_MAX_HW_QUEUES=$q timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$O/q$q/rank0" -o run -- \
    python3 tools/queue_probe.py 0 2 /tmp/qp$q > "$O/q$q.rank0.log" 2>&1 &
  p0=$!
  GPU_MAX_HW_QUEUES=$q timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$O/q$q/rank1" -o run -- \
    python3 tools/queue_probe.py 1 2 /tmp/qp$q > "$O/q$q.rank1.log" 2>&1 &
  p1=$!
  wait $p0; r0=$?
  wait $p1; r1=$?
  if [ $r0 -ne 0 ] || [ $r1 -ne 0 ]; then echo "[r03] queue probe q=$q failed: $r0 $r1" >&2; exit 1; fi
done
echo "[r03] done" >&2
