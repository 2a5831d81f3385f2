set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04h
timeout -k 10 300 python3 -u tools/one_rank_keep_probe.py --rounds 3 --keeps=-1,256,320,384,448,512 > gpurun_out/r04h/keep_probe2.jsonl 2> gpurun_out/r04h/keep_probe2.err
rc=$?; echo "done rc=$rc"; [ $rc -eq 0 ] && bash tools/r04_probe8.sh
