set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05final_prof" -o b -- python3 "$GRAFT_REPO_ROOT/bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/r05final_prof_line.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05final_prof.err"
