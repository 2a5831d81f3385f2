#!/bin/bash
# round 6, after the 1-bit kernel changes: the GPU suite, smoke(), the default N = 1 line
# and the 1-bit line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${VAL_DIR:-r06val2}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/b_default.json 2> $O/b_default.err || exit 1
timeout -k 10 400 python -u bench.py --workload onebit > $O/b_onebit.json 2> $O/b_onebit.err || exit 1
