#!/bin/bash
# Round 6 final tree: the whole GPU suite and smoke() on a fresh box.
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/ > gpurun_out/r06f_gputest.log 2>&1
rc=$?
echo "tests_rc=$rc" >> gpurun_out/r06f_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06f_smoke.log 2>&1
