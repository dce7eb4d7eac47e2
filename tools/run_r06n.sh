#!/bin/bash
# Round 6 final tree (after the diagnostic clock-stamp sources, off by default): the whole GPU suite, smoke() and the default bench line.
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/ > gpurun_out/r06n_gputest.log 2>&1
rc=$?
echo "tests_rc=$rc" >> gpurun_out/r06n_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06n_smoke.log 2>&1
[ $? -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06n_bench.json 2> gpurun_out/r06n_bench.err
