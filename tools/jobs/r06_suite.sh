#!/bin/bash
# round 6: the whole GPU suite at HEAD, then smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r06_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r06_suite.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1
exit $rc
