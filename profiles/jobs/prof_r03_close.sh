#!/usr/bin/env bash
# Round-3 close: the GPU suite, smoke, the default bench line, batch-8 and int8 lines, and the
# rocprofv3 kernel stats of the default bench (B=1 persistent step, plain launch: rocprofv3 crashes
# at exit after a cooperative one) — each step under its own limit (tools/gpujob.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_close && \
B="python bench.py --skip-cpu --no-long --no-requests-point" && \
tools/gpujob.sh \
 "suite:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py" \
 "b8:300:$B --batch 8 --steps 3" \
 "int8:300:$B --dtype int8 --steps 3" \
 "prof:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_close -o b1 -- $B --steps 5 --prof-steps 4"
