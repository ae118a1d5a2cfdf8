cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "dbg1:200:python tools/debug_q8.py 1 3" \
 "dbg0:200:python tools/debug_q8.py 0 4" \
 "dbg2:200:python tools/debug_q8.py 2 2"
