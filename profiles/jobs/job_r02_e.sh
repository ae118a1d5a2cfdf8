cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "norm2:200:python tools/debug_q8.py 2 3 norm"
