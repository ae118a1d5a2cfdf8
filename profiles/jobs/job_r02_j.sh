# The reference's own GPU decode (oracle/_ref/libref_gpu.so) on this MI355X: 110M first (a fault
# there stops the job), then llama2-7B at batch 1 and 8; tokens / last-step drift vs the reference
# CPU goldens and tok/s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "ref110:150:python tools/ref_gpu.py stories110m_unshared" \
 "ref110s:150:python tools/ref_gpu.py stories110m_shared" \
 "ref7b:400:python tools/ref_gpu.py llama2_7b" \
 "ref7b_b8:400:python tools/ref_gpu.py llama2_7b --batch 8"
