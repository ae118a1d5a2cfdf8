# Round-end evidence in one call: full GPU tests + smoke + the single-GPU bench lines, then the
# rocprofv3 kernel stats and separate PMC passes (profiles/jobs/job_r01_final.sh) and the traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && bash profiles/jobs/job_validate.sh && bash profiles/jobs/job_r01_final.sh && tools/gpujob.sh \
 "tr8:120:python tools/persist_trace.py --model 7b --pos 8" \
 "trq8:120:python tools/persist_trace.py --model 7b --pos 8 --dtype int8"
