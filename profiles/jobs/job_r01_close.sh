# Round-1 close: full GPU suite, smoke, every bench line (profiles/jobs/job_validate.sh), then the
# int8 B=8 kernel stats of the default path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_q8b8c && profiles/jobs/job_validate.sh && tools/gpujob.sh \
 "prof_q8b8c:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q8b8c -o q8b8 -- python bench.py --steps 64 --skip-cpu --batch 8 --dtype int8"
