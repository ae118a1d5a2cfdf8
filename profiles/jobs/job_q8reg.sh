# Validate the register-resident activation-quantisation kernel (int8, >= 2 sequences): full GPU
# suite, smoke, every bench line, then kernel stats of the int8 B=8 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_q8b8r && profiles/jobs/job_validate.sh && tools/gpujob.sh \
 "prof_q8b8r:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q8b8r -o q8b8 -- python bench.py --steps 64 --skip-cpu --batch 8 --dtype int8"
