# Round-2 measurement refresh at HEAD: the default bench line (fp32 7B B=1, CPU baseline included),
# rocprofv3 kernel stats of the fp32 / int8 persistent steps and the fp32 batch-8 step, and the
# HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE, one counter per run) for both persistent steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -rf gpurun_out/job.log gpurun_out/prof_* gpurun_out/pmc_* gpurun_out/pmcw_* && tools/gpujob.sh \
 "bench:500:python bench.py" \
 "prof_ps:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ps -o ps -- python bench.py --steps 20 --skip-cpu" \
 "prof_q8:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q8 -o q8 -- python bench.py --steps 20 --skip-cpu --dtype int8" \
 "prof_b8:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b8 -o b8 -- python bench.py --steps 20 --skip-cpu --batch 8" \
 "pmc_ps:300:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_ps -o pmc -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2" \
 "pmcw_ps:300:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_ps -o pmcw -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2" \
 "pmc_q8:300:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_q8 -o pmc -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2 --dtype int8" \
 "pmcw_q8:300:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_q8 -o pmcw -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2 --dtype int8"
