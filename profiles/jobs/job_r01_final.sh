# Round-1 profile refresh: rocprofv3 kernel stats (fp32 B=1 persistent, int8 B=1 persistent,
# fp32 B=8 matrix-core GEMV) and the HBM traffic PMC passes (FETCH_SIZE / WRITE_SIZE, separate
# runs) for the two persistent steps; summaries by tools/rocprof_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_* gpurun_out/pmc_* && tools/gpujob.sh \
 "prof_ps:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ps -o ps -- python bench.py --steps 64 --skip-cpu" \
 "prof_q8:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q8 -o q8 -- python bench.py --steps 64 --skip-cpu --dtype int8" \
 "prof_b8:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b8 -o b8 -- python bench.py --steps 64 --skip-cpu --batch 8" \
 "pmc_ps:500:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_ps -o pmc -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2" \
 "pmcw_ps:500:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_ps -o pmcw -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2" \
 "pmc_q8:500:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_q8 -o pmc -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2 --dtype int8" \
 "pmcw_q8:500:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_q8 -o pmcw -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2 --dtype int8"
