# Same-box A/B of the fp32 B=1 headline: va = the round-2 start (commit df5220e, with today's test
# hooks), vb = HEAD; then the rocprofv3 kernel stats and PMC passes with a plain (non-cooperative)
# persistent launch — rocprofv3 crashes at exit after a cooperative launch (same kernel either way).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -rf gpurun_out/job.log gpurun_out/prof_* gpurun_out/pmc_* gpurun_out/pmcw_* && L=hip_llama.cpp_amd/lib && cp $L/libthallama.so $L/libthallama.so.keep && \
for r in 1 2; do for v in va vb; do cp $L/libthallama.so.$v $L/libthallama.so && timeout -k 10 200 python bench.py --skip-cpu > gpurun_out/ab_$v$r.out 2>gpurun_out/ab_$v$r.err || { cp $L/libthallama.so.keep $L/libthallama.so; exit 1; }; done; done; cp $L/libthallama.so.keep $L/libthallama.so && tools/gpujob.sh \
 "prof_ps:400:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ps -o ps -- python bench.py --steps 20 --skip-cpu" \
 "prof_q8:400:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q8 -o q8 -- python bench.py --steps 20 --skip-cpu --dtype int8" \
 "prof_b8:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b8 -o b8 -- python bench.py --steps 20 --skip-cpu --batch 8" \
 "pmc_ps:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_ps -o pmc -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2" \
 "pmcw_ps:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_ps -o pmcw -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2" \
 "pmc_q8:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_q8 -o pmc -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2 --dtype int8" \
 "pmcw_q8:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_q8 -o pmcw -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2 --dtype int8"
