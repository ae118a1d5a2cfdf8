# Round-2 close at HEAD: the whole GPU suite, smoke, the default bench line, and for the batch-4 step
# (register-resident GEMV) rocprofv3 kernel stats plus separate FETCH_SIZE / WRITE_SIZE passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "gpuall:800:python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py" \
 "prof_b4:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b4 -o b4 -- python bench.py --batch 4 --skip-cpu --steps 64" \
 "pmcf_b4:120:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_b4 -o pmc -- python bench.py --batch 4 --steps 4 --warmup 1 --skip-cpu --prof-steps 2" \
 "pmcw_b4:120:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_b4 -o pmc -- python bench.py --batch 4 --steps 4 --warmup 1 --skip-cpu --prof-steps 2"
