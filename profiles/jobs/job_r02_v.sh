# Checkpoint at HEAD (register-resident GEMV default at 4 sequences): the whole GPU suite, smoke,
# the default / int8 / batch-8 / batch-4 bench lines, rocprofv3 kernel stats of the batch-4 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "gpuall:800:python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py" \
 "bench_q8:300:python bench.py --dtype int8 --skip-cpu" \
 "bench_b8:300:python bench.py --batch 8 --skip-cpu" \
 "bench_b4:300:python bench.py --batch 4 --skip-cpu" \
 "prof_b4:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b4 -o b4 -- python bench.py --batch 4 --skip-cpu --steps 64"
