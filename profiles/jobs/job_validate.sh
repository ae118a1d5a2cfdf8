# Validate HEAD on the GPU: full GPU test suite, smoke, the bench lines of every BASELINE config
# that fits one GPU (7B fp32 = the default line, 7B int8, 7B fp32 B=8, 110M fp32) and int8 B=8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "gpuall:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py" \
 "bench_q8:400:python bench.py --dtype int8" \
 "bench_b8:400:python bench.py --batch 8" \
 "bench_q8b8:400:python bench.py --batch 8 --dtype int8" \
 "bench_110m:400:python bench.py --model 110m"
