# Validate HEAD on the GPU: full GPU test suite, smoke, default bench line, int8 and B=8 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "gpuall:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py" \
 "bench_q8:400:python bench.py --dtype int8" \
 "bench_b8:400:python bench.py --batch 8 --skip-cpu"
