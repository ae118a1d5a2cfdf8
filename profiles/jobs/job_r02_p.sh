# Checkpoint at HEAD: the whole GPU suite, smoke, and the default / int8 / batch-8 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "gpuall:800:python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py" \
 "bench_q8:300:python bench.py --dtype int8 --skip-cpu" \
 "bench_b8:300:python bench.py --batch 8 --skip-cpu"
