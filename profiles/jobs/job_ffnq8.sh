# The SwiGLU launch stores its output quantised for W2 (int8, 4..8 sequences): full GPU suite,
# smoke, the int8 B=8 / B=4 bench lines, kernel stats of the int8 B=8 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_q8b8f gpurun_out/job.log && tools/gpujob.sh \
 "gpuall:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench_q8b8:400:python bench.py --batch 8 --dtype int8" \
 "bench_q8b4:400:python bench.py --batch 4 --dtype int8 --skip-cpu" \
 "prof_q8b8f:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q8b8f -o q8b8 -- python bench.py --steps 64 --skip-cpu --batch 8 --dtype int8"
