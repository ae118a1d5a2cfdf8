# Round-2 first GPU pass: full GPU suite, smoke, the default bench line (new headline / CPU
# aggregate / cooperative launch fields) and its rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "gpuall:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:500:python bench.py" \
 "bench_s20:300:python bench.py --steps 20 --skip-cpu" \
 "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02a -o r02a -- python bench.py --steps 20 --skip-cpu"
