# HEAD check: the whole GPU suite, smoke, the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "gpuall:800:python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py"
