# Round-2 validation at HEAD: the whole GPU suite (one process), the smoke entry point, and the
# fp32 batch-8 bench with and without the carried norm sums (A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "b8:300:python bench.py --batch 8 --skip-cpu" \
 "b8_nossq:300:THALLAMA_NO_SSQ=1 python bench.py --batch 8 --skip-cpu" \
 "gpuall:800:python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'"
