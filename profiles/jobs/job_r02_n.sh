# seqsum guess fix: rounds/cycles fit, the seqsum and exact int8 tests, int8 trace + bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "rounds:200:python tools/seqsum_rounds.py" \
 "sstest:300:python -u -m pytest tests/test_seqsum_gpu.py tests/test_q8_persist_gpu.py tests/test_golden_long_gpu.py -q -s -m gpu -k 'seqsum or bitexact or q8 or int8' --timeout 200 --timeout-method thread" \
 "tr_q8:200:python tools/persist_trace.py --dtype int8 --pos 8" \
 "bench_q8:300:python bench.py --dtype int8 --skip-cpu"
