# Round-2: the new parity tests (256-step reference goldens, gen_in_128 CLI fixture, the reference's
# own CLI on the library), the default bench line (now with the reference-token check), and a
# rocprofv3 stats pass with a plain (non-cooperative) persistent launch (exit-crash diagnosis).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "newtests:600:python -u -m pytest tests/test_golden_long_gpu.py tests/test_cli_gpu.py tests/test_dropin.py -m gpu -v --timeout 300 --timeout-method thread" \
 "bench:500:python bench.py" \
 "prof_plain:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02b -o r02b -- python bench.py --steps 20 --skip-cpu"
