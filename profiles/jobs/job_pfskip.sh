# Sweep of the persistent step's prefetch-skip knob (THALLAMA_PF_SKIP), fp32 and int8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp
for dt in f32 int8; do
  for m in 0 64 1 4 8 16 29 0; do
    THALLAMA_PF_SKIP=$m timeout -k 10 120 python bench.py --steps 128 --warmup 4 --skip-cpu --dtype $dt > gpurun_out/pf.log 2>&1 || { echo "rc=$? dt=$dt m=$m"; tail -5 gpurun_out/pf.log; exit 1; }
    tail -1 gpurun_out/pf.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$dt', $m, d['value'], d['roofline']['avg_us'])"
  done
done
