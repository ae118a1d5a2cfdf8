set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q > gpurun_out/t.log 2>&1 || { echo "TESTS FAIL rc=$?"; tail -40 gpurun_out/t.log; exit 1; }
tail -3 gpurun_out/t.log
for b in 4 8 16; do
  timeout -k 10 240 python bench.py --batch $b --steps 64 --warmup 4 --skip-cpu > gpurun_out/b$b.log 2>&1 || { echo "bench b$b rc=$?"; tail -20 gpurun_out/b$b.log; exit 1; }
  tail -1 gpurun_out/b$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('kernels_ms', d.get('kernels')))"
done
