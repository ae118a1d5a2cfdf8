# Same-box A/B/n of library variants lib/libthallama.so.<name> for VARIANTS="a b c", two rounds,
# BENCH_ARGS passed to bench.py.  Prints name, tok/s, ms/step, dominant-kernel avg us.
set -o pipefail
export TMPDIR=/tmp
L=hip_llama.cpp_amd/lib
cp $L/libthallama.so $L/libthallama.so.keep
for round in 1 2; do
  for v in ${VARIANTS}; do
    cp $L/libthallama.so.$v $L/libthallama.so
    timeout -k 10 300 python bench.py --steps 128 --warmup 4 --skip-cpu ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || { echo "bench $v rc=$?"; tail -20 gpurun_out/ab.log; cp $L/libthallama.so.keep $L/libthallama.so; exit 1; }
    tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_us'])"
  done
done
cp $L/libthallama.so.keep $L/libthallama.so
