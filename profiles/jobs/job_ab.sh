# A/B two builds of the library on the same box: lib/libthallama.so.{old,new}
set -o pipefail
export TMPDIR=/tmp
L=hip_llama.cpp_amd/lib
for round in 1 2; do
  for v in old new; do
    cp $L/libthallama.so.$v $L/libthallama.so
    timeout -k 10 300 python bench.py --steps 128 --warmup 4 --skip-cpu ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_us'])"
  done
done
