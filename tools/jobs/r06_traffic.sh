#!/bin/bash
# round 6: where the persistent steps' bytes beyond the algorithmic ones come from — FETCH_SIZE /
# WRITE_SIZE passes (separate runs) of the 7B fp32 and int8 batch-1 steps at positions 0..7, on the
# normal library and on a traffic-attribution build whose phases do not gather their input
# (PERSIST_DIAG_NO_GATHER, tools/build_variant.sh): the difference is the hand-off gathers' traffic.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=hip_llama.cpp_amd/lib
cp $L/libthallama.so $L/libthallama.so.keep
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point --steps 1 --warmup 0 --decode-len 8"
rc=0
for v in ${VARIANTS:-base nogather}; do
  cp $L/libthallama.so.$v $L/libthallama.so
  for dt in f32 int8; do
    for c in FETCH_SIZE WRITE_SIZE; do
      THALLAMA_PERSIST_COOP=0 timeout -k 10 120 rocprofv3 --pmc $c -d gpurun_out/tr_${v}_${dt}_$c -o o -- $B --dtype $dt \
        > gpurun_out/tr_${v}_${dt}_$c.log 2>&1 || { rc=$?; echo "step $v $dt $c rc=$rc"; break 3; }
    done
    f=$(find gpurun_out/tr_${v}_${dt}_FETCH_SIZE -name '*results.db' | head -1)
    w=$(find gpurun_out/tr_${v}_${dt}_WRITE_SIZE -name '*results.db' | head -1)
    python tools/rocprof_summary.py pmc "$f" "$w" gpurun_out/r06_traffic_${v}_${dt}.json "$v $dt" llama2-7B 1
    rm -rf gpurun_out/tr_${v}_${dt}_*/
    echo "done $v $dt"
  done
done
cp $L/libthallama.so.keep $L/libthallama.so
exit $rc
