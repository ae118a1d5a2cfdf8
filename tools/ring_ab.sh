#!/usr/bin/env bash
# A/B of the persistent step's LDS slot ring (loader wave): default vs THALLAMA_PERSIST_RING=0,
# 7B fp32 and int8 batch 1, alternating; prints ms per token of the 256-step decode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B="python bench.py --skip-cpu --no-long --no-requests-point --steps 2 --warmup 1 --prof-steps 4"
for r in 1 2; do
  for dt in f32 int8; do
    for ring in 7 0; do
      THALLAMA_PERSIST_RING=$ring timeout -k 10 200 $B --dtype $dt > gpurun_out/ring_${dt}_${ring}_$r.json 2> gpurun_out/ring_${dt}_${ring}_$r.err || exit 1
      echo "$dt ring=$ring run $r: $(python -c "import json;d=json.load(open('gpurun_out/ring_${dt}_${ring}_$r.json'));print(d['ms_per_token'], d['value'], d['roofline']['frac'], d['reference_tokens']['match_prefix'])")"
    done
  done
done
