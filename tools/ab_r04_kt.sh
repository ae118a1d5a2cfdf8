#!/usr/bin/env bash
# Round-4 same-box A/B of the attention window's K layout (attention.hpp ATTN_K_TRANSPOSED 0 / 1,
# lib/libthallama.so.kt0 / .kt1 from tools/build_variant.sh): stories110M B=1 and llama2-7B B=1
# with the long-context tail, two rounds, interleaved.  Restores the library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
L=hip_llama.cpp_amd/lib
cp $L/libthallama.so $L/libthallama.so.keep
B="python bench.py --skip-cpu --no-requests-point --warmup 1 --prof-steps 4"
for r in 1 2; do
  for v in kt0 kt1; do
    cp $L/libthallama.so.$v $L/libthallama.so
    timeout -k 10 200 $B --model 110m --steps 5 > gpurun_out/kt_110m_${v}_$r.json 2> gpurun_out/kt_110m_${v}_$r.err || { cp $L/libthallama.so.keep $L/libthallama.so; exit 1; }
    timeout -k 10 300 $B --steps 2 > gpurun_out/kt_7b_${v}_$r.json 2> gpurun_out/kt_7b_${v}_$r.err || { cp $L/libthallama.so.keep $L/libthallama.so; exit 1; }
    python - "$v" "$r" <<'PY'
import json, sys
v, r = sys.argv[1:]
a = json.load(open(f"gpurun_out/kt_110m_{v}_{r}.json")); b = json.load(open(f"gpurun_out/kt_7b_{v}_{r}.json"))
print(v, r, "110m", a["value"], a["reference_tokens"]["match_prefix"], "7b", b["value"], "long", b["long_context"]["value"],
      b["long_context"]["reference_tokens"]["match_prefix"], flush=True)
PY
  done
done
cp $L/libthallama.so.keep $L/libthallama.so
