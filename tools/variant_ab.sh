#!/usr/bin/env bash
# Same-box A/B of library variants lib/libthallama.so.<v> (tools/build_variant.sh): for each
# round and variant, swap it in and run the bench line given in BENCH_ARGS; restores the library.
# Usage: tools/variant_ab.sh "va vb" [rounds]   (AB_LONG=" " adds the long-context line)   (env per variant: VARIANT_ENV_<v>="K=V ...")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
L=hip_llama.cpp_amd/lib
cp $L/libthallama.so $L/libthallama.so.keep
B="python bench.py --skip-cpu ${AB_LONG:---no-long} --no-requests-point --steps 2 --warmup 1 --prof-steps 4 $BENCH_ARGS"
for r in $(seq 1 ${2:-2}); do
  for v in $1; do
    cp $L/libthallama.so.$v $L/libthallama.so
    ev="VARIANT_ENV_$v"
    env ${!ev} timeout -k 10 200 $B > gpurun_out/var_${v}_$r.json 2> gpurun_out/var_${v}_$r.err || { cp $L/libthallama.so.keep $L/libthallama.so; exit 1; }
    echo "$v run $r: $(python -c "import json;d=json.load(open('gpurun_out/var_${v}_$r.json'));print(d['ms_per_token'], d['value'], d['roofline']['frac'], d['reference_tokens']['match_prefix'], (d.get('long_context') or {}).get('value'))")"
  done
done
cp $L/libthallama.so.keep $L/libthallama.so
