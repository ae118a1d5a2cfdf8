#!/usr/bin/env bash
# Round-4 sweep of the persistent step's Infinity-Cache weight prefetch (THALLAMA_PERSIST_PF =
# slots per streaming wave, persist.hip prefetch_slots): llama2-7B fp32 B=1 (with the long-context
# tail) and int8 B=1, interleaved, one line each with tok/s and the reference-token prefix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B="python bench.py --skip-cpu --no-requests-point --warmup 1 --prof-steps 4"
for pf in ${PF_LIST:-0 2 4 8}; do
  THALLAMA_PERSIST_PF=$pf timeout -k 10 300 $B --steps 2 > gpurun_out/pf_f32_$pf.json 2> gpurun_out/pf_f32_$pf.err || exit 1
  THALLAMA_PERSIST_PF=$pf timeout -k 10 300 $B --steps 3 --dtype int8 --no-long > gpurun_out/pf_int8_$pf.json 2> gpurun_out/pf_int8_$pf.err || exit 1
  python - "$pf" <<'PY'
import json, sys
pf = sys.argv[1]
a = json.load(open(f"gpurun_out/pf_f32_{pf}.json")); b = json.load(open(f"gpurun_out/pf_int8_{pf}.json"))
print("pf", pf, "f32", a["value"], a["roofline"]["frac"], a["reference_tokens"]["match_prefix"], "long", a["long_context"]["value"],
      a["long_context"]["reference_tokens"]["match_prefix"], "| int8", b["value"], b["roofline"]["frac"] if b["roofline"] else None,
      b["reference_tokens"]["match_prefix"], flush=True)
PY
done
