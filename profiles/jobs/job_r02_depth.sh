# B=8 matrix-core GEMV split depth (THALLAMA_MFMA_DEPTH blocks per CU; 4 = default), same box, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "d4a:200:THALLAMA_MFMA_DEPTH=4 python bench.py --batch 8 --skip-cpu" \
 "d2a:200:THALLAMA_MFMA_DEPTH=2 python bench.py --batch 8 --skip-cpu" \
 "d3a:200:THALLAMA_MFMA_DEPTH=3 python bench.py --batch 8 --skip-cpu" \
 "d6a:200:THALLAMA_MFMA_DEPTH=6 python bench.py --batch 8 --skip-cpu" \
 "d8a:200:THALLAMA_MFMA_DEPTH=8 python bench.py --batch 8 --skip-cpu" \
 "d4b:200:THALLAMA_MFMA_DEPTH=4 python bench.py --batch 8 --skip-cpu" \
 "d3b:200:THALLAMA_MFMA_DEPTH=3 python bench.py --batch 8 --skip-cpu" \
 "d6b:200:THALLAMA_MFMA_DEPTH=6 python bench.py --batch 8 --skip-cpu"
