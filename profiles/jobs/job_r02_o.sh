# fp32 batch-8 attention split sweep (THALLAMA_ATTN_SPLITS; auto = 1 at B=8 x 32 heads).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "s1:200:THALLAMA_ATTN_SPLITS=1 python bench.py --batch 8 --skip-cpu" \
 "s2:200:THALLAMA_ATTN_SPLITS=2 python bench.py --batch 8 --skip-cpu" \
 "s4:200:THALLAMA_ATTN_SPLITS=4 python bench.py --batch 8 --skip-cpu" \
 "s8:200:THALLAMA_ATTN_SPLITS=8 python bench.py --batch 8 --skip-cpu" \
 "s16:200:THALLAMA_ATTN_SPLITS=16 python bench.py --batch 8 --skip-cpu"
