# Same-box A/B of the matrix-core GEMV's 16-k steps per group (MFMA_U 4 = base, 8 = 512-B row runs)
# on the fp32 batch-8 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && L=hip_llama.cpp_amd/lib && cp $L/libthallama.so $L/libthallama.so.keep && \
for r in 1 2; do for v in base u8; do cp $L/libthallama.so.$v $L/libthallama.so && timeout -k 10 200 python bench.py --batch 8 --skip-cpu > gpurun_out/ab_$v$r.out 2>gpurun_out/ab_$v$r.err || { cp $L/libthallama.so.keep $L/libthallama.so; exit 1; }; done; done; cp $L/libthallama.so.keep $L/libthallama.so
