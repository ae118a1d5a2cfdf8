# Same-box A/B of the persistent step's XCD skew (rows dealt 100+s : 100-s to even : odd blocks;
# s = 4 is the default) on the fp32 headline and the int8 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && L=hip_llama.cpp_amd/lib && cp $L/libthallama.so $L/libthallama.so.keep && \
for r in 1 2; do for v in sk4 sk6 sk8 sk11; do cp $L/libthallama.so.$v $L/libthallama.so && timeout -k 10 200 python bench.py --skip-cpu > gpurun_out/ab_$v$r.out 2>gpurun_out/ab_$v$r.err && timeout -k 10 200 python bench.py --skip-cpu --dtype int8 > gpurun_out/abq_$v$r.out 2>gpurun_out/abq_$v$r.err || { cp $L/libthallama.so.keep $L/libthallama.so; exit 1; }; done; done; cp $L/libthallama.so.keep $L/libthallama.so
