export TMPDIR=/tmp
L=hip_llama.cpp_amd/lib
cp $L/libthallama.so $L/libthallama.so.keep
for v in base u8 w8; do
  cp $L/libthallama.so.$v $L/libthallama.so
  echo "== $v"; timeout -k 10 200 python tools/mfma_sweep.py 8 || { cp $L/libthallama.so.keep $L/libthallama.so; exit 1; }
done
cp $L/libthallama.so.keep $L/libthallama.so
