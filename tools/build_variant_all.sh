#!/usr/bin/env bash
# build_variant_all.sh NAME "-DFOO=1 ..." — lib/libthallama.so.NAME with EVERY HIP source compiled
# under the given defines (objects in /tmp/variants/NAME), for same-box A/B runs.
set -e
cd "$(dirname "$0")/../hip_llama.cpp_amd"
name=$1; shift
out=/tmp/variants/$name; mkdir -p $out
for f in csrc/*.hip; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=off -Wall -Wno-unused-function \
    -I../include $* -c $f -o $out/$b.o &
  while [ $(jobs -r | wc -l) -ge 8 ]; do sleep 1; done
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/libthallama.so.$name $out/*.o
echo built lib/libthallama.so.$name
