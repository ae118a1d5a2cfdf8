#!/usr/bin/env bash
# build_variant.sh NAME "-DFOO=1 ..." — lib/libthallama.so.NAME with persist.hip compiled under
# the given defines (every other object from the normal build), for same-box A/B runs.
set -e
cd "$(dirname "$0")/../hip_llama.cpp_amd"
name=$1; shift
mkdir -p /tmp/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=off -Wall -Wno-unused-function \
  -I../include $* -c csrc/persist.hip -o /tmp/variants/persist_$name.o
objs=$(ls build/*.o | grep -v '/persist.o')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/libthallama.so.$name $objs /tmp/variants/persist_$name.o
echo built lib/libthallama.so.$name
