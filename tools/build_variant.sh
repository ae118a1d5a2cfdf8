#!/usr/bin/env bash
# build_variant.sh NAME "-DFOO=1 ..." — lib/libthallama.so.NAME with persist.hip (or $SRC, e.g.
# SRC=persist_b) compiled under the given defines (every other object from the normal build), for
# same-box A/B runs.
set -e
cd "$(dirname "$0")/../hip_llama.cpp_amd"
name=$1; shift
src=${SRC:-persist}
mkdir -p /tmp/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=off -Wall -Wno-unused-function \
  -I../include $* -c csrc/$src.hip -o /tmp/variants/${src}_$name.o
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/libthallama.so.$name $objs /tmp/variants/${src}_$name.o
echo built lib/libthallama.so.$name
