#!/bin/bash
# Build A/B variants of libmoegan_hip.so that differ only in mg_gemm.hip compile flags.
#   tools/build_variants.sh name1 "-DFLAG=.." name2 "-DFLAG=.." ...
# (SRC=<file.hip> varies another source; default mg_gemm.hip)
# -> moe-gan_cpsc541_amd/moegan_mi/libmoegan_hip_<name>.so  (select with MOEGAN_HIP_LIB=<path>)
set -e
cd "$(dirname "$0")/../moe-gan_cpsc541_amd/csrc"
make -s >/dev/null
OBJ=../../build/obj
SRC=${SRC:-mg_gemm.hip}
B=${SRC%.hip}
mkdir -p ../../build/var
pids=()
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-function $f \
      -c $SRC -o ../../build/var/${B}_$n.o 2>&1 | { grep -v hip-link || true; }
    objs=$(ls $OBJ/*.o | grep -v "/$B.o")
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../moegan_mi/libmoegan_hip_$n.so $objs ../../build/var/${B}_$n.o \
      2>&1 | { grep -v hip-link || true; }; echo "built $n" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
