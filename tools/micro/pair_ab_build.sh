#!/bin/bash
# Timing-only A/B libraries of the box pair (kr_pair.hip, KR_ST2B_AB bits):
# only kr_pair.o is rebuilt, linked with the library's other objects.
#   bash tools/micro/pair_ab_build.sh 1 2 4 8  ->  parallel-krylov_amd/libkrylov_amd_ab<N>.so
set -e
cd "$(dirname "$0")/../../parallel-krylov_amd/csrc"
make -s -j8 >/dev/null
objs=$(ls build/*.o | grep -v kr_pair.o)
for ab in "$@"; do
  mkdir -p build_ab$ab
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I/opt/rocm/include \
      -DKR_ST2B_AB=$ab -DKR_ALLOW_WRONG_RESULTS $EXTRA -c kr_pair.hip -o build_ab$ab/kr_pair.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib \
      -o ../libkrylov_amd_ab$ab.so $objs build_ab$ab/kr_pair.o
  echo "built libkrylov_amd_ab$ab.so"
done
