#!/bin/bash
# Build (here) or run (GPU box) the DIA-walk ablation binaries of walk_micro.
#   bash tools/micro/walk_ab.sh build   -> tools/micro/walk_ab/walk_micro_<AB>
#   bash tools/micro/walk_ab.sh run [n] -> one line pair per build
ABS=${ABS:-"0 1 2 6 8 16 32 63"}
d=tools/micro/walk_ab
if [ "$1" = build ]; then
  mkdir -p $d
  for ab in $ABS; do
    hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -x hip -I/opt/rocm/include \
      -DKR_DIAW_AB=$ab -o $d/walk_micro_$ab tools/micro/walk_micro.cpp &
  done
  wait
else
  for ab in $ABS; do
    timeout -k 10 120 $d/walk_micro_$ab ${2:-50000000} 10 || exit $?
  done
fi
