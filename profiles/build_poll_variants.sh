#!/bin/bash
# Tuning builds of the engine's polling shape: the two
# engine units compiled with -DKBHIP_POLL_DEPTH=D -DKBHIP_POLL_SLEEP=S and
# linked with the product's other objects into _build/libkbhip_pD_sS.so
# (run here, on the CPU, after `make`; loaded on the GPU box with KBHIP_LIB).
# usage: bash profiles/build_poll_variants.sh "D:S D:S ..."
set -e
cd "$(dirname "$0")/../kube-batch-1_amd"
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-function"
OBJS="_build/kbhip_kernels_p1.o _build/kbhip_kernels_p2.o _build/kbhip_kernels_p3.o _build/kbhip_evict.o \
      $(ls _build/session_*.o) _build/kbhip_affinity.o"
for v in ${1:-"1:1 2:0 8:2"}; do
  D=${v%%:*}; S=${v##*:}
  T=$(mktemp -d)
  /opt/rocm/bin/hipcc $FLAGS -DKBHIP_POLL_DEPTH=$D -DKBHIP_POLL_SLEEP=$S -c csrc/kbhip_engine.hip -o $T/e.o &
  /opt/rocm/bin/hipcc $FLAGS -DKBHIP_POLL_DEPTH=$D -DKBHIP_POLL_SLEEP=$S -c csrc/kbhip_engine_lists.hip -o $T/l.o &
  wait
  /opt/rocm/bin/hipcc $FLAGS -shared -o _build/libkbhip_p${D}_s${S}.so $OBJS $T/e.o $T/l.o -L/opt/rocm/lib -lrccl
  rm -rf $T
  echo "_build/libkbhip_p${D}_s${S}.so"
done
