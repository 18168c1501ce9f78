#!/bin/bash
# Profiling-build ablations of the band conv main loop (results INVALID, timing only):
# lib/abl<N>/libdroid_hip.so with DROID_CONV_ABLATE=N (bit 0: no stage barrier, bit 1: no DMA after stage 0, bit 2: no DMA waits)
set -e
cd "$(dirname "$0")/../droid-slam_amd/csrc"
make -j8 prof > /dev/null
for n in 1 2 3 4; do
  d=../lib/abl$n; mkdir -p $d/obj
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DDROID_CONV_PROFILE=1 -DDROID_CONV_ABLATE=$n -x hip -c conv_kernels.hip -o $d/obj/conv_kernels.o &
done
wait
for n in 1 2 3 4; do
  d=../lib/abl$n
  objs=$(ls ../lib/prof/obj/*.o | grep -v conv_kernels.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libdroid_hip.so $objs $d/obj/conv_kernels.o
done
