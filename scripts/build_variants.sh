#!/bin/bash
# A/B builds of conv_kernels.hip: lib/v_<name>/libdroid_hip.so = the regular
# objects + conv_kernels.o compiled with extra -D flags.
#   bash scripts/build_variants.sh name1 "-DFOO=1" name2 "-DBAR=0 -DBAZ=1" ...
set -e
cd "$(dirname "$0")/../droid-slam_amd/csrc"
make -j8 > /dev/null
args=("$@")
for ((i = 0; i < ${#args[@]}; i += 2)); do
  d=../lib/v_${args[i]}; mkdir -p $d/obj
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 ${args[i+1]} -x hip -c conv_kernels.hip -o $d/obj/conv_kernels.o &
done
wait
for ((i = 0; i < ${#args[@]}; i += 2)); do
  d=../lib/v_${args[i]}
  objs=$(ls ../lib/obj/*.o | grep -v conv_kernels.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libdroid_hip.so $objs $d/obj/conv_kernels.o
done
