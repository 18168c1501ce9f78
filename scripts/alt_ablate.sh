# Timing ablations of corr_alt_ce0_kernel (DROID_ALT_ABL bits, see the kernel):
# builds droid-slam_amd/lib/abl<k>/libdroid_hip.so for each mask given
# (ALT_PROF=1: profiling builds with the stage stamps, for scripts/alt_timeline.py).
set -e
cd "$(dirname "$0")/../droid-slam_amd/csrc"
extra=""; objdir=../lib/obj
if [ "${ALT_PROF:-0}" = 1 ]; then extra="-DDROID_CONV_PROFILE=1"; objdir=../lib/prof/obj; fi
for k in "$@"; do
  mkdir -p ../lib/abl$k
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $extra -DDROID_ALT_ABL=$k -x hip -c corr_alt_kernels.hip -o ../lib/abl$k/corr_alt_kernels.o
  objs=$(ls $objdir/*.o | grep -v corr_alt_kernels)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib/abl$k/libdroid_hip.so $objs ../lib/abl$k/corr_alt_kernels.o
done
