#!/usr/bin/env bash
# Product-library clones with the split stream's build constants:
#   tools/ab_libs/build_split.sh "16 1" "8 2" "8 1 32"  ->  libmmb_split_tu16_x1.so libmmb_split_tu8_x2.so libmmb_split_tu8_x1_fu32.so
# (MMB_SPLIT_TU text rows in flight per thread group, MMB_SPLIT_TEXT_X text
# ranges per frame range of the automatic plan, MMB_SPLIT_FU frame rows in flight)
set -e
cd "$(dirname "$0")/../../multimodal-baselines_amd/csrc"
make -s all
OBJS="build/pc_kernels.o build/mm2_kernels.o build/mlp_kernels.o build/latent_kernels.o build/probe_kernels.o build/host_rng.o"
for c in "$@"; do
  set -- $c
  fu=${3:-16}
  tag=tu$1_x$2; [ "$fu" != 16 ] && tag=${tag}_fu$fu; o=build/split_$tag.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I/opt/rocm/include \
    -Wall -Wno-unused-function -DMMB_SPLIT_TU=$1 -DMMB_SPLIT_TEXT_X=$2 -DMMB_SPLIT_FU=$fu -c sif_kernels.hip -o $o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/ab_libs/libmmb_split_$tag.so $o $OBJS
  echo "built libmmb_split_$tag.so"
done
