#!/usr/bin/env bash
# Product-library clones with MMB_SQ_PER_WG (G2 tiles per squaring workgroup
# of the PC solve's launch):  tools/ab_libs/build_sq.sh 2 4  ->  libmmb_sq2.so libmmb_sq4.so
set -e
cd "$(dirname "$0")/../../multimodal-baselines_amd/csrc"
make -s all
OBJS="build/sif_kernels.o build/mm2_kernels.o build/mlp_kernels.o build/latent_kernels.o build/probe_kernels.o build/host_rng.o"
for v in "$@"; do
  o=build/pc_sq$v.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I/opt/rocm/include \
    -Wall -Wno-unused-function -DMMB_SQ_PER_WG=$v -c pc_kernels.hip -o $o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/ab_libs/libmmb_sq$v.so $o $OBJS
  echo "built libmmb_sq$v.so"
done
