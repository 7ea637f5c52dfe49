#!/usr/bin/env bash
# Product-library clones with the narrow fused kernel's knobs (NF_UNR: cold
# words per load group, NF_HU: hot words per LDS group, optional NF_ABL:
# timing-only ablation bits):
#   tools/ab_libs/build_nf.sh "4 1" "4 1 2"  ->  libmmb_nf_4_1.so libmmb_nf_4_1_a2.so
set -e
cd "$(dirname "$0")/../../multimodal-baselines_amd/csrc"
make -s all
OBJS="build/pc_kernels.o build/mm2_kernels.o build/mlp_kernels.o build/latent_kernels.o build/probe_kernels.o build/host_rng.o"
for c in "$@"; do
  set -- $c
  tag=$1_$2; abl=${3:-0}; [ "$abl" != 0 ] && tag=${tag}_a$abl
  o=build/nf_$tag.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I/opt/rocm/include \
    -Wall -Wno-unused-function -DNF_UNR=$1 -DNF_HU=$2 -DNF_ABL=$abl -c sif_kernels.hip -o $o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/ab_libs/libmmb_nf_$tag.so $o $OBJS
  echo "built libmmb_nf_$tag.so"
done
