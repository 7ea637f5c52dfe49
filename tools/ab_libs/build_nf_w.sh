#!/usr/bin/env bash
# Product-library clones of the narrow fused kernel at other wave counts and
# load-group depths (NF_WAVES, NF_UNR, NF_HU, NF_GA, NF_GV):
#   tools/ab_libs/build_nf_w.sh "12 2 1 4 2" "12 1 1 3 2"  ->  libmmb_nf_w12_2_1_4_2.so ...
# Each variant gets an object of its own (removed first), and the library's
# gfx950 code objects are checked for the instantiation the launcher runs:
# r05's hand-built libmmb_nf_w12_2_1_4_2.so lacked
# utt_narrow_fused_kernel<2,1,4,2,false> and the run aborted in HIP's launch
# ("Cannot find Symbol", gpurun_out r05be) -- a build script that was never
# committed.  This one fails loudly instead.
set -e
cd "$(dirname "$0")/../../multimodal-baselines_amd/csrc"
make -s all
OBJS="build/pc_kernels.o build/mm2_kernels.o build/mlp_kernels.o build/latent_kernels.o build/probe_kernels.o build/host_rng.o"
LLVM=/opt/rocm/lib/llvm/bin
for c in "$@"; do
  set -- $c
  tag=w$1_$2_$3_$4_$5
  o=build/nf_$tag.o
  lib=$(cd ../../tools/ab_libs && pwd)/libmmb_nf_$tag.so
  rm -f "$o" "$lib"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I/opt/rocm/include \
    -Wall -Wno-unused-function -DNF_WAVES=$1 -DNF_UNR=$2 -DNF_HU=$3 -DNF_GA=$4 -DNF_GV=$5 \
    -c sif_kernels.hip -o "$o"
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$lib" "$o" $OBJS
  sym="_ZN3mmb23utt_narrow_fused_kernelILi$2ELi$3ELi$4ELi$5ELb0EEEvNS_15NarrowFusedArgsE"
  tmp=$(mktemp -d)
  cp "$lib" "$tmp/lib.so"
  (cd "$tmp" && $LLVM/llvm-objdump --offloading lib.so > /dev/null)
  if for co in "$tmp"/lib.so.*gfx950*; do $LLVM/llvm-readelf --symbols "$co"; done | grep -q "$sym"; then
    echo "built libmmb_nf_$tag.so ($sym in the gfx950 code object)"
  else
    echo "libmmb_nf_$tag.so: $sym MISSING from the gfx950 code object" >&2
    rm -rf "$tmp" "$lib"; exit 1
  fi
  rm -rf "$tmp"
done
