#!/bin/bash
# A/B variant of libggd.so with extra defines in the persistent-loop unit (ggd_mega.hip):
#   bash scripts/build_variant.sh NAME "-DGGD_MK_FUSE_KD=1 -DGGD_MK_SPOLL=1"  -> ab/libggd_NAME.so
# (the other objects are the in-tree build's: run the normal build first)
cd "$(dirname "$0")/.." || exit 1
P=speech-driven-gesture-generation-using-transformer-based-denoising-diffusion-probabilistic-models_amd
mkdir -p ab /tmp/ggd_variant
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fno-slp-vectorize -Wno-unused-value -Wno-unused-result $2 \
  -c $P/csrc/ggd_mega.hip -o /tmp/ggd_variant/ggd_mega_$1.o || exit 1
objs=""
for s in ggd_kernels ggd_fused ggd_persist ggd_encoder ggd_train ggd_chain ggd_attn ggd_long ggd_api; do objs="$objs $P/build/$s.o"; done
hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/ggd_variant/ggd_mega_$1.o -o ab/libggd_$1.so && echo "ab/libggd_$1.so"
