#!/bin/bash
# A/B variant of libggd.so: one translation unit rebuilt with extra defines (or from its current
# source), every other object the in-tree build's:
#   bash scripts/build_variant.sh NAME "-DSOME_SWITCH=1" [UNIT]   -> ab/libggd_NAME.so
# DIAG=1 also links ab/libggd_NAME_diag.so (the ggd_diag build).  UNIT defaults to ggd_mega (the f32 clip-group loop; ggd_rows is the bf16 one); run the normal build first.
cd "$(dirname "$0")/.." || exit 1
P=speech-driven-gesture-generation-using-transformer-based-denoising-diffusion-probabilistic-models_amd
U=${3:-ggd_mega}
mkdir -p ab /tmp/ggd_variant
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fno-slp-vectorize -Wno-unused-value -Wno-unused-result $2 \
  -c $P/csrc/$U.hip -o /tmp/ggd_variant/${U}_$1.o || exit 1
objs=""
for s in ggd_kernels ggd_fused ggd_mega ggd_rows ggd_persist ggd_encoder ggd_train ggd_chain ggd_attn ggd_long ggd_api; do
  [ "$s" = "$U" ] || objs="$objs $P/build/$s.o"
done
hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/ggd_variant/${U}_$1.o -o ab/libggd_$1.so && echo "ab/libggd_$1.so" || exit 1
if [ -n "$DIAG" ]; then  # the stamp / microbenchmark build of the same variant (GGD_DIAG=1 GGD_LIB=...)
  dobjs=$(echo "$objs" | sed "s#$P/build/ggd_api.o#$P/build/ggd_api_diag.o $P/build/ggd_diag.o#")
  hipcc --offload-arch=gfx950 -shared -fPIC $dobjs /tmp/ggd_variant/${U}_$1.o -o ab/libggd_$1_diag.so && echo "ab/libggd_$1_diag.so"
fi
