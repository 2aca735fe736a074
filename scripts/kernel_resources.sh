#!/bin/bash
# VGPR / AGPR / SGPR / scratch of every gfx950 kernel of the given csrc files (CPU only).
cd "$(dirname "$0")/../speech-driven-gesture-generation-using-transformer-based-denoising-diffusion-probabilistic-models_amd/csrc" || exit 1
B=/opt/rocm/lib/llvm/bin
for f in ${@:-ggd_fused.hip}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -Wno-unused-value -Wno-unused-result --cuda-device-only \
    --no-gpu-bundle-output -c $f -o /tmp/$f.co || exit 1
  $B/llvm-readelf --notes /tmp/$f.co | grep -E "^ +\.name:|\.vgpr_count:|\.private_segment_fixed_size:|\.sgpr_count:|\.agpr_count:" |
    awk '/\.agpr_count/{a=$2} /\.name:/{n=$2} /private_segment/{p=$2} /sgpr_count/{s=$2} /vgpr_count/{v=$2; printf "%-56s vgpr %4s agpr %4s sgpr %4s scratch %6s\n", substr(n,1,56), v, a, s, p}'
done
