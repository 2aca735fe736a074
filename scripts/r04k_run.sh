# round-4 GPU call (r04s): per-clip loops with transposed out-projection / FFN epilogues (pskt1) and
# + the convolved cross-attention queries read in place (pskq) -- tests on pskq, then C5 A/B
T=r04s
GGD_LIB=ab/libggd_pskq.so timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "pair or psk or persist or unresident or eps_routes or c5 or prefetch or generator" > gpurun_out/${T}_pytest.txt 2>&1
tail -2 gpurun_out/${T}_pytest.txt; grep -E "^FAILED|psk_bf16 t=|pair_bf16 t=" gpurun_out/${T}_pytest.txt | head -14
TAG=$T ROUNDS=2 bash scripts/ab.sh c5 ab/libggd_pskt0.so ab/libggd_pskt1.so ab/libggd_pskq.so
