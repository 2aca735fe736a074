# round-4 GPU call (r04r): per-clip loops with the QKV conv in registers -- their tests, then C5 A/B
T=r04r
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "pair or psk or persist or unresident or eps_routes or c5 or prefetch" > gpurun_out/${T}_pytest.txt 2>&1
tail -2 gpurun_out/${T}_pytest.txt; grep -E "^FAILED|psk_bf16 t=|pair_bf16 t=" gpurun_out/${T}_pytest.txt | head -14
TAG=$T ROUNDS=2 bash scripts/ab.sh c5 ab/libggd_pskc0.so ab/libggd_pskc1.so
