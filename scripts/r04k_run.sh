# round-4 GPU call (r04o): fp8-MFMA long loop with the transposed F1 epilogue + DPP block maxima:
# its eps / MX-oracle tests, then A/B on C4: fp8 MFMA (mx), + block-scaled attention out-projections
# (mxr), widened (--no-fp8-mfma); then the C2 loop's phase stamps
T=r04o
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "lk or fp8 or long" \
  > gpurun_out/${T}_fp8_pytest.txt 2>&1; tail -2 gpurun_out/${T}_fp8_pytest.txt; grep -E "FAILED|lk_fp8 t=|MX oracle|fp8 long" gpurun_out/${T}_fp8_pytest.txt | head -24
TAG=$T ROUNDS=2 bash scripts/ab.sh c4 ab/libggd_mx.so ab/libggd_mxr.so
TAG=${T}w BENCH_ARGS="--steps 3 --no-cpu-baseline --no-fp8-mfma" bash scripts/gpu.sh bench:c4
TAG=$T bash scripts/gpu.sh stamps
