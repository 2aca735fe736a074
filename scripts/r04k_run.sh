# round-4 GPU call (r04n): full suite on the new defaults (fused last-layer KD, coalesced KE update,
# block-scaled fp8 long loop, multi-tile encoder convs), encoder tiling A/B on C5 / C2, the C4 line
# with fp8 MFMA (FFN / projections; + the attention out-projections: mxr) and widened, the C2 line
T=r04n
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest.txt 2>&1; tail -3 gpurun_out/${T}_pytest.txt; grep -E "FAILED|rel-RMS" gpurun_out/${T}_pytest.txt | grep -E "FAILED|lk_fp8|fp8 long" | head -20
for r in 1 2; do
  for mt in 1 0; do
    out=gpurun_out/${T}_c5_mt${mt}_$r.json
    GGD_ENC_CONV_MT=$mt timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $out 2> ${out%.json}.err || { tail -5 ${out%.json}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('c5 mt=$mt', d['value'], 'ms/pass', d['ms_per_step'], 'kernel_us', d['roofline']['avg_launch_us'])"
  done
done
for mt in 1 0; do
  out=gpurun_out/${T}_c2_mt${mt}.json
  GGD_ENC_CONV_MT=$mt timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord > $out 2> ${out%.json}.err || { tail -5 ${out%.json}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('c2 mt=$mt', d['value'], 'ms/pass', d['ms_per_step'], 'kernel_us', d['roofline']['avg_launch_us'])"
done
TAG=$T ROUNDS=2 bash scripts/ab.sh c4 ab/libggd_mx.so ab/libggd_mxr.so
TAG=${T}w BENCH_ARGS="--steps 3 --no-cpu-baseline --no-fp8-mfma" bash scripts/gpu.sh bench:c4
TAG=$T bash scripts/gpu.sh bench:c2
