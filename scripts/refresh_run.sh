# round-4 refresh of the older evidence on the final tree (r04v): C1 line, training step (B = 64,
# encoder trained), encoder kernel traces at 32 and 128 clips
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
T=r04v
TAG=$T BENCH_ARGS="--steps 2" bash scripts/gpu.sh bench:c1 || exit 1
timeout -k 10 300 python3 -u scripts/train_bench.py 64 10 full > gpurun_out/${T}_train_bench.txt 2>&1 || { tail -5 gpurun_out/${T}_train_bench.txt; exit 1; }
tail -3 gpurun_out/${T}_train_bench.txt
for B in 32 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_enc_$B -o run --output-format csv -- python3 scripts/enc_trace.py $B \
    > gpurun_out/${T}_enc_$B.log 2>&1 || { tail -5 gpurun_out/${T}_enc_$B.log; exit 1; }
  python3 scripts/enc_trace.py --report gpurun_out/${T}_enc_$B > gpurun_out/${T}_encoder_b${B}_trace.txt && rm -rf gpurun_out/${T}_enc_$B
  tail -1 gpurun_out/${T}_encoder_b${B}_trace.txt
done
# the hipGraph-captured per-step route at C5's shape (BASELINE configs[4]'s wording), for comparison
TAG=${T}g BENCH_ARGS="--steps 2 --graph --no-cpu-baseline --no-profile" bash scripts/gpu.sh bench:c5
