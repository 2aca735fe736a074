# training-step profile (r04w): kernel stats of 5 timed steps (B = 64, encoder trained)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
T=r04w
timeout -k 10 300 python3 -u scripts/train_bench.py 64 10 full > gpurun_out/${T}_train_bench.txt 2>&1 || { tail -5 gpurun_out/${T}_train_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_train_bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trprof -o tr -- python3 -u scripts/train_bench.py 64 5 full > gpurun_out/${T}_train_prof.log 2>&1 || { tail -5 gpurun_out/${T}_train_prof.log; exit 1; }
tail -1 gpurun_out/${T}_train_prof.log
f=$(find gpurun_out/${T}_trprof -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/${T}_train_kernel_stats.csv
head -25 gpurun_out/${T}_train_kernel_stats.csv | cut -c1-160
