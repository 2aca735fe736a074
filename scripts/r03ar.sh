set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03ar}
WORKLOADS="c2" bash scripts/pmc_all.sh $T || { echo "pmc failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2 -o run --output-format csv -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_prof_c2.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/${T}_prof_c2.log; exit 1; }
f=$(find gpurun_out/${T}_prof_c2 -name '*kernel_stats.csv' | head -1)
cp $f gpurun_out/${T}_c2_kernel_stats.csv
rm -rf gpurun_out/${T}_prof_c2
head -2 gpurun_out/${T}_c2_kernel_stats.csv | tail -1 | cut -c1-140
cp gpurun_out/${T}_pmc_c2_summary.json profiles/ 2>/dev/null
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_c2_bench.json 2> gpurun_out/${T}_c2_bench.err || { echo "bench failed"; tail -5 gpurun_out/${T}_c2_bench.err; exit 1; }
cut -c1-300 gpurun_out/${T}_c2_bench.json
