set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03ba}
WORKLOADS="c4" bash scripts/pmc_all.sh $T || { echo "pmc failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c4 -o run --output-format csv -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_prof_c4.log 2>&1 || { echo "rocprof c4 failed"; tail -5 gpurun_out/${T}_prof_c4.log; exit 1; }
f=$(find gpurun_out/${T}_prof_c4 -name '*kernel_stats.csv' | head -1)
cp $f gpurun_out/${T}_c4_kernel_stats.csv
head -2 gpurun_out/${T}_c4_kernel_stats.csv | tail -1 | cut -c1-140
rm -rf gpurun_out/${T}_prof_c4
cp gpurun_out/${T}_pmc_c4_summary.json profiles/
sed -i 's/"c4": "r03ae"/"c4": "'${T}'"/' bench.py
timeout -k 10 500 python -u bench.py --workload c4 > gpurun_out/${T}_c4_bench.json 2> gpurun_out/${T}_c4_bench.err || { echo "bench failed"; tail -5 gpurun_out/${T}_c4_bench.err; exit 1; }
cut -c1-400 gpurun_out/${T}_c4_bench.json
