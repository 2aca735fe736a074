set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03ae}
WORKLOADS="c2 c5 c4" bash scripts/pmc_all.sh $T || { echo "pmc failed"; exit 1; }
for w in c2 c5 c4; do
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail -5 gpurun_out/${T}_prof_$w.log; exit 1; }
f=$(find gpurun_out/${T}_prof_$w -name '*kernel_stats.csv' | head -1)
cp $f gpurun_out/${T}_${w}_kernel_stats.csv
head -2 gpurun_out/${T}_${w}_kernel_stats.csv | tail -1 | cut -c1-140
rm -rf gpurun_out/${T}_prof_$w
done
