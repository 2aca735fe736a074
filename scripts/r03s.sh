set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03s}
WORKLOADS="c2 c5 c4" bash scripts/pmc_all.sh $T || { echo "pmc failed"; exit 1; }
for w in c2 c5 c4; do
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail -5 gpurun_out/${T}_prof_$w.log; exit 1; }
f=$(find gpurun_out/${T}_prof_$w -name '*kernel_stats.csv' | head -1)
cp $f gpurun_out/${T}_${w}_kernel_stats.csv
head -3 gpurun_out/${T}_${w}_kernel_stats.csv | cut -c1-160
rm -rf gpurun_out/${T}_prof_$w
done
B=32
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_enc$B -o run --output-format csv -- python3 scripts/enc_trace.py $B > gpurun_out/${T}_enc$B.log 2>&1 || { echo "trace $B failed"; exit 1; }
python3 scripts/enc_trace.py --report gpurun_out/${T}_enc$B > gpurun_out/${T}_enc${B}_trace.txt
rm -rf gpurun_out/${T}_enc$B
tail -1 gpurun_out/${T}_enc${B}_trace.txt
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4_bench.json 2> gpurun_out/${T}_c4_bench.err || { echo "bench c4 failed"; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_c4_bench.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
