set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03az}
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_training.py > gpurun_out/${T}_training_pytest.txt 2>&1
rc=$?
echo "training pytest rc=$rc"; tail -2 gpurun_out/${T}_training_pytest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_training_pytest.txt | head -20; exit 1; }
WORKLOADS="c5" bash scripts/pmc_all.sh $T || { echo "pmc failed"; exit 1; }
for w in c5; do
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail -5 gpurun_out/${T}_prof_$w.log; exit 1; }
f=$(find gpurun_out/${T}_prof_$w -name '*kernel_stats.csv' | head -1)
cp $f gpurun_out/${T}_${w}_kernel_stats.csv
head -2 gpurun_out/${T}_${w}_kernel_stats.csv | tail -1 | cut -c1-140
rm -rf gpurun_out/${T}_prof_$w
done
cp gpurun_out/${T}_pmc_c5_summary.json profiles/
sed -i 's/"c5": "r03ae"/"c5": "'${T}'"/' bench.py
timeout -k 10 500 python -u bench.py --workload c5 > gpurun_out/${T}_c5_bench.json 2> gpurun_out/${T}_c5_bench.err || { echo "bench failed"; tail -5 gpurun_out/${T}_c5_bench.err; exit 1; }
cut -c1-400 gpurun_out/${T}_c5_bench.json
