set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03h}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -s tests/test_gpu_encoder.py > gpurun_out/${T}_enc_pytest.txt 2>&1 || { echo "encoder tests failed"; tail -30 gpurun_out/${T}_enc_pytest.txt; exit 1; }
tail -3 gpurun_out/${T}_enc_pytest.txt
for w in c5 c2; do
timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || { echo "bench $w failed"; tail -5 gpurun_out/${T}_${w}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_${w}_bench.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/${T}_prof.log; exit 1; }
f=$(find gpurun_out/${T}_prof -name '*kernel_stats.csv' | head -1)
cp $f gpurun_out/${T}_c5_kernel_stats.csv
head -30 gpurun_out/${T}_c5_kernel_stats.csv | cut -c1-200
rm -rf gpurun_out/${T}_prof
