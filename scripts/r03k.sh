set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03k}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -s tests/test_gpu_encoder.py > gpurun_out/${T}_enc_pytest.txt 2>&1 || { echo "encoder tests failed"; tail -30 gpurun_out/${T}_enc_pytest.txt; exit 1; }
grep -E "PASSED|FAILED|err|rel" gpurun_out/${T}_enc_pytest.txt | tail -12
B=128
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_enc$B -o run --output-format csv -- python3 scripts/enc_trace.py $B > gpurun_out/${T}_enc$B.log 2>&1 || { echo "trace $B failed"; tail -5 gpurun_out/${T}_enc$B.log; exit 1; }
python3 scripts/enc_trace.py --report gpurun_out/${T}_enc$B > gpurun_out/${T}_enc${B}_trace.txt
rm -rf gpurun_out/${T}_enc$B
tail -1 gpurun_out/${T}_enc${B}_trace.txt
for w in c5 c2; do
timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || { echo "bench $w failed"; tail -5 gpurun_out/${T}_${w}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_${w}_bench.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
