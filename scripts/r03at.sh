set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03ay}
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused_ke.py > gpurun_out/${T}_fused_pytest.txt 2>&1
rc=$?
echo "fused pytest rc=$rc"
tail -2 gpurun_out/${T}_fused_pytest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_fused_pytest.txt | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_c2_bench.json 2> gpurun_out/${T}_c2_bench.err || { echo "bench failed"; tail -5 gpurun_out/${T}_c2_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_c2_bench.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
timeout -k 10 300 python -u scripts/mega_stamps.py > gpurun_out/${T}_stamps.txt 2>&1
echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/${T}_stamps.txt | tail -7 | cut -c1-400
