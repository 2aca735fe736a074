set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03ad}
timeout -k 10 1500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${T}_pytest.txt 2>&1
echo "pytest rc=$?"
tail -2 gpurun_out/${T}_pytest.txt
grep -E "FAILED|ERROR" gpurun_out/${T}_pytest.txt | head -5 || true
for w in c4 c2 c5; do
timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || { echo "bench $w failed"; tail -5 gpurun_out/${T}_${w}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_${w}_bench.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
