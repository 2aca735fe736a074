set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03ag}
timeout -k 10 300 python -u bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_c2_bench.json 2> gpurun_out/${T}_c2_bench.err || { echo "bench failed"; tail -5 gpurun_out/${T}_c2_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_c2_bench.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
timeout -k 10 300 python -u scripts/mega_stamps.py > gpurun_out/${T}_stamps.txt 2>&1
echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/${T}_stamps.txt | tail -8
timeout -k 10 300 python -u scripts/mega_arrivals.py > gpurun_out/${T}_arrivals.txt 2>&1
echo "arrivals rc=$?"
grep -v amdgpu.ids gpurun_out/${T}_arrivals.txt | tail -6
