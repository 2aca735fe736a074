set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03z}
for w in ${WL:-c2}; do
timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || { echo "bench $w failed"; tail -5 gpurun_out/${T}_${w}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_${w}_bench.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
timeout -k 10 300 python -u scripts/mega_stamps.py > gpurun_out/${T}_stamps.txt 2>&1
echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/${T}_stamps.txt | tail -6
