set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03t}
for w in c1 c5 c4; do
timeout -k 10 500 python -u bench.py --workload $w --steps 3 --warmup 1 > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || { echo "bench $w failed"; tail -5 gpurun_out/${T}_${w}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_${w}_bench.json')); print('$w', d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['cpu_baseline']['value'], d['cpu_baseline']['sample'][:150])"
done
