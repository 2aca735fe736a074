cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
for ov in on off; do
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --overlap $ov > gpurun_out/c5_ov_$ov.log 2>&1 || exit 1
python -c "import json;d=json.loads(open('gpurun_out/c5_ov_$ov.log').read().strip().splitlines()[-1]);print('$ov', d['value'], d['ms_per_step'], d['roofline']['kernel'][:40], d['roofline']['avg_launch_us'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o run --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5prof.log 2>&1 || exit 1
python scripts/c5_timeline.py gpurun_out/c5prof
