set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03i}
run() {  # name, extra args
  timeout -k 10 300 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline --no-f32-subrecord $2 > gpurun_out/${T}_$1.json 2> gpurun_out/${T}_$1.err || { echo "bench $1 failed"; tail -5 gpurun_out/${T}_$1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$1.json')); print('$1', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
}
run c2_serial "" && run c2_overlap "--overlap on" && GGD_ENC_CONV_DIRECT=1 run c2_overlap_direct "--overlap on"
