#!/bin/bash
# A/B of library builds on ONE box (devices differ by a few % between calls):
#   TAG=r04x ROUNDS=2 bash scripts/ab.sh WORKLOAD LIB_A LIB_B ...
# runs bench.py --steps 3 (no CPU baseline, no f32 sub-record) for each library in turn, ROUNDS times,
# and prints the dominant kernel's average launch time per run.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-ab}
wl=$1
shift
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    out=gpurun_out/${T}_${wl}_$(basename $lib .so)_$r.json
    GGD_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline \
      --no-f32-subrecord --no-subrecords ${BENCH_ARGS} > $out 2> ${out%.json}.err || { echo "FAILED $lib"; tail -5 ${out%.json}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl', '$(basename $lib)', 'round $r', d['value'], 'frames/s', 'kernel_us', r['avg_launch_us'])"
  done
done
