#!/bin/bash
# One parameterised GPU runner (replaces the per-experiment r0N*.sh wrappers).
#
#   TAG=r04a bash scripts/gpu.sh STEP [STEP ...]
#
# Steps (each under its own time limit; the script stops at the first failure):
#   tests[:EXPR]      pytest -m gpu (optionally -k EXPR)            -> gpurun_out/$TAG_pytest.txt
#   smoke             __graft_entry__.smoke()                       -> gpurun_out/$TAG_smoke.log
#   bench[:WL]        bench.py line for workload WL (default c2)    -> gpurun_out/$TAG_WL_bench.json
#   quick[:WL]        bench.py --steps 3, no CPU baseline / f32 sub-record
#   prof[:WL]         rocprofv3 --kernel-trace --stats               -> gpurun_out/$TAG_WL_kernel_stats.csv
#   pmc[:WL]          HBM / SQ counter passes (scripts/pmc.sh)      -> gpurun_out/$TAG_pmc_WL_summary.json
#   stamps            phase stamps of the clip-group loop           -> gpurun_out/$TAG_stamps.txt
#   probe             L2 -> CU intake probe (scripts/build/l2probe) -> gpurun_out/$TAG_l2_intake.txt
#   py:SCRIPT[:ARGS]  python3 scripts/SCRIPT ARGS                   -> gpurun_out/$TAG_SCRIPT.txt
#   suite             the whole GPU suite without -x (every failure listed) -> gpurun_out/$TAG_pytest.txt
#   train[:MODE]      training step, B = 64, MODE full|frozen        -> gpurun_out/$TAG_train_bench.txt (appended)
#   trprof            rocprofv3 kernel stats of 5 training steps     -> gpurun_out/$TAG_train_kernel_stats.csv
#   enctrace:B        encoder kernel trace at B clips               -> gpurun_out/$TAG_encoder_bB_trace.txt
#   envab:WL:VAR      quick WL passes with VAR=0,1,0,1 on one box   -> gpurun_out/$TAG_WL_VAR_ab.txt
# Extra bench.py arguments: BENCH_ARGS.  A round's evidence is two calls, e.g.
#   TAG=r04t bash scripts/gpu.sh suite smoke prof:c2 prof:c4 prof:c5 bench:c2
#   TAG=r04t bash scripts/gpu.sh pmc:c2 pmc:c4 pmc:c5 bench:c4 bench:c5
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04}

fail() { echo "FAILED: $1"; [ -n "$2" ] && tail -25 "$2"; exit 1; }

for step in "$@"; do
  name=${step%%:*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*:}
  echo "== $step ($(date +%T))"
  case $name in
    tests)
      out=gpurun_out/${T}_pytest.txt
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
        ${arg:+-k "$arg"} > $out 2>&1 || fail tests $out
      tail -1 $out ;;
    smoke)
      out=gpurun_out/${T}_smoke.log
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out 2>&1 || fail smoke $out
      tail -2 $out ;;
    bench|quick)
      wl=${arg:-c2}
      out=gpurun_out/${T}_${wl}_bench.json
      extra=""
      [ "$name" = quick ] && extra="--steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord --no-subrecords"
      timeout -k 10 600 python -u bench.py --workload $wl $extra ${BENCH_ARGS} > $out 2> gpurun_out/${T}_${wl}_bench.err \
        || fail bench gpurun_out/${T}_${wl}_bench.err
      python3 -c "import json,sys; d=json.loads(open('$out').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$wl', d['value'], d['unit'], 'ms/pass', d['ms_per_step'], 'kernel_us', r.get('avg_launch_us'), 'frac', r.get('frac'))" ;;
    prof)
      wl=${arg:-c2}
      d=gpurun_out/${T}_prof_$wl
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
        python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord --no-subrecords ${BENCH_ARGS} \
        > gpurun_out/${T}_prof_$wl.log 2>&1 || fail prof gpurun_out/${T}_prof_$wl.log
      f=$(find $d -name '*kernel_stats.csv' | head -1)
      cp "$f" gpurun_out/${T}_${wl}_kernel_stats.csv
      rm -rf $d
      head -4 gpurun_out/${T}_${wl}_kernel_stats.csv | cut -c1-160 ;;
    pmc)
      wl=${arg:-c2}
      WORKLOADS=$wl bash scripts/pmc_all.sh $T > gpurun_out/${T}_pmc_$wl.log 2>&1 || fail pmc gpurun_out/${T}_pmc_$wl.log
      tail -3 gpurun_out/${T}_pmc_$wl.log ;;
    stamps)
      out=gpurun_out/${T}_stamps.txt
      timeout -k 10 300 python -u scripts/mega_stamps.py > $out 2>&1 || fail stamps $out
      grep -v amdgpu.ids $out | tail -8 ;;
    probe)
      out=gpurun_out/${T}_l2_intake.txt
      timeout -k 10 120 ./scripts/build/l2probe > $out 2>&1 || fail probe $out
      cat $out ;;
    py)
      s=${arg%%:*}
      a=""
      [ "$s" != "$arg" ] && a=${arg#*:}
      out=gpurun_out/${T}_${s%.py}.txt
      timeout -k 10 600 python3 -u scripts/$s $a > $out 2>&1 || fail "$s" $out
      grep -v amdgpu.ids $out | tail -12 ;;
    suite)
      out=gpurun_out/${T}_pytest.txt
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
        > $out 2>&1 || fail suite $out
      tail -1 $out ;;
    train)
      out=gpurun_out/${T}_train_bench.txt
      timeout -k 10 300 python3 -u scripts/train_bench.py 64 10 ${arg:-full} >> $out 2>&1 || fail train $out
      grep "train step" $out | tail -1 ;;
    trprof)
      d=gpurun_out/${T}_trprof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o tr --output-format csv -- \
        python3 -u scripts/train_bench.py 64 5 full > gpurun_out/${T}_trprof.log 2>&1 || fail trprof gpurun_out/${T}_trprof.log
      f=$(find $d -name '*kernel_stats.csv' | head -1)
      cp "$f" gpurun_out/${T}_train_kernel_stats.csv
      rm -rf $d
      head -6 gpurun_out/${T}_train_kernel_stats.csv | cut -c1-160 ;;
    enctrace)
      B=${arg:-32}
      d=gpurun_out/${T}_enc_$B
      timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 scripts/enc_trace.py $B \
        > gpurun_out/${T}_enc_$B.log 2>&1 || fail enctrace gpurun_out/${T}_enc_$B.log
      python3 scripts/enc_trace.py --report $d > gpurun_out/${T}_encoder_b${B}_trace.txt && rm -rf $d
      tail -1 gpurun_out/${T}_encoder_b${B}_trace.txt ;;
    envab)
      wl=${arg%%:*}
      var=${arg#*:}
      out=gpurun_out/${T}_${wl}_${var}_ab.txt
      : > $out
      for v in 0 1 0 1; do
        env "$var=$v" timeout -k 10 300 python3 -u bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline \
          --no-profile --no-f32-subrecord --no-subrecords > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err || fail envab gpurun_out/${T}_ab.err
        python3 -c "import json; d=json.load(open('gpurun_out/${T}_ab.json')); print('$wl $var=$v', d['value'], d['ms_per_step'])" \
          | tee -a $out
      done ;;
    *)
      fail "unknown step $step" ;;
  esac
done
echo "== all steps done ($(date +%T))"
