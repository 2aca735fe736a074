#!/bin/bash
# PMC passes (scripts/pmc.sh) over the bench workloads c2, c4, c5; one summary per workload.
cd "$(dirname "$0")/.." || exit 1
TAG=${1:-r01n}
for w in ${WORKLOADS:-c2 c4 c5}; do
  WORKLOAD=$w BENCH_ARGS="--workload $w --no-f32-subrecord --no-subrecords" bash scripts/pmc.sh ${TAG}_pmc_$w FETCH_SIZE WRITE_SIZE \
    'SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE' \
    'TCC_HIT_sum TCC_MISS_sum' > gpurun_out/${TAG}_pmc_$w.out 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_$w.out; exit 1; }
  rm -rf gpurun_out/${TAG}_pmc_${w}_[0-9]*   # raw per-dispatch CSVs: too large to copy back (C4: 36k dispatches)
  echo "$w done"
done
