set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/build/l2probe > gpurun_out/r03bd_l2_intake.txt 2>&1
rc=$?; cat gpurun_out/r03bd_l2_intake.txt; exit $rc
