cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python scripts/placement_check.py 32 1000 > gpurun_out/place32.log 2>&1; rc=$?; cat gpurun_out/place32.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/placement_check.py 4 300 > gpurun_out/place4.log 2>&1; rc=$?; tail -8 gpurun_out/place4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/placement_check.py 12 300 > gpurun_out/place12.log 2>&1; rc=$?; tail -8 gpurun_out/place12.log; exit $rc
