set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03bc}
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${T}_pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest_gpu.txt
grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.txt | head -5 || true
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
echo smoke ok; tail -3 gpurun_out/${T}_smoke.log
