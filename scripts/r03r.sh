set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03r}
timeout -k 10 1500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${T}_pytest.txt 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/${T}_pytest.txt
grep -E "FAILED|ERROR" gpurun_out/${T}_pytest.txt | head
