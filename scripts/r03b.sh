set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_eps_routes.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r03b_pytest.txt 2>&1
echo "pytest rc=$?"
grep -E "rel-RMS|PASSED|FAILED|speech" gpurun_out/r03b_pytest.txt | tail -60
