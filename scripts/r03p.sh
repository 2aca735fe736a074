set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03p}
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -s tests/test_gpu_encoder.py "tests/test_gpu_parity.py::test_clip_attention_matches_query_split" > gpurun_out/${T}_pytest.txt 2>&1
echo "pytest rc=$?"
grep -E "PASSED|FAILED|rel-RMS|assert" gpurun_out/${T}_pytest.txt | cut -c1-200 | head -30
