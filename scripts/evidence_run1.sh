# round-4 evidence call 1 (r04t): GPU suite, smoke, rocprof kernel stats of C2 / C4 / C5, the C2 line
T=r04t
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest.txt 2>&1; tail -2 gpurun_out/${T}_pytest.txt; grep -E "^FAILED" gpurun_out/${T}_pytest.txt | head
TAG=$T bash scripts/gpu.sh smoke prof:c2 prof:c4 prof:c5 bench:c2
