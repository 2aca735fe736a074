set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -k "eps_routes or prefetch or c1_tedexp or trained_checkpoint or eval_mode or optimizer_state or sample_injected or long_loop or per_clip_loop or clip_pair_loop or graph_step" > gpurun_out/r03a_pytest.txt 2>&1
echo "pytest rc=$?"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err
echo "bench rc=$?"
tail -3 gpurun_out/r03a_pytest.txt
