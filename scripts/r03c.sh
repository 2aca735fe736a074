set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_eps_routes.py tests/test_gpu_parity.py -v -s --timeout 400 --timeout-method thread -k "mk_ or sample_injected or per_clip_loop or graph_step or full_loop or counter_noise or inpaint_generate or speech_driven" > gpurun_out/r03c_pytest.txt 2>&1
echo "pytest rc=$?"
grep -E "rel-RMS|PASSED|FAILED|speech" gpurun_out/r03c_pytest.txt | tail -40
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err
echo "bench rc=$?"
python -c "import json; d=json.load(open('gpurun_out/r03c_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
timeout -k 10 300 python -u scripts/mega_stamps.py > gpurun_out/r03c_stamps.txt 2>&1
echo "stamps rc=$?"
cat gpurun_out/r03c_stamps.txt | grep -v amdgpu.ids
