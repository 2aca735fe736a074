set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03d}
timeout -k 10 900 python -u -m pytest tests/test_gpu_eps_routes.py tests/test_gpu_parity.py -v -s --timeout 400 --timeout-method thread -k "mk_ or sample_injected or per_clip_loop or graph_step or ddpm_T1000 or counter_noise" > gpurun_out/${T}_pytest.txt 2>&1
echo "pytest rc=$?"
grep -E "mk_bf16 t=|PASSED|FAILED" gpurun_out/${T}_pytest.txt | tail -30
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
echo "bench rc=$?"
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
timeout -k 10 300 python -u scripts/mega_stamps.py > gpurun_out/${T}_stamps.txt 2>&1
echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/${T}_stamps.txt | tail -9
