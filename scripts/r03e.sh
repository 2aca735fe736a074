set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03e}
timeout -k 10 900 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_eps_routes.py tests/test_gpu_parity.py -v -s --timeout 400 --timeout-method thread -k "encoder or mk_ or pair_bf16 or per_clip_loop or ddim50 or speech_driven" > gpurun_out/${T}_pytest.txt 2>&1
echo "pytest rc=$?"
grep -E "mk_bf16 t=|bf16 encoder|PASSED|FAILED|speech moves" gpurun_out/${T}_pytest.txt | tail -40
for w in c2 c5; do
timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/${T}_${w}_bench.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
timeout -k 10 300 python -u scripts/mega_stamps.py > gpurun_out/${T}_stamps.txt 2>&1
echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/${T}_stamps.txt | tail -9
