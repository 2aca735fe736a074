set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03w}
timeout -k 10 300 python -u scripts/mega_stamps.py > gpurun_out/${T}_stamps.txt 2>&1
echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/${T}_stamps.txt | tail -7
