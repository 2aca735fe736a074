set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03aj}
timeout -k 10 300 python -u scripts/mega_arrivals.py > gpurun_out/${T}_arrivals.txt 2>&1
echo "arrivals rc=$?"
grep -v amdgpu.ids gpurun_out/${T}_arrivals.txt | tail -16
