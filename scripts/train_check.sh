# training path check (r04x): the GPU training tests, then the training-step bench (B = 64, encoder trained)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
T=r04x
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_training.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_training.txt 2>&1 || { tail -15 gpurun_out/${T}_pytest_training.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest_training.txt
timeout -k 10 300 python3 -u scripts/train_bench.py 64 10 full > gpurun_out/${T}_train_bench.txt 2>&1 || { tail -5 gpurun_out/${T}_train_bench.txt; exit 1; }
timeout -k 10 300 python3 -u scripts/train_bench.py 64 10 frozen >> gpurun_out/${T}_train_bench.txt 2>&1 || { tail -5 gpurun_out/${T}_train_bench.txt; exit 1; }
grep "train step" gpurun_out/${T}_train_bench.txt
