mkdir -p gpurun_out && export TMPDIR=/tmp
for v in fp8 bf16; do
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/var_$v -o run --output-format csv -- python3 scripts/chain_probe.py $v > gpurun_out/var_$v.log 2>&1 || exit 1
done
