set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03j}
for B in 128 32; do
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_enc$B -o run --output-format csv -- python3 scripts/enc_trace.py $B > gpurun_out/${T}_enc$B.log 2>&1 || { echo "trace $B failed"; tail -5 gpurun_out/${T}_enc$B.log; exit 1; }
python3 scripts/enc_trace.py --report gpurun_out/${T}_enc$B > gpurun_out/${T}_enc${B}_trace.txt
rm -rf gpurun_out/${T}_enc$B
tail -3 gpurun_out/${T}_enc${B}_trace.txt
done
