set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03af}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -3 gpurun_out/${T}_smoke.txt
start=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
cat gpurun_out/${T}_bench.json
