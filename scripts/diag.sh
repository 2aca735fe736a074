#!/bin/bash
# GPU session: parity tests, then optional per-kernel diagnostics / profile.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ "$1" = "diag" ]; then
  timeout -k 10 300 python scripts/diag_kernels.py bf16 > gpurun_out/diag.log 2>&1; rc=$?
  echo "diag rc=$rc"; grep -v amdgpu.ids gpurun_out/diag.log | tail -30
  exit $rc
fi
if [ -n "$1" ]; then bash scripts/profile.sh "$@"; fi
