#!/bin/bash
# One GPU iteration: the -m gpu suite, then the persistent-loop placement / timing check.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/iter_pytest.log 2>&1
  rc=$?
  tail -15 gpurun_out/iter_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python scripts/placement_check.py 32 1000 > gpurun_out/iter_place.log 2>&1
rc=$?
tail -8 gpurun_out/iter_place.log
exit $rc
