#!/bin/bash
# Run the GPU test suite on the box; stop the call on anything but pass/fail (faults,
# aborts, timeouts end the call, per the pool's rules).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 "${1:-900}" python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -30 gpurun_out/pytest_gpu.log
exit $rc
