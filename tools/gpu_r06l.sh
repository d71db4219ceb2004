# round 6: full -m gpu suite + smoke at the head (after ABI 24)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06l}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 3; }
tail -3 gpurun_out/${T}_smoke.log
echo done
