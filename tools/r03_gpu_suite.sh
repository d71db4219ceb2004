#!/bin/bash
# round 3: the full GPU suite, the stream probe, then the default bench; every step under its own limit
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/graph_stream_probe.py > gpurun_out/${T}_probe.log 2>&1
echo "probe rc=$?" >> gpurun_out/${T}_probe.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
