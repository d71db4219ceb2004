#!/bin/bash
# round 3, first GPU call: the stream-alias probe, the chain-schedule tests, the default bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u tools/graph_stream_probe.py > gpurun_out/r03_probe.log 2>&1
echo "probe rc=$?" >> gpurun_out/r03_probe.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_chain_schedule_gpu.py > gpurun_out/r03_chain_test.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03_bench_a.json 2> gpurun_out/r03_bench_a.err
