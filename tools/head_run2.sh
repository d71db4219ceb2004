#!/bin/bash
# Round-2 head: GPU test suite, default bench, rocprofv3 kernel stats of the bench, PMC traffic passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && bash tools/gpu_pytest.sh 900 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/prof && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 10 > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err && \
cd $R && bash tools/pmc_run.sh && python3 tools/pmc_summary.py gpurun_out/pmc --json gpurun_out/pmc_summary.json > gpurun_out/pmc_summary.txt && \
cat gpurun_out/bench.json
