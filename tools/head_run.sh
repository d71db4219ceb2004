set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && bash tools/gpu_pytest.sh 900 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/prof && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 10 > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err && \
cat $R/gpurun_out/bench.json
