set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_critic_fused_gpu.py tests/test_learner_golden_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?; tail -5 gpurun_out/fused_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err && \
cd /tmp && export TMPDIR=/tmp && rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_fused && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_fused.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_fused.err && \
cd $GRAFT_REPO_ROOT && PMC_EXTRA=1 BENCH_ARGS="--steps 4 --warmup 2 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0" bash tools/pmc_run.sh
