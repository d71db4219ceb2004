set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_iqn && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_iqn -o run --output-format csv rocpd -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 2 --iqn-steps 30 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_iqn.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_iqn.err
