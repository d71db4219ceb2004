# Rainbow and config-5 lines: iterations per captured graph 1 / 2 (previous) vs 10, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/rb_c5_unroll_ab.txt
for rep in 1 2 3; do
  for u in 1 2 10; do
    ASVRL_UNROLL=$u timeout -k 10 200 python bench.py --steps 10 --warmup 10 --iqn-steps 0 --rainbow-steps 20 --config5-steps 20 --plateau-envs 0 --no-cpu-baseline > gpurun_out/rc.json 2> gpurun_out/rc.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/rc.json').read().strip().splitlines()[-1]);print('unroll $u rainbow', round(d['rainbow']['ms_per_step'],4), 'config5', round(d['config5']['ms_per_step'],4))" >> gpurun_out/rb_c5_unroll_ab.txt
  done
done
