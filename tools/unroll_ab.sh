# A/B of iterations per captured graph (ASVRL_UNROLL) on the headline AC-IQN line, interleaved runs
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/unroll_ab.txt
for rep in 1 2 3; do
  for u in 2 5 10; do
    ASVRL_UNROLL=$u timeout -k 10 200 python bench.py --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/ub.json 2> gpurun_out/ub.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ub.json').read().strip().splitlines()[-1]);print('unroll $u', round(d['ms_per_step'],4), round(d['value']/1e6,3))" >> gpurun_out/unroll_ab.txt
  done
done
