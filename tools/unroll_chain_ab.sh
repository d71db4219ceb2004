# iterations per captured graph with the chained schedule: 2 (shipped) vs 10, interleaved, AC-IQN headline line
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/unroll_chain_ab.txt
for rep in 1 2 3 4; do
  for u in 2 10; do
    ASVRL_UNROLL=$u timeout -k 10 200 python bench.py --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/uc.json 2> gpurun_out/uc.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/uc.json').read().strip().splitlines()[-1]);print('unroll $u', round(d['ms_per_step'],4), round(d['value']/1e6,3))" >> gpurun_out/unroll_chain_ab.txt
  done
done
