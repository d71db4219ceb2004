# IQN line: iterations per graph 2 (shipped) vs 10, joined vs chained schedule, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/iqn_unroll_ab.txt
for rep in 1 2 3; do
  for cfg in "2 0" "10 0" "10 1"; do
    set -- $cfg
    ASVRL_UNROLL=$1 ASVRL_CHAIN=$2 timeout -k 10 200 python bench.py --steps 10 --warmup 10 --iqn-steps 40 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/iu.json 2> gpurun_out/iu.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/iu.json').read().strip().splitlines()[-1]);print('unroll $1 chain $2 iqn', round(d['iqn']['ms_per_step'],4), round(d['iqn']['learn_steps_per_s'],1))" >> gpurun_out/iqn_unroll_ab.txt
  done
done
