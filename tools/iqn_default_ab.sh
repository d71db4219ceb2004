# default bench command: the unroll rule vs ASVRL_UNROLL=2, interleaved (IQN / Rainbow / config 5 lines)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/iqn_default_ab.txt
for rep in 1 2; do
  for u in "" 2; do
    ASVRL_UNROLL=$u timeout -k 10 300 python bench.py --plateau-envs 0 --no-cpu-baseline > gpurun_out/idf.json 2> gpurun_out/idf.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/idf.json').read().strip().splitlines()[-1]);print('unroll [$u]', 'main', round(d['ms_per_step'],4), 'iqn', round(d['iqn']['ms_per_step'],4), 'rb', round(d['rainbow']['ms_per_step'],4), 'c5', round(d['config5']['ms_per_step'],4))" >> gpurun_out/iqn_default_ab.txt
  done
done
