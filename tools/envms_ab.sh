set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/envms_ab.txt
for rep in 1 2; do
  for u in "" 2; do
    ASVRL_UNROLL=$u timeout -k 10 300 python bench.py --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/em.json 2> gpurun_out/em.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/em.json').read().strip().splitlines()[-1]);print('unroll [$u]', round(d['ms_per_step'],4), 'env', round(d['env_kernel_ms'],4), 'roof', round(d['roofline']['ms_per_launch'],4))" >> gpurun_out/envms_ab.txt
  done
done
