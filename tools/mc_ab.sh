# A/B of the weight-gradient chunk floor per group (ASVRL_WGRAD_MIN_CHUNKS 4 shipped, 8, 16): headline AC-IQN line + IQN + Rainbow
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/mc_ab.txt
for rep in 1 2 3; do
  for v in base mc8 mc16; do
    L=$PWD/distributional_rl_decision_and_control_amd/lib/libasvrl.so; [ $v != base ] && L=$PWD/variants/libasvrl_$v.so
    ASVRL_LIB=$L timeout -k 10 200 python bench.py --iqn-steps 20 --rainbow-steps 20 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/mc.json 2> gpurun_out/mc.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/mc.json').read().strip().splitlines()[-1]);print('$v', round(d['ms_per_step'],4), 'iqn', round(d['iqn']['ms_per_step'],4), 'rb', round(d['rainbow']['ms_per_step'],4))" >> gpurun_out/mc_ab.txt
  done
done
