# the chained graph schedule: equivalence test, then an interleaved A/B against the joined schedule (ASVRL_CHAIN)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
[ -n "$SKIP_TEST" ] || timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_chain_schedule_gpu.py > gpurun_out/chain_tests.log 2>&1 || exit 1
: > gpurun_out/chain_ab.txt
for rep in 1 2 3 4 5; do
  for c in 1 0; do
    ASVRL_CHAIN=$c timeout -k 10 200 python bench.py --iqn-steps 30 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/ch.json 2> gpurun_out/ch.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ch.json').read().strip().splitlines()[-1]);print('chain=$c', round(d['ms_per_step'],4), round(d['value']/1e6,3), 'iqn', round(d['iqn']['ms_per_step'],4), round(d['iqn']['learn_steps_per_s'],1))" >> gpurun_out/chain_ab.txt
  done
done
