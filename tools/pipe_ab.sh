# the pipelined learner on the chained schedule: equivalence tests, then an interleaved A/B (ASVRL_PIPELINE)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_chain_schedule_gpu.py > gpurun_out/chain_tests.log 2>&1 || exit 1
: > gpurun_out/pipe_ab.txt
for rep in 1 2 3 4; do
  for pp in 1 0; do
    ASVRL_PIPELINE=$pp timeout -k 10 200 python bench.py --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/pp.json 2> gpurun_out/pp.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/pp.json').read().strip().splitlines()[-1]);print('pipeline=$pp', round(d['ms_per_step'],4), round(d['value']/1e6,3))" >> gpurun_out/pipe_ab.txt
  done
done
