# round 6: the Rainbow clip norm from the reduction + the noisy backward (ABI 26): Rainbow tests and the line
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06t
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_per_gpu.py tests/test_fused_rainbow_gpu.py \
  tests/test_rainbow_golden_gpu.py tests/test_dp_fused_gpu.py tests/test_dp_graph_gpu.py tests/test_agent_gpu.py > gpurun_out/${T}_tests.log 2>&1 \
  || { tail -40 gpurun_out/${T}_tests.log; exit 2; }
tail -2 gpurun_out/${T}_tests.log
BASE="--no-cpu-baseline --iqn-steps 0 --config5-steps 0 --plateau-envs 0 --fp32-steps 0 --dropin-seconds 0 --steps 5 --warmup 2"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py $BASE --rainbow-steps 50 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); r=d['rainbow']; print('rainbow', round(r['ms_per_step'],4), round(r['learn_steps_per_s']), 'b64', round(d['learn_b64']['rainbow']['ms_per_step']*1e3,2), 'us')" >> gpurun_out/${T}_rainbow.txt || exit 3
done
cat gpurun_out/${T}_rainbow.txt
