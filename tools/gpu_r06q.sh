# round 6: the PER loop's tail work folded into its kernels (ABI 25): tests, the Rainbow line (3 runs) and its step window
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06q
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_per_gpu.py tests/test_fused_rainbow_gpu.py \
  tests/test_rainbow_golden_gpu.py tests/test_chain_schedule_gpu.py tests/test_dp_graph_gpu.py tests/test_dp_fused_gpu.py > gpurun_out/${T}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.log; exit 2; }
tail -2 gpurun_out/${T}_tests.log
BASE="--no-cpu-baseline --iqn-steps 0 --config5-steps 0 --plateau-envs 0 --fp32-steps 0 --dropin-seconds 0 --steps 5 --warmup 2"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py $BASE --rainbow-steps 50 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); r=d['rainbow']; print('rainbow', round(r['ms_per_step'],4), round(r['learn_steps_per_s']), 'b64', round(d['learn_b64']['rainbow']['ms_per_step']*1e3,2), 'us')" >> gpurun_out/${T}_rainbow.txt || exit 3
done
cat gpurun_out/${T}_rainbow.txt
R=$PWD
(cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
   -- python3 $R/bench.py $BASE --no-learn-b64 --rainbow-steps 60 > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 4
python tools/step_window.py gpurun_out/${T}_prof/run_results.db --anchor rainbow_train_kernel > gpurun_out/${T}_rainbow_window.txt 2>&1
cat gpurun_out/${T}_rainbow_window.txt
