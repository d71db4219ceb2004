# round 6: the IQN loop with the act pass held behind the target pass: bit-identity tests and the A/B
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06v
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_chain_schedule_gpu.py \
  tests/test_iqn_fused_gpu.py > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 2; }
tail -2 gpurun_out/${T}_tests.log
BASE="--no-cpu-baseline --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 --steps 5 --warmup 2 --iqn-steps 200"
for rep in 1 2 3; do for V in 0 1; do
  printf "act-after-target %s rep %s: " $V $rep >> gpurun_out/${T}_iqn_aat_ab.txt
  timeout -k 10 200 python bench.py $BASE --iqn-act-after-target $V 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1])['iqn']; print(round(d['ms_per_step'],4), round(d['learn_steps_per_s']), d['act_after_target'])" >> gpurun_out/${T}_iqn_aat_ab.txt || exit 3
done; done
cat gpurun_out/${T}_iqn_aat_ab.txt
R=$PWD
(cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
   -- python3 $R/bench.py $BASE --iqn-steps 100 --iqn-act-after-target 1 > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 4
python tools/step_window.py gpurun_out/${T}_prof/run_results.db --anchor "critic_fused_kernel<32, true" > gpurun_out/${T}_iqn_step_window.txt 2>&1
head -14 gpurun_out/${T}_iqn_step_window.txt
