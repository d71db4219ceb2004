# round 6: the IQN target's max inside the fused IQN launch (ABI 24): bit-identity tests, the IQN suites, and the
# IQN-loop A/B (--iqn-target-in-fused 0 / 1) at the driver's shape, with one IQN step window per form.
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06j
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_iqn_fused_gpu.py \
  tests/test_learner_golden_gpu.py tests/test_chain_schedule_gpu.py -k "iqn or IQN" > gpurun_out/${T}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.log; exit 2; }
tail -2 gpurun_out/${T}_tests.log
OUT=gpurun_out/${T}_iqn_tq_ab.txt
BASE="--no-cpu-baseline --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 --steps 5 --warmup 2"
for rep in 1 2 3; do for V in 0 1; do
  printf "iqn-target-in-fused %s | rep %s: " $V $rep >> $OUT
  timeout -k 10 200 python bench.py $BASE --iqn-steps 200 --iqn-target-in-fused $V 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['iqn']['ms_per_step'],4), round(d['iqn']['learn_steps_per_s']), d['iqn']['target_in_fused'])" >> $OUT || exit 3
done; done
cat $OUT
R=$PWD
for V in 0 1; do
  (cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof$V && \
   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof$V -o run --output-format csv rocpd \
     -- python3 $R/bench.py $BASE --iqn-steps 100 --iqn-target-in-fused $V > $R/gpurun_out/${T}_prof$V.json 2> $R/gpurun_out/${T}_prof$V.err) || exit 4
  python tools/step_window.py gpurun_out/${T}_prof$V/run_results.db --anchor "critic_fused_kernel<32, true" > gpurun_out/${T}_iqn_step_window$V.txt 2>&1
  head -22 gpurun_out/${T}_iqn_step_window$V.txt
done
echo done
