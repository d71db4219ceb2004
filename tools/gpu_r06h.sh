# round 6: cooperative probe v2 (barrier and in-launch reduction timed apart), the ACTOR launch with the actor's
# backward inside (ABI 24) -- its tests and the loop-level bit-identity -- and its A/B in the bench (the separate
# backward launch / in-launch / in-launch with two tiles per wave, variants/libasvrl_tpw2.so).
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06h
timeout -k 10 60 ./tools/coop_capture_probe > gpurun_out/${T}_coop_probe.json 2> gpurun_out/${T}_coop_probe.err || { echo "coop probe failed"; cat gpurun_out/${T}_coop_probe.err; exit 1; }
cat gpurun_out/${T}_coop_probe.json
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_actor_bwd_in_launch_gpu.py \
  tests/test_chain_schedule_gpu.py tests/test_learner_golden_gpu.py tests/test_fused_critic_gpu.py > gpurun_out/${T}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.log; exit 2; }
tail -3 gpurun_out/${T}_tests.log
ASVRL_LIB=variants/libasvrl_tpw2.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_actor_bwd_in_launch_gpu.py > gpurun_out/${T}_tpw2_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tpw2_tests.log; exit 3; }
tail -2 gpurun_out/${T}_tpw2_tests.log
OUT=gpurun_out/${T}_abwd_ab.txt
BASE="--no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0 --dropin-seconds 0"
for shape in "--steps 20 --warmup 5" "--steps 300 --warmup 30"; do
  for rep in 1 2 3; do for V in sep tpw1 tpw2; do
    case $V in sep) A="--actor-bwd-in-launch 0"; unset ASVRL_LIB;; tpw1) A=""; unset ASVRL_LIB;; tpw2) A=""; export ASVRL_LIB=variants/libasvrl_tpw2.so;; esac
    printf "%s | %s | rep %s: " "$shape" "$V" "$rep" >> $OUT
    timeout -k 10 200 python bench.py $shape $BASE $A 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> $OUT || exit 4
  done; done
done
unset ASVRL_LIB
cat $OUT
R=$PWD
(cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
   -- python3 $R/bench.py --steps 50 --warmup 10 $BASE > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 5
python tools/step_window.py gpurun_out/${T}_prof/run_results.db > gpurun_out/${T}_step_window.txt 2>&1
head -16 gpurun_out/${T}_step_window.txt
echo done
