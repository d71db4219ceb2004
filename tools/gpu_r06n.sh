# round 6: the drop-in trainer's batched AC-IQN acts: parity test, the CLI tests, the drop-in line and its profile
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06n
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_agent_gpu.py \
  tests/test_train_script_gpu.py > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 2; }
tail -2 gpurun_out/${T}_tests.log
BASE="--no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0 --steps 5 --warmup 2"
for rep in 1 2; do
  timeout -k 10 200 python bench.py $BASE --dropin-seconds 6 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1])['dropin_single_env']; print('dropin', round(d['env_steps_per_s'],1), round(d['ms_per_env_step'],3), 'ms')" >> gpurun_out/${T}_dropin.txt || exit 3
done
cat gpurun_out/${T}_dropin.txt
timeout -k 10 300 python -u tools/profile_dropin.py --steps 400 > gpurun_out/${T}_dropin_profile.txt 2>&1 || exit 4
head -40 gpurun_out/${T}_dropin_profile.txt
