set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06b
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_critic_fused8_gpu.py tests/test_critic_bf16_oracle_gpu.py -s > gpurun_out/${T}_w8.log 2>&1 || { tail -40 gpurun_out/${T}_w8.log; exit 2; }
tail -3 gpurun_out/${T}_w8.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_critic_fused_gpu.py tests/test_fused_critic_gpu.py tests/test_learner_golden_gpu.py tests/test_chain_schedule_gpu.py tests/test_dp_fused_gpu.py > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 3; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"
echo done
