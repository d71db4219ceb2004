set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06a
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_critic_bf16_oracle_gpu.py tests/test_eval_iqn_golden_gpu.py -s > gpurun_out/${T}_new.log 2>&1; tail -5 gpurun_out/${T}_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --deselect tests/test_critic_bf16_oracle_gpu.py --deselect tests/test_eval_iqn_golden_gpu.py > gpurun_out/${T}_pytest_gpu.log 2>&1; tail -3 gpurun_out/${T}_pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 3
timeout -k 10 300 python -u bench.py --dp-rehearsal --steps 20 --warmup 5 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 > gpurun_out/${T}_dp_rehearsal.json 2> gpurun_out/${T}_dp.err
echo done
