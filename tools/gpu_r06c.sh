set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06c
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_critic_fused8_gpu.py tests/test_critic_bf16_oracle_gpu.py -s > gpurun_out/${T}_w8.log 2>&1
tail -15 gpurun_out/${T}_w8.log
timeout -k 10 200 python -u tools/ab_fused_variant.py > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err; cat gpurun_out/${T}_ab.json
echo done
