set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06e
R=$PWD
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_critic_fused8_gpu.py tests/test_critic_bf16_oracle_gpu.py -s > gpurun_out/${T}_w8.log 2>&1; tail -4 gpurun_out/${T}_w8.log
cd /tmp && export TMPDIR=/tmp
for V in 8 4; do
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES --kernel-trace -d $R/gpurun_out/${T}_pmc/sq$V -o run --output-format csv -- python3 $R/tools/ab_fused_variant.py --variants $V --forms update --reps 2 > $R/gpurun_out/${T}_pmc_sq$V.log 2>&1 || exit 3
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM --kernel-trace -d $R/gpurun_out/${T}_pmc/sq2$V -o run --output-format csv -- python3 $R/tools/ab_fused_variant.py --variants $V --forms update --reps 2 > $R/gpurun_out/${T}_pmc_sq2$V.log 2>&1 || exit 4
done
echo done
