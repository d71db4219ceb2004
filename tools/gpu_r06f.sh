set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06f
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; tail -3 gpurun_out/${T}_pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -20
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"
timeout -k 10 200 python -u tools/ab_fused_variant.py > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err; cat gpurun_out/${T}_ab.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM --kernel-trace -d $R/gpurun_out/${T}_pmc/sq24 -o run --output-format csv -- python3 $R/tools/ab_fused_variant.py --variants 4 --forms tq,update --reps 2 > $R/gpurun_out/${T}_pmc_sq24.log 2>&1 || exit 4
echo done
