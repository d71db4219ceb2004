#!/bin/bash
# PMC passes of the target critic's forward launch alone (tools/fused_time.py --mode target: critic_kernel<FWD>
# at B = 4096, N = 32, encoders in-kernel); summarise with tools/pmc_summary.py gpurun_out/pmc_fwd --match critic_kernel
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/pmc_fwd; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
W="python3 $ROOT/tools/fused_time.py --mode ${MODE:-target} --iters 5 --reps 2"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES --kernel-trace -d $OUT/sq -o run --output-format csv -- $W > $OUT/sq.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq2 -o run --output-format csv -- $W > $OUT/sq2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $W > $OUT/fetch.log 2>&1
