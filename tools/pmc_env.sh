#!/bin/bash
# PMC passes of the env-step kernel alone at 2^18 envs (tools/bench_env.py, f32 noise, automatic
# launch shape; ENV_ARGS overrides). Output gpurun_out/$PMC_NAME (default pmc_env)/<pass>/; summarise with
# tools/pmc_summary.py --match env_.
set -e
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${PMC_NAME:-pmc_env}"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
ARGS="${ENV_ARGS:---envs 262144 --noise f32 --iters 3}"
run() {
  local name="$1"; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- \
    python3 "$ROOT/tools/bench_env.py" $ARGS > "$OUT/$name.log" 2>&1
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE
run f64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 || echo "f64 pass failed"
run fetch FETCH_SIZE
run write WRITE_SIZE
echo "pmc passes done"
