#!/bin/bash
# PMC passes for the bench workload (run on the GPU box). One counter group per rocprofv3
# run, --kernel-trace only alongside (never sys/runtime traces with --pmc). Output:
# gpurun_out/pmc/<pass>/... ; summarise with tools/pmc_summary.py.
set -e
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 4 --warmup 2 --no-cpu-baseline --iqn-steps 0}"
run() {
  local name="$1"; shift
  timeout -k 10 400 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/$name.log" 2>&1
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES
[ -n "$PMC_EXTRA" ] && run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM
run fetch FETCH_SIZE
run write WRITE_SIZE
echo "pmc passes done"
