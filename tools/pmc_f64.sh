#!/bin/bash
# FP64 VALU instruction counts of the env kernel (bench workload): lists the counters the box
# offers, then one --pmc pass with the F64 VALU counters. Output under gpurun_out/pmc_f64/.
set -e
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/pmc_f64"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
grep -o "SQ_INSTS_VALU_[A-Z0-9_]*F64[A-Z0-9_]*\|SQ_INSTS_VALU_[A-Z]*" "$OUT/counters.txt" | sort -u > "$OUT/valu_counters.txt" || true
C="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d "$OUT/f64" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 4 --warmup 2 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 > "$OUT/f64.log" 2>&1
echo done
