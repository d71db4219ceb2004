#!/bin/bash
# C51 projection A/B: the bit-exact tests, graph-timed variants (tools/bench_c51.py) and one PMC pass of the
# default library: bash tools/c51_ab.sh TAG variant...
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1; shift
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_learn_kernels_gpu.py \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for L in "$@" default; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  timeout -k 10 100 python tools/bench_c51.py 2>&1 | grep B= | tee -a gpurun_out/${T}_c51.txt || exit 1
done
unset ASVRL_LIB
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $R/gpurun_out/${T}_pmc -o run --output-format csv -- python3 $R/tools/bench_c51.py > /dev/null 2>&1 || exit 2
python3 - $R/gpurun_out/${T}_pmc <<'PY' | tee -a $R/gpurun_out/${T}_c51.txt
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "c51" in r["Kernel_Name"]:
        key = (r["Kernel_Name"][:40], r["Grid_Size"])
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v) * (1 if c != "SQ_WAVES" else 1)) for c, v in sorted(d.items())})
PY
