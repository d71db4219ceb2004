set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for rep in 1 2; do
  for v in default w8; do
    if [ $v = default ]; then L=""; else L="ASVRL_LIB=variants/libasvrl_$v.so"; fi
    echo -n "$v: "; env $L timeout -k 10 120 python tools/bench_iqn_act.py 2>&1 | grep iqn_act
    echo -n "$v iqn step: "; env $L timeout -k 10 120 python tools/bench_iqn.py --iters 200 2>&1 | grep -o '"ms_per_iter": [0-9.]*'
  done
done
