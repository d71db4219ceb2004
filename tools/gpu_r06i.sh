# round 6: the target pass with two tiles per wave (variants/libasvrl_tqpair.so, -DASVRL_TQ_PAIR=1): bit-identity
# gates against the forward launch, then the launch A/B and the bench A/B against the shipped library.
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06i
ASVRL_LIB=variants/libasvrl_tqpair.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_critic_fused_gpu.py tests/test_fused_critic_gpu.py -k "target_critic_in_launch or in_launch_target" \
  > gpurun_out/${T}_tqpair_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tqpair_tests.log; exit 2; }
tail -2 gpurun_out/${T}_tqpair_tests.log
OUT=gpurun_out/${T}_tqpair_launch_ab.txt
for rep in 1 2 3; do for L in default tqpair; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  printf "%s rep %s: " $L $rep >> $OUT
  timeout -k 10 120 python tools/ab_fused_variant.py --variants 4 --forms tq,update --reps 3 >> $OUT || exit 3
done; done
unset ASVRL_LIB
cat $OUT
REPS=2 timeout -k 10 700 bash tools/ab_libs.sh ${T}_tqpair default tqpair || exit 4
cat gpurun_out/${T}_tqpair_ab.txt
echo done
