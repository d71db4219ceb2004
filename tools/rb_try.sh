set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_rainbow_gpu.py -v -s -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/rb_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|agreement|update:|Error" gpurun_out/rb_tests.log | head -40; tail -3 gpurun_out/rb_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 2 --iqn-steps 0 --rainbow-steps 30 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/bench_rb.json 2> gpurun_out/bench_rb.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_rb.json')); print(d['rainbow'])"
