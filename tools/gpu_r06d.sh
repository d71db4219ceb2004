set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06d
timeout -k 10 200 python -u tools/debug_fused8.py --B 4096 > gpurun_out/${T}_dbg4096.json 2> gpurun_out/${T}_dbg.err || { tail -20 gpurun_out/${T}_dbg.err; exit 2; }
timeout -k 10 200 python -u tools/debug_fused8.py --B 1536 > gpurun_out/${T}_dbg1536.json 2>> gpurun_out/${T}_dbg.err
timeout -k 10 200 python -u tools/debug_fused8.py --B 2048 > gpurun_out/${T}_dbg2048.json 2>> gpurun_out/${T}_dbg.err
echo done
