set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
python -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)), 'OMP', os.environ.get('OMP_NUM_THREADS'))" > gpurun_out/cpuinfo.txt
nproc >> gpurun_out/cpuinfo.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/cpuinfo.txt 2>/dev/null || true
timeout -k 10 300 python tools/bench_env.py --envs 4096,65536,262144 --noise f32 --launch "auto;1,128,12;1,128,24;1,256,24;1,256,48;1,64,12;1,128,6;2,0,0" > gpurun_out/envsweep5.jsonl 2>&1 && \
timeout -k 10 300 python tools/bench_env.py --robots 17 --width 110 --envs 4096,65536 --noise f32 --launch "auto;1,128,7;1,256,15;1,256,7;1,64,3;2,0,0" > gpurun_out/envsweep17.jsonl 2>&1
