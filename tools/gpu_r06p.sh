# round 6: a Rainbow (config 4) step window at the head, full kernel names
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06p
R=$PWD
BASE="--no-cpu-baseline --iqn-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 --steps 5 --warmup 2"
(cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
   -- python3 $R/bench.py $BASE --rainbow-steps 60 > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 4
python tools/step_window.py gpurun_out/${T}_prof/run_results.db --anchor rainbow_train_kernel > gpurun_out/${T}_rainbow_window.txt 2>&1
python - <<'PY'
import sqlite3, re
c = sqlite3.connect("gpurun_out/r06p_prof/run_results.db")
rows = list(c.execute("select name, start, end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if "rainbow_train_kernel" in r[0]]
k = int(len(idx) * 0.6)
for r in rows[idx[k]:idx[k + 1]]:
    if "asvrl" not in r[0]:
        print(round((r[2] - r[1]) / 1e3, 1), r[0][:400])
PY
cat gpurun_out/${T}_rainbow_window.txt
