#!/bin/bash
# One GPU call of the build loop, every step under its own limit, stopping at the first failure:
#   bash tools/gpu_round.sh TAG [tests|suite|none] [bench|nobench] [prof|noprof] [pmc|nopmc]
# tests: the learner / chain tests ($TESTS overrides); suite: the whole -m gpu suite; then the default bench
# line, a rocprofv3 --kernel-trace --stats run of the bench with one graph-replayed step's window
# (tools/step_window.py), and optionally the PMC passes of tools/pmc_run.sh (tools/pmc_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r04}
WHAT=${2:-tests}
TESTS=${TESTS:-"tests/test_chain_schedule_gpu.py tests/test_critic_fused_gpu.py tests/test_learner_golden_gpu.py"}
if [ "$WHAT" = suite ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.log; exit 2; }
  tail -3 gpurun_out/${T}_pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 2
elif [ "$WHAT" = tests ]; then
  timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread $TESTS \
    > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 2; }
  tail -3 gpurun_out/${T}_pytest.log
fi
if [ "${3:-bench}" = bench ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
    || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"
fi
if [ "${4:-prof}" = prof ]; then
  R=$PWD
  (cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof && \
   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
     -- python3 $R/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 \
     --no-cpu-baseline --no-learn-b64 --fp32-steps 0 > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 4
  python tools/step_window.py gpurun_out/${T}_prof/run_results.db > gpurun_out/${T}_step_window.txt 2>&1
  head -20 gpurun_out/${T}_step_window.txt
fi
if [ "${5:-nopmc}" = pmc ]; then
  rm -rf gpurun_out/pmc
  BENCH_ARGS="--steps 10 --warmup 5 --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0" \
    PMC_EXTRA=1 timeout -k 10 1200 bash tools/pmc_run.sh || exit 5
  python tools/pmc_summary.py gpurun_out/pmc --json gpurun_out/${T}_pmc_summary.json > gpurun_out/${T}_pmc_summary.txt 2>&1
fi
exit 0
