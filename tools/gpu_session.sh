#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, short bench.  Every GPU step has its
# own time limit; a crash/timeout (exit >= 124 or signal) stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }   # 1 = test failures (no crash)

echo "== device"; timeout -k 10 120 python -c "import torch;print(torch.cuda.get_device_name(0))" || exit 2
echo "== pytest -m gpu"
timeout -k 10 ${PYTEST_TIMEOUT:-700} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 30 $OUT/pytest_gpu.log; ok $rc || { echo "pytest rc=$rc, stopping"; exit $rc; }
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -n 5 $OUT/smoke.log; ok $rc || { echo "smoke rc=$rc, stopping"; exit $rc; }
echo "== bench"
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; tail -n 5 $OUT/bench.log; exit $rc
