#!/usr/bin/env bash
# Round-3 GPU session: GPU tests, then the driver's bench command, then an
# A/B bench line with a switch (AB_ENV, e.g. "KPD_NO_CBODY=1").  Every step
# has its own time limit; the first failure ends the script.
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOTD/gpurun_out/${TAG:-r03}"
mkdir -p "$OUT"
cd "$ROOTD"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'ms', d['ms_per_step'], 'stages', d['stages_ms'])"
if [ -n "${AB_ENV:-}" ]; then
  env $AB_ENV timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --secondary= \
    --alt-streams 0 > "$OUT/bench_ab.json" 2> "$OUT/bench_ab.err" || { echo "ab rc=$?"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_ab.json').read().strip().splitlines()[-1]); print('AB $AB_ENV value', d['value'], 'ms', d['ms_per_step'], 'stages', d['stages_ms'])"
fi
