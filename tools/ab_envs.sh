#!/usr/bin/env bash
# Same-box A/B of environment variants of the current build: GPU parity
# under each variant, then single-stream bench stage times, alternated twice.
# usage: bash tools/ab_envs.sh "" "KPD_HM_BDIR=1"
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
for v in "$@"; do
  env $v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > $O/pt.log 2>&1 || { echo "parity failed [$v]"; tail -20 $O/pt.log; exit 1; }
  echo "[$v] $(tail -1 $O/pt.log)"
done
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 120 python3 bench.py --steps 40 --warmup 30 --no-cpu-baseline --secondary= --alt-streams 0 \
      ${BENCH_ARGS:-} > $O/c.log 2>&1 || { tail $O/c.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c.log').read().strip().splitlines()[-1]); s=d['stages_ms']; print('[$v]', d['value'], d['ms_per_step'], {k: round(x, 4) for k, x in s.items()})"
  done
done
