#!/usr/bin/env bash
# Bench-only A/B of environment variants (no parity: for ablations that are
# wrong by design), alternated twice: value + heatmap / FPN stage times.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 120 python3 bench.py --steps 40 --warmup 30 --no-cpu-baseline --secondary= --alt-streams 0 \
      --c3 0 ${BENCH_ARGS:-} > $O/n.log 2>&1 || { tail $O/n.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/n.log').read().strip().splitlines()[-1]); print('[$v]', d['value'], {k: round(v, 4) for k, v in d['stages_ms'].items() if k.startswith('hm_conv') or k in ('fpn0', 'body')})"
  done
done
