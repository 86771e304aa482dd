#!/usr/bin/env bash
# Same-box A/B of environment variants on the C3 object only (bench.py
# --c3-only, no CPU baseline): per variant the C3 value and its stage times,
# alternated twice.  usage: bash tools/ab_c3.sh "KPD_DIAG_LIB=1" "KPD_DIAG_LIB=1 KPD_X=1"
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 180 python3 bench.py --c3-only --steps 10 --warmup 5 --no-cpu-baseline --alt-streams 0 \
      > $O/c3.log 2>&1 || { tail $O/c3.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c3.log').read().strip().splitlines()[-1]); c=d.get('configs',{}).get('C3',d); print('[$v]', c['value'], c['ms_per_step'], {k: round(x, 3) for k, x in c['stages_ms'].items()}, c.get('parity'))"
  done
done
