#!/usr/bin/env bash
# A/B of sub-batch scheduling (KPD_PIPE / KPD_PIPE_PRI) at S streams: a
# bit-identity check per variant, then the bench, variants alternated twice.
# usage: bash tools/ab_pipe.sh "S=2" "S=2 KPD_PIPE=3 KPD_PIPE_PRI=1" ...
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
for v in "$@"; do
  S=$(echo "$v" | sed -n 's/.*S=\([0-9]\).*/\1/p'); E=$(echo "$v" | sed 's/S=[0-9]//')
  env $E timeout -k 10 120 python3 tools/pipe_check.py $S || { echo "check failed: $v"; exit 1; }
done
for rep in 1 2; do
  for v in "$@"; do
    S=$(echo "$v" | sed -n 's/.*S=\([0-9]\).*/\1/p'); E=$(echo "$v" | sed 's/S=[0-9]//')
    env $E timeout -k 10 120 python3 bench.py --steps 40 --warmup 30 --no-cpu-baseline --secondary= --alt-streams 0 \
      --streams $S > $O/p.log 2>&1 || { tail $O/p.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/p.log').read().strip().splitlines()[-1]); print('$v', '|', d['value'], d['ms_per_step'])"
  done
done
