#!/usr/bin/env bash
# headline bench at 1 / 2 / 3 sub-batch streams, alternated twice (same box)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
for rep in 1 2; do
  for s in 1 2 3; do
    timeout -k 10 120 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --secondary= --streams $s ${BENCH_ARGS:-} > $O/s.log 2>&1 || { tail $O/s.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/s.log').read().strip().splitlines()[-1]); print('streams', $s, d['value'], d['ms_per_step'], d['config']['precision'])"
  done
done
