#!/usr/bin/env bash
# A/B of heatmap-conv variants by environment switch: parity on the bench
# batch per variant, then single-stream bench stage times, alternated twice.
# usage: bash tools/ab_conv1.sh "" "KPD_HM1_BN128=1" ...
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
for v in "$@"; do
  env $v timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread \
    -k "bench_batch_properties or odd_size or batch_independence" -p no:cacheprovider > $O/pt.log 2>&1 \
    || { echo "parity failed: $v"; tail -20 $O/pt.log; exit 1; }
done
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 120 python3 bench.py --steps 40 --warmup 30 --no-cpu-baseline --secondary= --alt-streams 0 \
      > $O/c.log 2>&1 || { tail $O/c.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c.log').read().strip().splitlines()[-1]); s=d['stages_ms']; print('[$v]', d['value'], d['ms_per_step'], 'c1', s['hm_conv1'], 'c2', s['hm_conv2'], 'c3', s['hm_conv3'])"
  done
done
