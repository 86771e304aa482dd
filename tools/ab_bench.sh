#!/usr/bin/env bash
# parity tests, then the headline bench per env variant (alternated): value + chosen stages
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 120 python3 bench.py --no-cpu-baseline --secondary= --alt-streams 0 ${BENCH_ARGS:-} > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print('[$v]', d['value'], {k: round(v, 4) for k, v in d['stages_ms'].items() if k.startswith('hm_conv') or k in ('fpn0', 'body', 'roi_align')})"
  done
done
