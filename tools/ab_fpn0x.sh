#!/usr/bin/env bash
# fpn0x A/B: parity tests once, then per variant the K-loop stamps and a short single-stream bench
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "$@"; do
  echo "== variant: $v"
  env $v KPD_STAMPS=1 timeout -k 10 120 python3 tools/stamps_fpn0x.py split || exit 1
  env $v timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary= --streams 1 > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k:round(v,4) for k,v in d['stages_ms'].items()})"
done
