#!/usr/bin/env bash
# env A/B with HBM traffic: per variant a short bench (stage times) and one
# rocprofv3 FETCH_SIZE / WRITE_SIZE pass summarised per stage (prof_stages)
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
O=$R/gpurun_out/abp; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for v in "$@"; do
  i=$((i + 1))
  env $v timeout -k 10 120 python3 bench.py --no-cpu-baseline --secondary= --alt-streams 0 > $O/b$i.log 2>&1 || { tail $O/b$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b$i.log').read().strip().splitlines()[-1]); print('[$v]', d['value'], {k: round(v, 4) for k, v in d['stages_ms'].items()})"
  (cd /tmp && export TMPDIR=/tmp && env $v timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --secondary= --alt-streams 0 > $O/p$i.log 2>&1) || { echo "pmc rc=$?"; exit 1; }
  python3 tools/prof_stages.py $O/p$i --skip 2 | grep -E "fpn0|hm_conv" | cut -c1-200
done
