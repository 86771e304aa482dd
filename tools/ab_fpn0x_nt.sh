#!/usr/bin/env bash
# fpn0x streaming A-row loads (KPD_FPN0X_ANT): parity, bench stage time and a
# FETCH_SIZE PMC pass per setting (same box)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
KPD_FPN0X_ANT=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 \
  --timeout-method thread -k "bench_batch_properties or odd_size or forward_main" -p no:cacheprovider > $O/pt.log 2>&1 \
  || { echo "parity failed"; tail -20 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for v in 0 1 0 1; do
  KPD_FPN0X_ANT=$v timeout -k 10 120 python3 bench.py --steps 40 --warmup 30 --no-cpu-baseline --secondary= --alt-streams 0 \
    > $O/c.log 2>&1 || { tail $O/c.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c.log').read().strip().splitlines()[-1]); s=d['stages_ms']; print('ANT=$v', d['value'], 'fpn0', s['fpn0'])"
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  KPD_FPN0X_ANT=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_ant$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 10 --no-cpu-baseline --secondary= --alt-streams 0 > $GRAFT_REPO_ROOT/$O/pmc$v.log 2>&1 \
    || { echo "pmc rc=$?"; exit 1; }
  python3 - $GRAFT_REPO_ROOT/$O/pmc_ant$v/run_counter_collection.csv $v <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'fpn0x' in r['Kernel_Name'] and r['Counter_Name'] == 'FETCH_SIZE']
by = {}
for r in rows:
    by.setdefault(r['Dispatch_Id'], 0.0)
    by[r['Dispatch_Id']] += float(r['Counter_Value'])
v = sorted(by.values())
print('ANT=%s fpn0x FETCH_SIZE per launch (KB, median of %d): %.0f -> HBM read bytes 2x = %.1f MB' % (sys.argv[2], len(v), v[len(v)//2], 2 * v[len(v)//2] * 1024 / 1e6))
PY
done
