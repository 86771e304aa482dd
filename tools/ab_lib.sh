#!/usr/bin/env bash
# Same-box A/B of the current libkpd.so against a baseline build
# (KPD_LIB=keypoint-detection_amd/dll/_lib/libkpd_base.so): parity of the
# current build, then single-stream bench stage times, alternated twice.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
BASE=keypoint-detection_amd/dll/_lib/libkpd_base.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread \
  -p no:cacheprovider > $O/pt.log 2>&1 || { echo "parity failed"; tail -20 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for rep in 1 2; do
  for v in "KPD_LIB=$BASE" "KPD_AB_CUR=1"; do
    env $v timeout -k 10 120 python3 bench.py --steps 40 --warmup 30 --no-cpu-baseline --secondary= --alt-streams 0 \
      ${BENCH_ARGS:-} > $O/c.log 2>&1 || { tail $O/c.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c.log').read().strip().splitlines()[-1]); s=d['stages_ms']; print('[$v]', d['value'], d['ms_per_step'], {k: round(x, 4) for k, x in s.items()})"
  done
done
