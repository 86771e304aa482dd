#!/usr/bin/env bash
# Same-box per-kernel A/B: GPU parity of the current build, then a kernel
# trace of the baseline library (KPD_LIB=libkpd_base.so) and of the current
# one; prints the per-forward time of the kernels matching $PAT for both.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread \
  -p no:cacheprovider > $O/pt.log 2>&1 || { echo "parity failed"; tail -20 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for v in "KPD_LIB=$GRAFT_REPO_ROOT/keypoint-detection_amd/dll/_lib/libkpd_base.so" "KPD_AB_CUR=1"; do
  echo "== $v"
  env $v bash tools/ktrace.sh > $O/kt.txt 2>&1 || { tail $O/kt.txt; exit 1; }
  grep -E "${PAT:-forward}" $O/kt.txt || true
done
