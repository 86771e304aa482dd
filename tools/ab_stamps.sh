#!/usr/bin/env bash
# Per-variant phase stamps (tools/stamps_probe.py) of the kernels matching
# $PAT, one environment variant per argument ("" = defaults).
# usage: PAT="fir|latchain" bash tools/ab_stamps.sh "" "KPD_FIR_TH=2"
set -u
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  echo "== variant: $v"
  env $v KPD_STAMPS=1 timeout -k 10 120 python3 tools/stamps_probe.py > gpurun_out/stamps.log 2>&1 || { tail gpurun_out/stamps.log; exit 1; }
  grep -E "${PAT:-.}" gpurun_out/stamps.log || true
done
