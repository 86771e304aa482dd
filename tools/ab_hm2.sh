#!/usr/bin/env bash
# heatmap conv 2 (split) ablations with phase stamps: full, no MFMA, no K-loop DMA
set -u
cd "$GRAFT_REPO_ROOT"
for v in 0 1 2; do
  echo "== KPD_HMCONV_DBG=$v"
  KPD_HMCONV_DBG=$v KPD_STAMPS=1 timeout -k 10 120 python3 tools/stamps_hm2.py stamps_hm2 split || exit 1
done
