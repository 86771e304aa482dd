#!/usr/bin/env bash
# Phase stamps of the three heatmap convs (split and mixed) on the GPU box.
set -u
cd "$GRAFT_REPO_ROOT"
for prec in split mixed; do
  for k in stamps_hm1 stamps_hm2 stamps_hm3; do
    KPD_STAMPS=1 timeout -k 10 120 python3 tools/stamps_hm2.py $k $prec || exit 1
  done
done
