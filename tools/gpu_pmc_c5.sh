#!/usr/bin/env bash
# C5 (384x288, 5 boxes, dual head, 256 images) under rocprofv3: one PMC pass
# per counter group (FETCH_SIZE | WRITE_SIZE | MFMA busy + GUI active, each
# with the kernel trace only), summarised per stage by tools/prof_stages.py
# -> gpurun_out/pmc_c5/pmc_c5.json
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_c5
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for G in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/pass$i -o run -- \
    python3 $R/tools/bench_configs.py --configs C5 --steps 3 --warmup 2 --cpu-sample 0 --streams 1 > $O/pass$i.log 2>&1 \
    || { echo "pmc pass $i rc=$?"; tail -5 $O/pass$i.log; exit 1; }
done
cd $R
python3 tools/prof_stages.py $O --skip 3 --out $O/pmc_c5.json
