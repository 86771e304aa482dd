#!/usr/bin/env bash
# HBM-traffic / counter A/B of diagnostic switches on the C2 command (diag
# build): one rocprofv3 --pmc pass per (variant, counter group), each variant's
# environment exported before rocprofv3 starts.  PMC_AB_ENVS=";"-separated
# variants ("-" = none), PMC_GROUPS=";"-separated counter groups.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_ab; rm -rf $O; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
C2="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --configs none --secondary= --alt-streams 0"
IFS=";" read -ra VARS <<< "${PMC_AB_ENVS:--}"
IFS=";" read -ra PG <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE}"
v=0
for V in "${VARS[@]}"; do
  v=$((v+1)); i=0
  for G in "${PG[@]}"; do
    i=$((i+1))
    ( export KPD_DIAG_LIB=1; [ "$V" != "-" ] && export $V
      timeout -k 10 -s KILL 200 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/v$v/pmc/p$i -o run -- $C2 > $O/v${v}_p$i.log 2>&1 ) \
      || { echo "variant $v pass $i rc=$?"; tail -5 $O/v${v}_p$i.log; exit 1; }
  done
  (cd $R && python3 tools/prof_stages.py $O/v$v --skip 6 --take 20 --out $O/v$v.json > /dev/null)
  echo "== $V"; python3 - $O/v$v.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, e in d.items():
    if ":" in k:
        print(" ", k, {c: round(x, 4) if isinstance(x, float) else x for c, x in e.items()
                       if c in ("avg_us", "hbm_bytes_per_launch", "FETCH_SIZE", "WRITE_SIZE", "mfma_busy_frac")})
PY
done
