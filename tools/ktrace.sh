#!/usr/bin/env bash
# Kernel trace of a short C2 bench (or C3 with CFG=c3), per-kernel mean
# durations: gpurun_out/$TAG/ktrace_<cfg>.txt.  ENVS: extra environment
# (e.g. "KPD_DIAG_LIB=1 KPD_NO_FIR23=1").
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r06}"; CFG="${CFG:-c2}"; O="$R/gpurun_out/$TAG/kt_$CFG${SUFFIX:-}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
case $CFG in
  c3) ARGS="--only C3 --steps 10 --warmup 5 --no-cpu-baseline --alt-streams 0" ;;
  c5) ARGS="--only C5 --steps 10 --warmup 5 --no-cpu-baseline" ;;
  *) ARGS="--steps 20 --warmup 10 --no-cpu-baseline --no-exact-check --configs none --secondary= --alt-streams 0" ;;
esac
env ${ENVS:-} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o run -- \
  python3 "$R/bench.py" $ARGS > "$O/run.log" 2>&1 || { echo "ktrace rc=$?"; tail -5 "$O/run.log"; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    print(f'{float(r["AverageNs"])/1e3:9.2f} us x{r["Calls"]:>5}  {r["Name"][:110]}')
PY
