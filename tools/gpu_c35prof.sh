#!/usr/bin/env bash
# C3 / C5: the configs lines (stages, roofline, CPU baseline), then a
# rocprofv3 kernel trace of each config alone (kernel stats per forward).
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTD"
OUT="$ROOTD/gpurun_out/c35"
mkdir -p "$OUT"
if [ "${SKIP_CFG:-0}" != 1 ]; then
timeout -k 10 420 python3 -u tools/bench_configs.py --configs C3,C5 ${CFG_ARGS:-} > "$OUT/configs.jsonl" 2> "$OUT/configs.err" \
  || { echo "configs rc=$?"; tail -20 "$OUT/configs.err"; exit 1; }
cat "$OUT/configs.jsonl"
fi
cd /tmp && export TMPDIR=/tmp
for C in ${PROF_CONFIGS:-C3 C5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$C" -o run -- \
    python3 "$ROOTD/tools/bench_configs.py" --configs $C --steps 5 --warmup 10 --cpu-sample 0 > "$OUT/prof_$C.log" 2>&1 \
    || { echo "prof $C rc=$?"; tail -5 "$OUT/prof_$C.log"; exit 1; }
  python3 - "$OUT/prof_$C/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print("%6.2f%% %10.1f us  %5s  %s" % (100 * float(r["TotalDurationNs"]) / tot, float(r["AverageNs"]) / 1e3, r["Calls"], r["Name"][:90]))
PY
done
