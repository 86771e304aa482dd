#!/usr/bin/env bash
# A/B sweep of env-var knobs: one bench.py run per "NAME=VAL ..." argument
# (quoted), printing images/s and the single-stream stage times.
#   bash tools/env_sweep.sh "" "KPD_LAT_BLOCKS=1024" "KPD_LAT_NT=1"
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$ROOTD/gpurun_out"
for cfg in "$@"; do
  out="$ROOTD/gpurun_out/sweep_$(echo "${cfg:-base}" | tr ' =' '_-').json"
  env $cfg timeout -k 10 ${SWEEP_TIMEOUT:-240} python3 "$ROOTD/bench.py" --steps ${SWEEP_STEPS:-20} --no-cpu-baseline \
    ${BENCH_ARGS:-} > "$out" 2> "$out.err" || { echo "FAILED: $cfg"; tail -5 "$out.err"; exit 1; }
  python3 - "$cfg" "$out" <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = b.get("stages_ms", {})
print(f"{sys.argv[1] or 'base':40s} {b['value']:9.1f} img/s  " + " ".join(f"{k}={v:.3f}" for k, v in st.items()))
PY
done
