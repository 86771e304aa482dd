#!/usr/bin/env bash
# Round-3 measurement session: the rocprofv3 trace + PMC passes of the
# driver's exact bench command (tools/gpu_prof_r03.sh), then C1 / C3 / C5
# with stages, roofline and CPU baseline (tools/bench_configs.py).
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTD"
OUT="$ROOTD/gpurun_out/r03cfg"
mkdir -p "$OUT"
if [ "${SKIP_PROF:-0}" != 1 ]; then
  bash tools/gpu_prof_r03.sh || exit 1
fi
timeout -k 10 420 python3 -u tools/bench_configs.py --configs "${CONFIGS:-C1,C3,C5}" ${CFG_ARGS:-} \
  > "$OUT/configs.jsonl" 2> "$OUT/configs.err" || { echo "configs rc=$?"; tail -20 "$OUT/configs.err"; exit 1; }
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d = json.loads(l); print(d['config'], d.get('images_per_s', d.get('gpu_latency_ms')), d.get('stages_ms'), (d.get('roofline') or {}).get('frac'))"
