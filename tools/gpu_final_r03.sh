#!/usr/bin/env bash
# Round-3 artifact session: GPU tests + smoke, the driver's exact bench
# command (plain, then under rocprofv3 --stats and the PMC passes:
# tools/gpu_prof_r03.sh), then C1 / C3 / C5 (tools/bench_configs.py).
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTD"
OUT="$ROOTD/gpurun_out/final"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver_cmd.json" 2> "$OUT/bench.err" \
  || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_driver_cmd.json').read().strip().splitlines()[-1]); print('driver cmd', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_ms'])"
timeout -k 10 300 python3 bench.py --steps 100 --warmup 50 > "$OUT/bench_default.json" 2> "$OUT/bench2.err" \
  || { echo "bench2 rc=$?"; tail -20 "$OUT/bench2.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('alt_streams'), d['secondary']['value'], d['cpu_baseline']['value'])"
bash tools/gpu_prof_r03.sh || exit 1
timeout -k 10 420 python3 -u tools/bench_configs.py --configs C1,C3,C5 > "$OUT/configs.jsonl" 2> "$OUT/configs.err" \
  || { echo "configs rc=$?"; tail -20 "$OUT/configs.err"; exit 1; }
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d = json.loads(l); print(d['config'], d.get('images_per_s', d.get('gpu_latency_ms')), (d.get('roofline') or {}).get('frac'))"
# kernel traces of C3 and C5 alone (profiles/r03/kernel_stats_c3.csv, _c5.csv)
SKIP_CFG=1 bash tools/gpu_c35prof.sh > "$OUT/c35prof.txt" 2>&1 || { echo "c35prof failed"; tail -5 "$OUT/c35prof.txt"; exit 1; }
echo "c35 kernel traces ok"
