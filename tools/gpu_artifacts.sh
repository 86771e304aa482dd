#!/usr/bin/env bash
# Round artifacts on the GPU box, every GPU step under its own limit, stop at the
# first failure: GPU tests, smoke, steady-state rocprofv3 stats + PMC passes for
# split and mixed (tools/gpu_prof_r02.sh), merged pmc.json, the default bench
# line (reading that pmc.json), the other configs (C1 / C3 / C5).
set -u
cd "$GRAFT_REPO_ROOT"
A=gpurun_out/art; mkdir -p $A
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $A/pytest_gpu.log 2>&1 || { tail -30 $A/pytest_gpu.log; exit 1; }
tail -1 $A/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $A/smoke.log 2>&1 || { tail -20 $A/smoke.log; exit 1; }
tail -1 $A/smoke.log
for P in split mixed; do
  PREC=$P bash tools/gpu_prof_r02.sh > $A/prof_$P.txt 2>&1 || { tail -20 $A/prof_$P.txt; exit 1; }
  cat $A/prof_$P.txt
done
python3 - <<'PY'
import json
m = {}
for p in ("split", "mixed"):
    d = json.load(open(f"gpurun_out/prof_{p}/stages.json"))
    for k, v in d.items():
        if ":" in k:
            m[k] = v
json.dump(m, open("gpurun_out/art/pmc.json", "w"), indent=1)
PY
timeout -k 10 400 python -u bench.py --pmc-json gpurun_out/art/pmc.json > $A/bench.log 2>&1 || { tail -20 $A/bench.log; exit 1; }
tail -1 $A/bench.log | cut -c1-400
timeout -k 10 400 python -u tools/bench_configs.py --precision split > $A/configs_split.jsonl 2>&1 || { tail -20 $A/configs_split.jsonl; exit 1; }
cat $A/configs_split.jsonl | cut -c1-300
