#!/usr/bin/env bash
# copy the round-3 artifact session's results (gpurun_out/final, prof_r03)
# into profiles/r03 (run here after tools/gpu_final_r03.sh)
set -eu
cd "$(dirname "$0")/.."
F=gpurun_out/final; P=gpurun_out/prof_r03; D=profiles/r03
cp $F/pytest_gpu.log $D/pytest_gpu.log
cp $F/smoke.log $D/smoke.log
tail -1 $F/bench_driver_cmd.json > $D/bench_driver_cmd.json
tail -1 $F/bench_default.json > $D/bench_default.json
cp $F/configs.jsonl $D/configs_c1_c3_c5.jsonl
for C in c3 c5; do
  U=$(echo $C | tr a-z A-Z)
  if [ -f gpurun_out/c35/prof_$U/run_kernel_stats.csv ]; then cp gpurun_out/c35/prof_$U/run_kernel_stats.csv $D/kernel_stats_$C.csv; fi
done
cp $P/trace/run_kernel_stats.csv $D/kernel_stats_driver_cmd.csv
cp $P/stages.json $D/stages_driver_cmd.json
grep -o '{"metric.*' $P/trace.log > $D/bench_driver_cmd_under_rocprof.json
python3 - <<'PY'
import json
d = json.load(open('profiles/r03/stages_driver_cmd.json'))
json.dump({k: v for k, v in d.items() if ':' in k}, open('profiles/r03/pmc.json', 'w'), indent=1)
PY
echo collected
