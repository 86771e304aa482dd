#!/usr/bin/env bash
# Kernel trace of a short single-stream bench run, summarised per kernel
# (tools/prof_stages.py): gpurun_out/ktrace.json.  BENCH_ARGS adds bench flags.
set -u
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/ktrace
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ktrace -o run -- \
  python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --secondary= --alt-streams 0 ${BENCH_ARGS:-} \
  > $R/gpurun_out/ktrace.log 2>&1) || { echo "rocprof rc=$?"; tail $R/gpurun_out/ktrace.log; exit 1; }
python3 $R/tools/prof_stages.py $R/gpurun_out/ktrace --skip 12 --out $R/gpurun_out/ktrace.json > /dev/null
python3 - <<'PY'
import json, os
d = json.load(open(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/ktrace.json"))
print("forward_kernel_us", d["_meta"]["forward_kernel_us"])
for k, v in list(d["kernels_us"].items())[:30]:
    print(f'{v["per_forward_us"]:8.1f} {v["avg_us"]:8.2f} {v["calls"]:4d} {k[:100]}')
PY
