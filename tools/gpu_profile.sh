#!/usr/bin/env bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC here: counters
# are collected in their own pass, tools/gpu_pmc.sh).
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
OUTD="$ROOTD/gpurun_out/prof_$TAG"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD" -o run -- \
  python3 "$ROOTD/bench.py" --steps ${PROF_STEPS:-10} --warmup 3 --no-cpu-baseline --streams 1 ${BENCH_ARGS:-} > "$OUTD/bench_under_prof.log" 2>&1
rc=$?
tail -n 3 "$OUTD/bench_under_prof.log"
find "$OUTD" -name "*kernel_stats.csv" -exec head -n 40 {} \;
exit $rc
