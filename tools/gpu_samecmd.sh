#!/usr/bin/env bash
# The headline bench command under rocprofv3 --kernel-trace --stats: the bench
# line's roofline avg_ms and the profiler's average for the same kernel come
# from the same run.
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUTD="$ROOTD/gpurun_out/samecmd"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD" -o run -- \
  python3 "$ROOTD/bench.py" --no-cpu-baseline --secondary= --alt-streams 0 ${BENCH_ARGS:-} > "$OUTD/bench.log" 2>&1 || { echo "rc=$?"; tail "$OUTD/bench.log"; exit 1; }
tail -1 "$OUTD/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench', d['value'], r['stage'], r['avg_ms'], r['launches_timed'])"
head -4 "$OUTD"/run_kernel_stats.csv | cut -c1-160
