#!/usr/bin/env bash
# rocprofv3 kernel trace of a short single-stream bench + the per-kernel
# timeline of one forward (tools/timeline.py).  BENCH_ARGS adds bench flags.
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUTD="$ROOTD/gpurun_out/trace"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUTD" -o run -- \
  python3 "$ROOTD/bench.py" --steps 5 --warmup 3 --no-cpu-baseline --secondary= --streams 1 ${BENCH_ARGS:-} > "$OUTD/bench.log" 2>&1
rc=$?; tail -n 1 "$OUTD/bench.log" | cut -c1-200; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
python3 "$ROOTD/tools/timeline.py" "$OUTD" > "$OUTD/timeline.txt"
cat "$OUTD/timeline.txt"
