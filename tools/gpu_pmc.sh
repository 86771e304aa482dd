#!/usr/bin/env bash
# HBM traffic of every kernel of a short bench run from rocprofv3 PMC counters,
# one counter group per pass (FETCH_SIZE and WRITE_SIZE do not fit one pass),
# kernel-trace only beside --pmc.  Summarised by tools/pmc_summary.py.
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
OUTD="$ROOTD/gpurun_out/pmc_$TAG"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUTD/$C" -o run -- \
    python3 "$ROOTD/bench.py" --steps 3 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUTD/$C.log" 2>&1 || exit $?
done
python3 "$ROOTD/tools/pmc_summary.py" "$OUTD" | tee "$OUTD/summary.txt"
