#!/usr/bin/env bash
# rocprofv3 PMC passes over a short bench run (kernel-trace only beside --pmc,
# one counter group per pass).  Default: HBM traffic (FETCH_SIZE, WRITE_SIZE);
# PMC_GROUPS="G1;G2;..." (space-separated counters per group) overrides.
# Summarised per kernel by tools/pmc_summary.py.
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
OUTD="$ROOTD/gpurun_out/pmc_$TAG"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
GROUPS_STR="${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE}"
IFS=";" read -ra PGROUPS <<< "$GROUPS_STR"
i=0
for G in "${PGROUPS[@]}"; do
  i=$((i + 1))
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --pmc $G --kernel-trace --output-format csv -d "$OUTD/pass$i" -o run -- \
    python3 "$ROOTD/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --streams 1 ${BENCH_ARGS:-} > "$OUTD/pass$i.log" 2>&1 || exit $?
done
python3 "$ROOTD/tools/pmc_summary.py" "$OUTD" | tee "$OUTD/summary.txt"
