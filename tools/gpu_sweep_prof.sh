#!/usr/bin/env bash
# Kernel-trace A/B sweep: for each "NAME=VAL ..." argument, a rocprofv3 kernel
# trace of a short single-stream bench under those env vars, then the
# per-kernel timeline of one forward (tools/timeline.py) filtered by
# $SWEEP_GREP (default: all kernels of the body).
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i + 1))
  OUTD="$ROOTD/gpurun_out/sweep/c$i"
  mkdir -p "$OUTD"
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUTD" -o run -- \
    python3 "$ROOTD/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --streams 1 ${BENCH_ARGS:-} > "$OUTD/bench.log" 2>&1 \
    || { echo "FAILED: $cfg"; tail -5 "$OUTD/bench.log"; exit 1; }
  python3 "$ROOTD/tools/timeline.py" "$OUTD" > "$OUTD/timeline.txt"
  echo "=== ${cfg:-base}"
  grep -E "${SWEEP_GREP:-exdw|seproj|se_kernel|splitk|conv_mfma|forward span}" "$OUTD/timeline.txt" | cut -c1-110
done
