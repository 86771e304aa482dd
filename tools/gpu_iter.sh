#!/usr/bin/env bash
# One build->measure iteration on the GPU box: GPU parity tests, then a
# rocprofv3 kernel trace of a short single-stream bench and the per-kernel
# timeline of one forward (tools/timeline.py).  Every GPU step has its own
# time limit and a failure stops the script.
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUTD="$ROOTD/gpurun_out/iter"
mkdir -p "$OUTD"
cd "$ROOTD"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUTD/pytest.log" 2>&1
rc=$?; tail -n 5 "$OUTD/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUTD" -o run -- \
  python3 "$ROOTD/bench.py" --steps 5 --warmup 3 --no-cpu-baseline --streams 1 ${BENCH_ARGS:-} > "$OUTD/bench.log" 2>&1
rc=$?; tail -n 1 "$OUTD/bench.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
python3 "$ROOTD/tools/timeline.py" "$OUTD" > "$OUTD/timeline.txt"
cat "$OUTD/timeline.txt"
