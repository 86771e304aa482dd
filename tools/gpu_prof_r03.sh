#!/usr/bin/env bash
# Round-3 profile of the driver's exact bench command
#   python3 bench.py --gpus 1 --steps 20 --warmup 5
# (1) rocprofv3 --kernel-trace --stats of that command, (2) PMC passes of the
# same command, each its own run under its own time limit; prof_stages.py
# keeps the headline's timed region only (forwards 7..26: --warmup 5 and the
# one stage-breakdown forward come first) and stamps every entry with the
# kernel-source hash bench.py compares against.
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUTD="$ROOTD/gpurun_out/prof_r03"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
CMD="python3 $ROOTD/bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/trace" -o run -- $CMD \
  > "$OUTD/trace.log" 2>&1 || { echo "trace rc=$?"; tail -5 "$OUTD/trace.log"; exit 1; }
i=0
IFS=";" read -ra PG <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE}"
for G in "${PG[@]}"; do
  i=$((i + 1))
  timeout -k 10 -s KILL 400 rocprofv3 --pmc $G --kernel-trace --output-format csv -d "$OUTD/pmc$i" -o run -- \
    $CMD > "$OUTD/pmc$i.log" 2>&1 || { echo "pmc pass $i ($G) rc=$?"; exit 1; }
done
cd "$ROOTD"
python3 tools/prof_stages.py "$OUTD" --precision split --skip 6 --take 20 --out "$OUTD/stages.json"
