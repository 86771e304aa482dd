#!/usr/bin/env bash
# Round-2 profile session on the GPU box: (1) kernel trace + stats of a bench
# run (steady state split out by tools/prof_stages.py), (2) PMC passes --
# HBM traffic (FETCH_SIZE; WRITE_SIZE) and MFMA occupancy (SQ_VALU_MFMA_BUSY_CYCLES,
# SQ_BUSY_CU_CYCLES, GRBM_GUI_ACTIVE + wave-state counters) -- each pass its own
# run under its own time limit.  PREC (split|mixed|fp32) selects the precision.
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
PREC="${PREC:-split}"
OUTD="$ROOTD/gpurun_out/prof_$PREC"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
BARGS="--steps 10 --warmup 40 --no-cpu-baseline --secondary= --alt-streams 0 --streams 1 --precision $PREC"  # past the clock ramp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUTD/trace" -o run -- \
  python3 "$ROOTD/bench.py" $BARGS > "$OUTD/trace.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
i=0
IFS=";" read -ra PG <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE}"
for G in "${PG[@]}"; do
  i=$((i + 1))
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $G --kernel-trace --output-format csv -d "$OUTD/pmc$i" -o run -- \
    python3 "$ROOTD/bench.py" $BARGS > "$OUTD/pmc$i.log" 2>&1 || { echo "pmc pass $i ($G) rc=$?"; exit 1; }
done
python3 "$ROOTD/tools/prof_stages.py" "$OUTD" --precision "$PREC" --skip 42 --out "$OUTD/stages.json"
