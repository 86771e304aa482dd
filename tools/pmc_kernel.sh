#!/usr/bin/env bash
# PMC counters of selected kernels in a short C2 bench: one rocprofv3 --pmc
# pass per ";"-separated counter group (PMC_SETS), kernel trace only beside it.
# Prints per-kernel mean counter values for kernels matching KRE (regex).
#   TAG=r06 PMC_SETS="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT;SQ_INSTS_VALU" KRE="fir23|exdw" bash tools/pmc_kernel.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r06}"; O="$R/gpurun_out/$TAG/pmck"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 3 --no-cpu-baseline --configs none --secondary= --alt-streams 0 --no-exact-check"
IFS=";" read -ra PG <<< "${PMC_SETS:-SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE}"
i=0
for G in "${PG[@]}"; do
  i=$((i + 1))
  env ${ENVS:-} timeout -k 10 -s KILL 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d "$O/p$i" -o run -- \
    python3 "$R/bench.py" $ARGS > "$O/p$i.log" 2>&1 || { echo "pmc pass $i ($G) rc=$?"; tail -3 "$O/p$i.log"; exit 1; }
done
python3 - "$O" "${KRE:-fir23}" <<'PY'
import csv, glob, re, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if re.search(sys.argv[2], r["Kernel_Name"]):
            acc[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):14.1f}  (n={len(v)})")
PY
