#!/usr/bin/env bash
# GPU session on one MI355X box (run through gpurun), every GPU step under its
# own limit, stop at the first failure.  STEPS (space-separated, default
# "test smoke bench prof"); output under gpurun_out/$TAG (TAG default r05):
#   test    pytest -m gpu (TESTS= overrides the selection, e.g. "-k nms"; TESTS_K= a -k expression with spaces)
#   smoke   __graft_entry__.smoke()
#   bench   the driver's exact command: python3 bench.py --gpus 1 --steps 20 --warmup 5
#   prof    rocprofv3 --kernel-trace --stats of the C2 driver command and of the
#           C3 / C5 objects alone, then PMC passes (one counter group per run,
#           kernel trace only beside --pmc) of each; prof_stages.py keeps each
#           timed region (5 warm-ups + 1 breakdown forward skipped, 20 kept; C5
#           runs 2 passes of 128 images per forward) -> $OUT/pmc.json
#           ("<stage>:split", "...@C3", "...@C5"), stamped with the kernel-source hash
#   ab      same-box A/B of diagnostic switches on libkpd_diag.so (make diag):
#           AB_ENVS="NAME=1;NAME2=1" (";"-separated variants, "-" = none), AB_CFG c2|c3|c5
#   stamps  KPD_STAMPS phase stamps of the heatmap convs (diag build)
#   bstamps KPD_STAMPS phase stamps of the body kernels (tools/stamps_probe.py, diag build)
#   grad    K6 backward timing at the heatmap conv 2 shape
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTD"
TAG="${TAG:-r05}"
OUT="$ROOTD/gpurun_out/$TAG"
mkdir -p "$OUT"
STEPS="${STEPS:-test smoke bench prof}"
summ() {   # one-line summary of a bench JSON line (C2 headline and config objects)
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
def show(tag, c, v):
    r = c.get("roofline") or {}
    print(tag, v, c.get("ms_per_step"), "dom", r.get("stage"), r.get("avg_ms"), "frac", r.get("frac"),
          "busy", r.get("mfma_busy_frac"), "traffic", r.get("traffic"), "cpu", (c.get("cpu_baseline") or {}).get("value"),
          "kh_tf", c.get("keypoint_head_tflops"))
    print("  stages", c.get("stages_ms"))
    print("  parity", c.get("parity"))
if "value" in d:
    show("C2", d, d["value"])
    print("  alt", (d.get("alt_streams") or {}).get("value"), "mixed", (d.get("secondary") or {}).get("value"))
for k, c in (d.get("configs") or {}).items():
    show(k, c, c.get("value"))
PY
}
for S in $STEPS; do
  case $S in
  test)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      -p no:cacheprovider ${TESTS:-} ${TESTS_K:+-k "$TESTS_K"} > "$OUT/pytest_gpu.log" 2>&1 \
      || { echo "pytest rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
    tail -1 "$OUT/pytest_gpu.log" ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
    tail -1 "$OUT/smoke.log" ;;
  bench)
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench_driver_cmd.json" \
      2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
    summ "$OUT/bench_driver_cmd.json" ;;
  prof)
    P="$OUT/prof"
    mkdir -p "$P"
    (
      cd /tmp && export TMPDIR=/tmp
      C2="python3 $ROOTD/bench.py --gpus 1 --steps 20 --warmup 5"
      C3="python3 $ROOTD/bench.py --only C3 --steps 20 --warmup 5 --no-cpu-baseline --alt-streams 0"
      C5="python3 $ROOTD/bench.py --only C5 --steps 20 --warmup 5 --no-cpu-baseline"
      for c in c2 c3 c5; do
        case $c in c2) CMD=$C2 ;; c3) CMD=$C3 ;; c5) CMD=$C5 ;; esac
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/$c/trace" -o run -- $CMD \
          > "$P/trace_$c.log" 2>&1 || { echo "trace $c rc=$?"; tail -5 "$P/trace_$c.log"; exit 1; }
      done
      IFS=";" read -ra PG <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE}"
      i=0
      for G in "${PG[@]}"; do
        i=$((i + 1))
        for c in c2 c3 c5; do
          case $c in c2) CMD="$C2 --no-cpu-baseline --configs none" ;; c3) CMD=$C3 ;; c5) CMD=$C5 ;; esac
          timeout -k 10 -s KILL 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d "$P/$c/pmc/p$i" -o run \
            -- $CMD > "$P/pmc_${c}_$i.log" 2>&1 || { echo "pmc $c pass $i ($G) rc=$?"; exit 1; }
        done
      done
    ) || exit 1
    python3 tools/prof_stages.py "$P/c2" --precision split --skip 6 --take 20 --out "$P/stages_c2.json" > "$P/stages_c2.txt"
    python3 tools/prof_stages.py "$P/c3" --precision split --skip 6 --take 20 --tag C3 --out "$P/stages_c3.json" > "$P/stages_c3.txt"
    python3 tools/prof_stages.py "$P/c5" --precision split --skip 12 --take 40 --tag C5 --out "$P/stages_c5.json" > "$P/stages_c5.txt"
    python3 - "$P" "$OUT/pmc.json" <<'PY'
import json, re, sys
p, out = sys.argv[1], sys.argv[2]
m = {}
for f in ("stages_c2.json", "stages_c3.json", "stages_c5.json"):
    d = json.load(open(f"{p}/{f}"))
    m.setdefault("_meta", {})[f] = d["_meta"]
    for k, v in d.items():
        if re.fullmatch(r"[a-z0-9_]+:(split|mixed|fp32)(@C[0-9])?", k):   # stage entries (not kernel names)
            m[k] = v
json.dump(m, open(out, "w"), indent=1)
for k, v in m.items():
    if ":" in k:
        print(k, {c: round(x, 4) if isinstance(x, float) else x for c, x in v.items()
                  if c in ("avg_us", "hbm_bytes_per_launch", "mfma_busy_frac")})
PY
    ;;
  ab)
    IFS=";" read -ra VARS <<< "${AB_ENVS:--}"
    for rep in 1 2; do
      for V in "${VARS[@]}"; do
        case "${AB_CFG:-c2}" in
          c3) ARGS="--only C3 --steps 10 --warmup 5 --no-cpu-baseline --alt-streams 0" ;;
          c5) ARGS="--only C5 --steps 10 --warmup 5 --no-cpu-baseline" ;;
          *) ARGS="--steps 20 --warmup 10 --no-cpu-baseline --configs none --secondary= --alt-streams 0 --no-exact-check" ;;
        esac
        if [ "$V" = "-" ]; then E=""; else E="$V"; fi
        env KPD_DIAG_LIB=1 $E timeout -k 10 300 python3 bench.py $ARGS > "$OUT/ab.json" 2> "$OUT/ab.err" \
          || { echo "ab rc=$? ($V)"; tail -5 "$OUT/ab.err"; exit 1; }
        python3 - "$OUT/ab.json" "$V" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = next(iter(d["configs"].values())) if "configs" in d and "value" not in d else d
print(sys.argv[2], "value", c["value"], "ms", c["ms_per_step"], {k: round(v, 3) for k, v in c["stages_ms"].items()})
PY
      done
    done ;;
  bstamps)
    # body / lateral-chain / ROI-align per-workgroup phase stamps (tools/stamps_probe.py)
    env KPD_DIAG_LIB=1 KPD_STAMPS=1 timeout -k 10 180 python3 tools/stamps_probe.py > "$OUT/stamps_body.txt" 2>&1 \
      || { echo "bstamps rc=$?"; tail -5 "$OUT/stamps_body.txt"; exit 1; }
    cat "$OUT/stamps_body.txt" | cut -c1-220 | head -120 ;;
  stamps)
    for k in ${STAMP_SETS:-stamps_hm1 stamps_hm2 stamps_hm3}; do
      env KPD_DIAG_LIB=1 KPD_STAMPS=1 timeout -k 10 120 python3 tools/stamps_hm2.py $k split \
        || { echo "stamps rc=$? ($k)"; exit 1; }
    done ;;
  grad)
    timeout -k 10 300 python3 tools/bench_conv3_grad.py --rois 64 > "$OUT/conv3_grad.json" 2> "$OUT/grad.err" \
      || { echo "grad rc=$?"; tail -5 "$OUT/grad.err"; exit 1; }
    cut -c1-600 "$OUT/conv3_grad.json" ;;
  *) echo "unknown step $S"; exit 1 ;;
  esac
done
