#!/usr/bin/env bash
# Round-4 GPU session, every GPU step under its own limit, stop at the first
# failure.  STEPS (space-separated, default "test smoke bench prof"):
#   test   pytest -m gpu (TESTS= overrides the selection, e.g. "-k detector")
#   smoke  __graft_entry__.smoke()
#   bench  the driver's exact command: python3 bench.py --gpus 1 --steps 20 --warmup 5
#   prof   rocprofv3 --kernel-trace --stats of that command, then PMC passes (one
#          counter group per run) of it and of the C3-only run; prof_stages.py
#          keeps each timed region (forwards 7..26: 5 warm-ups + 1 breakdown
#          forward first) -> gpurun_out/r04/pmc.json ("<stage>:split" for C2,
#          "<stage>:split@C3" for C3), stamped with the kernel-source hash
set -u
ROOTD="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTD"
OUT="$ROOTD/gpurun_out/r04"
mkdir -p "$OUT"
STEPS="${STEPS:-test smoke bench prof}"
for S in $STEPS; do
  case $S in
  test)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      -p no:cacheprovider ${TESTS:-} > "$OUT/pytest_gpu.log" 2>&1 \
      || { echo "pytest rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
    tail -1 "$OUT/pytest_gpu.log" ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
    tail -1 "$OUT/smoke.log" ;;
  bench)
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench_driver_cmd.json" \
      2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
    python3 - "$OUT/bench_driver_cmd.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("C2", d["value"], d["ms_per_step"], "frac", r["frac"], "avg_ms", r["avg_ms"], "traffic", r["traffic"],
      "alt", (d.get("alt_streams") or {}).get("value"), "mixed", (d.get("secondary") or {}).get("value"),
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
print("C2 stages", d["stages_ms"])
print("C2 parity", d.get("parity"))
c = (d.get("configs") or {}).get("C3")
if c:
    r = c["roofline"]
    print("C3", c["value"], c["ms_per_step"], "frac", r["frac"], "avg_ms", r["avg_ms"], "traffic", r["traffic"],
          "alt", (c.get("alt_streams") or {}).get("value"), "cpu", (c.get("cpu_baseline") or {}).get("value"),
          "kh_tflops", c.get("keypoint_head_tflops"))
    print("C3 stages", c["stages_ms"])
    print("C3 parity", c.get("parity"))
PY
    ;;
  prof)
    P="$OUT/prof"
    mkdir -p "$P"
    (
      cd /tmp && export TMPDIR=/tmp
      C2="python3 $ROOTD/bench.py --gpus 1 --steps 20 --warmup 5"
      C3="python3 $ROOTD/bench.py --c3-only --steps 20 --warmup 5 --no-cpu-baseline --alt-streams 0"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/trace_c2" -o run -- $C2 \
        > "$P/trace_c2.log" 2>&1 || { echo "trace c2 rc=$?"; tail -5 "$P/trace_c2.log"; exit 1; }
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/trace_c3" -o run -- $C3 \
        > "$P/trace_c3.log" 2>&1 || { echo "trace c3 rc=$?"; tail -5 "$P/trace_c3.log"; exit 1; }
      IFS=";" read -ra PG <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE}"
      i=0
      for G in "${PG[@]}"; do
        i=$((i + 1))
        timeout -k 10 -s KILL 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d "$P/pmc_c2/p$i" -o run -- \
          $C2 --no-cpu-baseline --c3 0 > "$P/pmc_c2_$i.log" 2>&1 || { echo "pmc c2 pass $i ($G) rc=$?"; exit 1; }
        timeout -k 10 -s KILL 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d "$P/pmc_c3/p$i" -o run -- \
          $C3 > "$P/pmc_c3_$i.log" 2>&1 || { echo "pmc c3 pass $i ($G) rc=$?"; exit 1; }
      done
    ) || exit 1
    mkdir -p "$P/c2" "$P/c3"
    cp -r "$P/trace_c2" "$P/c2/trace" && cp -r "$P/pmc_c2" "$P/c2/pmc"
    cp -r "$P/trace_c3" "$P/c3/trace" && cp -r "$P/pmc_c3" "$P/c3/pmc"
    python3 tools/prof_stages.py "$P/c2" --precision split --skip 6 --take 20 --out "$P/stages_c2.json" > "$P/stages_c2.txt"
    python3 tools/prof_stages.py "$P/c3" --precision split --skip 6 --take 20 --tag C3 --out "$P/stages_c3.json" > "$P/stages_c3.txt"
    python3 - "$P" "$OUT/pmc.json" <<'PY'
import json, sys
p, out = sys.argv[1], sys.argv[2]
m = {}
for f in ("stages_c2.json", "stages_c3.json"):
    d = json.load(open(f"{p}/{f}"))
    m.setdefault("_meta", {})[f] = d["_meta"]
    for k, v in d.items():
        if ":" in k:
            m[k] = v
json.dump(m, open(out, "w"), indent=1)
for k, v in m.items():
    if ":" in k:
        print(k, {c: round(x, 4) if isinstance(x, float) else x for c, x in v.items()
                  if c in ("avg_us", "hbm_bytes_per_launch", "mfma_busy_frac")})
PY
    ;;
  ab)
    # same-box A/B of diagnostic switches on the diagnostic build (make diag):
    # AB_ENVS="NAME=1;NAME2=1" (";"-separated variants, "-" = none), AB_CFG c2|c3
    IFS=";" read -ra VARS <<< "${AB_ENVS:--}"
    for rep in 1 2; do
      for V in "${VARS[@]}"; do
        if [ "${AB_CFG:-c3}" = c3 ]; then ARGS="--c3-only --steps 10 --warmup 5 --no-cpu-baseline --alt-streams 0"
        else ARGS="--steps 20 --warmup 10 --no-cpu-baseline --c3 0 --secondary split --alt-streams 0"; fi
        if [ "$V" = "-" ]; then E=""; else E="$V"; fi
        env KPD_DIAG_LIB=1 $E timeout -k 10 300 python3 bench.py $ARGS > "$OUT/ab.json" 2> "$OUT/ab.err" \
          || { echo "ab rc=$? ($V)"; tail -5 "$OUT/ab.err"; exit 1; }
        python3 - "$OUT/ab.json" "$V" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("configs", {}).get("C3") or d
print(sys.argv[2], "value", c["value"], "ms", c["ms_per_step"], {k: round(v, 3) for k, v in c["stages_ms"].items()})
PY
      done
    done ;;
  grad)
    # K6 backward timing at the heatmap conv 2 shape
    timeout -k 10 300 python3 tools/bench_conv3_grad.py --rois 64 > "$OUT/conv3_grad.json" 2> "$OUT/grad.err" \
      || { echo "grad rc=$?"; tail -5 "$OUT/grad.err"; exit 1; }
    cut -c1-600 "$OUT/conv3_grad.json" ;;
  *) echo "unknown step $S"; exit 1 ;;
  esac
done
