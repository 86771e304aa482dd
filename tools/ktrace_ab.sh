#!/usr/bin/env bash
# Same-box per-kernel A/B: kernel traces (tools/ktrace.sh) of the current
# library and of libkpd_base.so (tools/build_base.sh), alternated ROUNDS times
# (default 2), then one table of mean kernel durations per variant and the
# difference (current - base).  Kernel means move by ~0.1 us between runs on
# one box, where the stage timings of `gpu_session.sh ab` move by ~10 us.
#   gpurun -- 'TAG=r06x bash tools/ktrace_ab.sh'      (CFG c2|c3|c5, KRE kernel regex)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r06}"; CFG="${CFG:-c2}"; ROUNDS="${ROUNDS:-2}"
B="$R/keypoint-detection_amd/dll/_lib/libkpd_base.so"
[ -f "$B" ] || { echo "no $B (tools/build_base.sh first)"; exit 1; }
for i in $(seq 1 "$ROUNDS"); do
  TAG=$TAG CFG=$CFG SUFFIX=_new$i bash "$R/tools/ktrace.sh" > /dev/null || exit 1
  TAG=$TAG CFG=$CFG SUFFIX=_base$i ENVS="KPD_LIB=$B" bash "$R/tools/ktrace.sh" > /dev/null || exit 1
done
python3 - "$R/gpurun_out/$TAG" "$CFG" "$ROUNDS" "${KRE:-.}" <<'PY' | tee "$R/gpurun_out/$TAG/ktrace_ab_$CFG.txt"
import csv, glob, re, sys
root, cfg, rounds, kre = sys.argv[1], sys.argv[2], int(sys.argv[3]), re.compile(sys.argv[4])
def means(sfx):
    f = glob.glob(f"{root}/kt_{cfg}{sfx}/**/*kernel_stats.csv", recursive=True)[0]
    return {r["Name"]: (float(r["AverageNs"]) / 1e3, int(r["Calls"])) for r in csv.DictReader(open(f))}
new = [means(f"_new{i}") for i in range(1, rounds + 1)]
base = [means(f"_base{i}") for i in range(1, rounds + 1)]
names = sorted(set(new[0]) | set(base[0]), key=lambda k: -(new[0].get(k, base[0].get(k, (0, 0)))[0] *
                                                           new[0].get(k, base[0].get(k, (0, 0)))[1]))
print(f"{'kernel':70s} {'new (us)':>18s} {'base (us)':>18s} {'diff':>7s}")
for k in names:
    if not kre.search(k):
        continue
    nv = [m[k][0] for m in new if k in m]
    bv = [m[k][0] for m in base if k in m]
    d = (sum(nv) / len(nv) - sum(bv) / len(bv)) if nv and bv else float("nan")
    print(f"{k[:70]:70s} {' '.join(f'{v:8.2f}' for v in nv):>18s} {' '.join(f'{v:8.2f}' for v in bv):>18s} {d:7.2f}")
PY
