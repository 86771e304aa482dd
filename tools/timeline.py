#!/usr/bin/env python3
"""Per-kernel timeline of the last complete forward in a rocprofv3
kernel-trace CSV (tools/gpu_iter.sh): duration, gap to the previous kernel,
grid/workgroup/VGPR/LDS, and the per-stage sums of the body.
    python3 tools/timeline.py gpurun_out/iter/run_kernel_trace.csv
"""
import csv
import glob
import sys


def main(path):
    if not path.endswith(".csv"):
        path = glob.glob(path + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "stem_" in r["Kernel_Name"]]
    s, e = idx[-2], idx[-1]
    prev = None
    body = 0.0
    in_body = True
    for r in rows[s:e]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (st - prev) / 1000 if prev else 0.0
        prev = en
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        if "split_rows" in name or "lateral" in name or "fpn0x" in name:
            in_body = False
        if in_body:
            body += (en - st) / 1000
        print(f"{(en - st) / 1000:8.1f} gap {gap:6.1f}  {name[:72]:72s} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} "
              f"wg={r['Workgroup_Size_X']} vgpr={r['VGPR_Count']} agpr={r.get('Accum_VGPR_Count', '')} "
              f"lds={r['LDS_Block_Size']}")
    span = (int(rows[e - 1]["End_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1000
    print(f"forward span {span:.1f} us; body kernels (stem .. before the FPN laterals' split) {body:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
