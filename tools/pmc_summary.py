#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh) per kernel.

Every counter is averaged per dispatch of a kernel.  When FETCH_SIZE and
WRITE_SIZE are present, HBM bytes per launch = 2 * FETCH_SIZE * 1024 +
WRITE_SIZE * 1024 (MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half
the bytes of a wide 16-B/lane coalesced read stream -- the conv staging loads
are 16-B/lane loads; WRITE_SIZE is read as-is; both in KB).  Derived stall
ratios are printed when the SQ counters are present.  Writes <outdir>/pmc.json.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

STAGE_OF = {   # kernel-name substring -> "<stage>:<bench precision>"
    "conv_mfma_kernel<float, float, 3, 128, 128, 32": "fpn0:fp32",
    "conv16_kernel<true": "fpn0:mixed",       # direct 3x3 over lateral 0 (KPD_NO_FPN0X=1)
    "fpn0x_kernel": "fpn0:mixed",             # FPN level 0 by linearity (default)
}


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(ConvArgs")[0].split("(Split16")[0]


def main(outdir):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Value") is None:
                    continue
                vals[short(row.get("Kernel_Name", ""))][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for k, cs in vals.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        e["launches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in e or "WRITE_SIZE" in e:
            e["hbm_bytes_per_launch"] = 2 * e.get("FETCH_SIZE", 0.0) * 1024 + e.get("WRITE_SIZE", 0.0) * 1024
        wc = e.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
                if c in e:
                    e["frac_" + c] = e[c] / wc
        if e.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_ratio"] = e.get("SQ_LDS_BANK_CONFLICT", 0.0) / e["SQ_LDS_IDX_ACTIVE"]
        res[k] = e
        for sub, stage in STAGE_OF.items():
            if sub in k:
                res[stage] = dict(e, kernel=k, correction="2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 16B/lane reads)")
    order = sorted(res.items(), key=lambda kv: -kv[1].get("hbm_bytes_per_launch", kv[1].get("SQ_WAVE_CYCLES", 0)))
    for k, e in order:
        if ":" in k:
            continue
        parts = []
        if "hbm_bytes_per_launch" in e:
            parts.append(f"{e['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch")
        for c in sorted(e):
            if c.startswith("frac_") or c == "lds_conflict_ratio":
                parts.append(f"{c.replace('frac_SQ_', '')}={e[c]:.3f}")
        for c in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            if c in e:
                parts.append(f"{c.replace('SQ_', '')}={e[c]:.3g}")
        print(f"x{e['launches']:4d} {k[:70]:70s} " + " ".join(parts))
    with open(os.path.join(outdir, "pmc.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
