#!/usr/bin/env python3
"""Steady-state per-stage summaries of rocprofv3 runs of bench.py.

    prof_stages.py <rocprof_outdir> --precision split [--skip 2] [--out profiles/r02/x.json]

Dispatches are ordered (Dispatch_Id, else start time) and cut into forwards at
each stem_kernel launch (the first kernel of every forward); the first --skip
forwards (plan setup, warm-up) and everything before the first forward
(weight upload copies, workspace fills) are dropped, so the numbers describe
the steady state only.  Kernels are labelled with the plan's stage names:
fpn0x_kernel -> fpn0; hmconv_kernel<64,...> -> hm_conv3; the first / second
hmconv_kernel<256|128,...> of a forward -> hm_conv1 / hm_conv2.  A stage
with several launches in one forward (conv 3 and its 128-row tail launch) is
summed per forward: "per launch" below means per stage execution.

kernel_trace.csv -> mean / min / max duration per stage and per kernel.
counter_collection.csv (--pmc passes) -> counters averaged per stage; HBM
bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (gfx950: FETCH_SIZE
reports half the bytes of 16-byte-per-lane streaming reads, MI355X_MICROARCH.md
§HBM); MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8 XCDs).  Writes JSON keyed "<stage>:<precision>" (the key
bench.py --pmc-json reads) plus per-kernel entries.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0] if "(" in n else n


def label(forward):
    """Stage label per dispatch of one forward (list of kernel names)."""
    out, hm = [], 0
    for k in forward:
        targs = [t.strip() for t in k[len("hmconv_kernel<"):].split(">")[0].split(",")] \
            if k.startswith("hmconv_kernel<") else []
        margs = [t.strip() for t in k[len("hmconv_mixed_kernel<"):].split(">")[0].split(",")] \
            if k.startswith("hmconv_mixed_kernel<") else []
        if k.startswith("fpn0x_kernel"):
            out.append("fpn0")
        elif margs:   # <BN, SB, BMH, BMT, CIN, ...>: full + tail tiles in one launch
            out.append("hm_conv3" if margs[0] == "64" else "hm_conv1" if margs[4] == "64" else "hm_conv2")
        elif len(targs) >= 10 and targs[9] == "2":
            out.append("kh_conv")   # KEYPOINT_HEAD convs (MODE 2), dual-head configs
        elif k.startswith("hmconv_kernel<64"):
            out.append("hm_conv3")
        elif k.startswith("hmconv_kernel<"):
            # conv 1 / conv 2 by the compile-time input channels (6th template
            # argument: 64 / 256; a conv may be two launches), else by order
            hm += 1
            if len(targs) >= 6 and targs[5] in ("64", "256"):
                out.append("hm_conv1" if targs[5] == "64" else "hm_conv2")
            else:
                out.append("hm_conv1" if hm == 1 else "hm_conv2")
        else:
            out.append(None)
    return out


def forwards(rows, key):
    """rows: list of (order, name, payload) -> list of forwards [(name, payload), ...]."""
    rows.sort(key=key)
    fw, cur = [], None
    for r in rows:
        if r[1].startswith("stem_kernel") or r[1].startswith("stem_band_kernel"):
            cur = []
            fw.append(cur)
        if cur is not None:
            cur.append((r[1], r[2]))
    return fw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--precision", default="split")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--take", type=int, default=0, help="forwards kept after --skip (0 = all): the bench's timed region")
    ap.add_argument("--out", default=None)
    ap.add_argument("--tag", default=None, help="config tag appended to the stage keys ('<stage>:<precision>@<tag>', "
                                                "e.g. C3): the key bench.py reads for that config's roofline")
    a = ap.parse_args()
    # repo-relative source path (the GPU box's scratch root differs per call)
    src = os.path.relpath(os.path.abspath(a.outdir), os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
    res = {"_meta": {"source": src, "precision": a.precision, "skip_forwards": a.skip, "take_forwards": a.take,
                     "tag": a.tag}}
    pk = a.precision + (f"@{a.tag}" if a.tag else "")     # the key suffix of the stage entries
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import kernel_src_hash
    res["_meta"]["src_hash"] = kernel_src_hash()
    # ---- kernel trace
    kt = []
    tdir = os.path.join(a.outdir, "trace") if os.path.isdir(os.path.join(a.outdir, "trace")) else a.outdir
    for f in glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                kt.append((t0, short(r["Kernel_Name"]), (t1 - t0) * 1e-3))
    if kt:
        fw = forwards(kt, key=lambda r: r[0])[a.skip:]
        if a.take:
            fw = fw[:a.take]
        st, kn = defaultdict(list), defaultdict(list)
        for f in fw:
            per = defaultdict(float)   # a stage may be several launches (conv 3 + its tail launch): summed
            for (name, us), lab in zip(f, label([n for n, _ in f])):
                kn[name].append(us)
                if lab:
                    per[lab] += us
            for lab, us in per.items():
                st[lab].append(us)
        res["_meta"]["forwards_traced"] = len(fw)
        res["_meta"]["forward_kernel_us"] = round(sum(sum(v) for v in kn.values()) / max(len(fw), 1), 2)
        for lab, v in st.items():
            res[f"{lab}:{pk}"] = {"avg_us": round(sum(v) / len(v), 3), "min_us": round(min(v), 3),
                                           "max_us": round(max(v), 3), "launches": len(v),
                                           "src_hash": res["_meta"]["src_hash"]}
        res["kernels_us"] = {k: {"avg_us": round(sum(v) / len(v), 3), "calls": len(v),
                                 "per_forward_us": round(sum(v) / max(len(fw), 1), 3)}
                             for k, v in sorted(kn.items(), key=lambda kv: -sum(kv[1]))}
    # ---- counters
    disp = defaultdict(dict)
    names = {}
    for f in glob.glob(os.path.join(a.outdir, "**", "*counter_collection.csv"), recursive=True):
        tag = os.path.relpath(f, a.outdir).split(os.sep)[0]
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Value") in (None, ""):
                    continue
                did = (tag, int(r.get("Dispatch_Id") or r.get("Correlation_Id")))
                disp[did][r["Counter_Name"]] = disp[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                names[did] = short(r["Kernel_Name"])
    if disp:
        per_tag = defaultdict(list)
        for (tag, did), cs in disp.items():
            per_tag[tag].append((did, names[(tag, did)], cs))
        agg = defaultdict(lambda: defaultdict(list))
        for tag, rows in per_tag.items():
            fws = forwards(rows, key=lambda r: r[0])[a.skip:]
            for f in (fws[:a.take] if a.take else fws):
                per = defaultdict(lambda: defaultdict(float))
                for (name, cs), lab in zip(f, label([n for n, _ in f])):
                    for c, v in cs.items():
                        if lab:
                            per[lab][c] += v
                        agg[name][c].append(v)
                for lab, cs in per.items():
                    for c, v in cs.items():
                        agg[f"{lab}:{pk}"][c].append(v)
        for k, cs in agg.items():
            e = res.setdefault(k, {}) if ":" in k else res.setdefault("counters", {}).setdefault(k, {})
            for c, v in cs.items():
                e[c] = sum(v) / len(v)
            if "FETCH_SIZE" in e or "WRITE_SIZE" in e:
                e["hbm_bytes_per_launch"] = 2 * e.get("FETCH_SIZE", 0.0) * 1024 + e.get("WRITE_SIZE", 0.0) * 1024
            if e.get("SQ_VALU_MFMA_BUSY_CYCLES") and e.get("GRBM_GUI_ACTIVE"):   # (a stage's launches summed)
                e["mfma_busy_frac"] = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (128.0 * e["GRBM_GUI_ACTIVE"])
            if ":" in k:
                e["source"] = src
                e["src_hash"] = res["_meta"]["src_hash"]
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt)
    for k, e in res.items():
        if ":" in k:
            print(k, {c: (round(v, 4) if isinstance(v, float) else v) for c, v in e.items()
                      if c in ("avg_us", "min_us", "launches", "hbm_bytes_per_launch", "mfma_busy_frac",
                               "FETCH_SIZE", "WRITE_SIZE", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")})


if __name__ == "__main__":
    main()
