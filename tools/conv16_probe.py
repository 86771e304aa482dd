#!/usr/bin/env python3
"""Ablation timings of the LDS-DMA conv (kpd_bench_conv16): dbg 0 = the
production dispatch (launch_conv16), 65536 = the BN=128 / 3-stage kernel,
others = ablations of that kernel (no K-loop loads, no MFMAs, L2-resident A,
no epilogue, no K loop).  Prints one
JSON line per case (argv[1]: comma-separated dbg values)."""
import ctypes
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "keypoint-detection_amd"))
from dll import _native  # noqa: E402

lib = _native.load()
CASES = [  # (label, split, N, H, W, cin, cout, flop)
    ("fpn0_split", 1, 64, 128, 96, 128, 128, 2 * 64 * 128 * 96 * 128 * 128 * 9 * 3),
    ("hm1_bf16", 0, 64, 56, 56, 64, 256, 2 * 64 * 56 * 56 * 64 * 256 * 9),
    ("hm2_bf16", 0, 64, 56, 56, 256, 256, 2 * 64 * 56 * 56 * 256 * 256 * 9),
]
# warm-up (clocks / caches): the first timed case of a process otherwise reads ~5% slow
for label, split, N, H, W, cin, cout, flop in CASES:
    lib.kpd_bench_conv16(split, N, H, W, cin, cout, 0, 30, ctypes.byref(ctypes.c_float(0)))
for label, split, N, H, W, cin, cout, flop in CASES:
    for dbg in [int(v) for v in (sys.argv[1].split(',') if len(sys.argv) > 1 else '0,1,2,4,8,16,24'.split(','))]:
        ms = ctypes.c_float(0)
        rc = lib.kpd_bench_conv16(split, N, H, W, cin, cout, dbg, 40, ctypes.byref(ms))
        print(json.dumps({"case": label, "dbg": dbg, "rc": rc, "ms": round(ms.value, 4),
                          "mfma_tflops": round(flop / (ms.value * 1e-3) / 1e12, 1) if rc == 0 and ms.value else None}),
              flush=True)
