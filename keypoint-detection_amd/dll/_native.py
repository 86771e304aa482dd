"""ctypes binding of libkpd.so (include/kpd.h).

The product path has no CPU fallback: if the library is missing or fails to
load, every entry point raises ``KpdNativeError`` loudly.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

import torch

_LIB_PATH = Path(__file__).resolve().parent / "_lib" / "libkpd.so"
_lib: Optional[ctypes.CDLL] = None

KPD_PRECISION_FP32 = 0
KPD_PRECISION_MIXED = 1
KPD_PRECISION_SPLIT = 2
# "fp32": every conv on fp32-input MFMA; "split": fp32-accurate -- FPN level 0
# and the heatmap-head convs as three f16 MFMA products of hi/lo operand
# splits (fp32 tolerances); "mixed": split FPN level 0 + bf16 heatmap convs
PRECISIONS = {"fp32": KPD_PRECISION_FP32, "split": KPD_PRECISION_SPLIT, "mixed": KPD_PRECISION_MIXED,
              "bf16": KPD_PRECISION_MIXED}

# every symbol include/kpd.h declares (checked by tests/test_abi.py)
EXPORTS = ("kpd_last_error", "kpd_version", "kpd_plan_create", "kpd_plan_set_tensor",
           "kpd_plan_finalize", "kpd_plan_destroy", "kpd_forward", "kpd_debug_copy", "kpd_nms",
           "kpd_plan_timing", "kpd_plan_timing_stage", "kpd_plan_timing_query", "kpd_plan_set_detector",
           "kpd_bench_conv16",
           "kpd_plan_set_streams", "kpd_preprocess", "kpd_target_heatmaps", "kpd_keypoint_metrics")
FLAG_DETECT = 1
FLAG_DUAL_HEAD = 2
STAGES = ("body", "fpn_lateral", "fpn0", "topk", "person_detect", "roi_align", "hm_attention", "hm_conv1",
          "hm_conv2", "hm_conv3", "hm_final_decode", "keypoint_head")


class KpdNativeError(RuntimeError):
    pass


def lib_path() -> Path:
    return Path(os.environ.get("KPD_LIB", str(_LIB_PATH)))


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    p = lib_path()
    if not p.exists():
        raise KpdNativeError(f"libkpd.so not found at {p}; build it with "
                             f"`make -C keypoint-detection_amd/csrc` (or __graft_entry__.build())")
    lib = ctypes.CDLL(str(p))
    c_int, c_void_p, c_char_p = ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p
    lib.kpd_last_error.restype = c_char_p
    lib.kpd_version.restype = c_char_p
    lib.kpd_plan_create.argtypes = [c_int, c_int, ctypes.POINTER(c_void_p)]
    lib.kpd_plan_set_tensor.argtypes = [c_void_p, c_char_p, c_void_p, ctypes.POINTER(ctypes.c_int64), c_int]
    lib.kpd_plan_finalize.argtypes = [c_void_p, c_int]
    lib.kpd_plan_destroy.argtypes = [c_void_p]
    lib.kpd_plan_destroy.restype = None
    lib.kpd_forward.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.kpd_plan_set_detector.argtypes = [c_void_p, ctypes.c_float, ctypes.c_float]
    lib.kpd_debug_copy.argtypes = [c_void_p, c_char_p, c_void_p, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t), c_void_p]
    lib.kpd_plan_timing.argtypes = [c_void_p, c_int]
    lib.kpd_plan_timing_stage.argtypes = [c_void_p, c_char_p]
    lib.kpd_plan_timing_query.argtypes = [c_void_p, c_char_p, ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(c_int)]
    lib.kpd_target_heatmaps.argtypes = [c_void_p, c_int, c_int, c_int, ctypes.c_float, c_void_p, c_void_p]
    lib.kpd_keypoint_metrics.argtypes = [c_void_p, c_void_p, c_void_p, ctypes.c_long, ctypes.POINTER(ctypes.c_float),
                                         c_int, c_void_p, c_void_p]
    lib.kpd_nms.argtypes = [c_void_p, c_void_p, c_int, ctypes.c_float, c_int, c_void_p, c_void_p, c_void_p]
    for name in EXPORTS:
        if name not in ("kpd_last_error", "kpd_version", "kpd_plan_destroy"):
            getattr(lib, name).restype = c_int
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().kpd_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(f"{what}: {msg}")
        raise KpdNativeError(f"{what} failed ({rc}): {msg}")


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_cuda(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise KpdNativeError(f"{name} must be a HIP device tensor (got {t.device}); the native path "
                             f"has no CPU fallback")


class Plan:
    """Owns one ``kpd_plan`` (packed weights + workspace) on one device."""

    def __init__(self, device: torch.device, in_channels: int):
        self.lib = load()
        self.device = device
        h = ctypes.c_void_p()
        check(self.lib.kpd_plan_create(device.index or 0, in_channels, ctypes.byref(h)), "kpd_plan_create")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.lib.kpd_plan_destroy(h)
            self.h = None

    def set_tensor(self, name: str, t: torch.Tensor) -> None:
        t = t.detach().to("cpu", torch.float32).contiguous()
        shape = (ctypes.c_int64 * max(t.dim(), 1))(*t.shape)
        check(self.lib.kpd_plan_set_tensor(self.h, name.encode(), ctypes.c_void_p(t.data_ptr()), shape, t.dim()),
              f"kpd_plan_set_tensor({name})")

    def finalize(self, precision: int) -> None:
        check(self.lib.kpd_plan_finalize(self.h, precision), "kpd_plan_finalize")

    def set_detector(self, conf_threshold: float, nms_iou_threshold: float) -> None:
        check(self.lib.kpd_plan_set_detector(self.h, float(conf_threshold), float(nms_iou_threshold)),
              "kpd_plan_set_detector")

    def set_streams(self, n: int) -> None:
        """Sub-batch streams for large batches (kpd_plan_set_streams)."""
        check(self.lib.kpd_plan_set_streams(self.h, int(n)), "kpd_plan_set_streams")

    def forward(self, image: torch.Tensor, boxes: Optional[torch.Tensor], kpts, vis, heat, flags: int = 0,
                kh_kpts=None, kh_vis=None, box_scores=None, topk=None) -> None:
        """boxes [nb,P,4] (input; an output filled by the detector with FLAG_DETECT)."""
        _require_cuda(image, "image")
        B, C, H, W = image.shape
        nb, P = (0, 0) if boxes is None else (boxes.shape[0], boxes.shape[1])
        with torch.cuda.device(self.device):
            check(self.lib.kpd_forward(self.h, _ptr(image), B, C, H, W, _ptr(boxes), nb, P, int(flags), _ptr(kpts),
                                       _ptr(vis), _ptr(heat), _ptr(kh_kpts), _ptr(kh_vis), _ptr(box_scores),
                                       _ptr(topk), _stream(self.device)), "kpd_forward")

    def timing(self, enable: bool, stage: Optional[str] = None) -> None:
        """Record per-stage HIP events on the launch streams (only ``stage`` if given)."""
        check(self.lib.kpd_plan_timing_stage(self.h, stage.encode() if stage else None), "kpd_plan_timing_stage")
        check(self.lib.kpd_plan_timing(self.h, 1 if enable else 0), "kpd_plan_timing")

    def timing_query(self, stage: str):
        """(total_ms, launches) recorded for ``stage`` since timing(True)."""
        ms, n = ctypes.c_double(), ctypes.c_int()
        check(self.lib.kpd_plan_timing_query(self.h, stage.encode(), ctypes.byref(ms), ctypes.byref(n)),
              "kpd_plan_timing_query")
        return ms.value, n.value

    def debug_buffer(self, name: str) -> torch.Tensor:
        n = ctypes.c_size_t()
        check(self.lib.kpd_debug_copy(self.h, name.encode(), None, 0, ctypes.byref(n), None), "kpd_debug_copy")
        out = torch.empty(n.value // 4, dtype=torch.float32, device=self.device)
        check(self.lib.kpd_debug_copy(self.h, name.encode(), _ptr(out), n.value, None, _stream(self.device)),
              "kpd_debug_copy")
        return out


def nms(boxes: torch.Tensor, scores: torch.Tensor, iou_threshold: float, max_output: int = 0) -> torch.Tensor:
    """Device NMS with PERSON_HEAD.non_max_suppression semantics; returns int64 keep indices."""
    lib = load()
    _require_cuda(boxes, "boxes")
    boxes = boxes.float().contiguous()
    scores = scores.float().contiguous()
    n = boxes.shape[0]
    keep = torch.empty(max(n, 1), dtype=torch.int32, device=boxes.device)
    nk = torch.zeros(1, dtype=torch.int32, device=boxes.device)
    with torch.cuda.device(boxes.device):
        check(lib.kpd_nms(_ptr(boxes), _ptr(scores), n, float(iou_threshold), int(max_output or 0), _ptr(keep),
                          _ptr(nk), _stream(boxes.device)), "kpd_nms")
    return keep[: int(nk.item())].long()
