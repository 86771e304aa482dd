"""GPU ``ITransform`` -- drop-in for the reference's image transform
(dll/data/transforms.py:9-113) on the MI355X (kpd_preprocess, csrc/preprocess.hip).

Reference pipeline and what runs here:

* RGB (``grayscale=False``, :36-41, :80-108): per-channel CLAHE -> 3x3
  Gaussian (sigma 0.5) -> Resize((s, s)) -> ToTensor -> Normalize(ImageNet).
  All stages run on the device.
* Grayscale (``grayscale=True``, :28-33, :43-78): RGB->gray -> CLAHE -> edge
  blend (GaussianBlur 5x5 -> medianBlur 5 -> Canny(100, 200) -> dilate/erode
  x2 -> GaussianBlur 3x3 -> scale to 255 -> addWeighted(0.7, 0.3)) -> Resize
  -> ToTensor -> Normalize(0.5, 0.5).  All stages run on the device.

Resize/ToTensor/Normalize are bit-exact to Pillow + torchvision
(tests/golden/preprocess.npz).  CLAHE, the blurs, median, Canny, morphology
and addWeighted restate OpenCV's CV_8U algorithms and are bit-exact to the
oracle (oracle/preprocess_oracle.py) -- parity unpinned against OpenCV itself,
which is absent from this image.
"""
import ctypes
from typing import Optional, Sequence, Tuple, Union

import numpy as np
import torch

from .. import _native

FLAG_GRAY, FLAG_CLAHE, FLAG_BLUR, FLAG_EDGES = 1, 2, 4, 8
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def preprocess(image: torch.Tensor, out_size: Tuple[int, int], mean: Sequence[float], std: Sequence[float],
               flags: int = 0, clip_limit: float = 2.0, tiles: Tuple[int, int] = (8, 8),
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 HWC (or HW) image on a GPU -> fp32 [C', out_h, out_w] on the same GPU."""
    if image.dtype != torch.uint8 or not image.is_cuda:
        raise TypeError("preprocess expects a uint8 CUDA tensor [H,W] or [H,W,C]")
    img = image if image.dim() == 3 else image[:, :, None]
    img = img.contiguous()
    H, W, C = img.shape
    c_out = 1 if flags & FLAG_GRAY else C
    if len(mean) != c_out or len(std) != c_out:
        raise ValueError(f"mean/std need {c_out} values")
    oh, ow = out_size
    if out is None:
        out = torch.empty(c_out, oh, ow, device=img.device, dtype=torch.float32)
    lib = _native.load()
    m = (ctypes.c_float * 3)(*mean, *([0.0] * (3 - len(mean))))
    s = (ctypes.c_float * 3)(*std, *([1.0] * (3 - len(std))))
    stream = torch.cuda.current_stream(img.device).cuda_stream
    with torch.cuda.device(img.device):
        rc = lib.kpd_preprocess(ctypes.c_void_p(img.data_ptr()), H, W, C, W * C, flags, ctypes.c_float(clip_limit),
                                tiles[0], tiles[1], oh, ow, m, s, ctypes.c_void_p(out.data_ptr()),
                                ctypes.c_void_p(stream))
    _native.check(rc, "kpd_preprocess")
    return out


class ITransform:
    """Same constructor and call as the reference ITransform; runs on ``device``."""

    def __init__(self, img_size: Union[int, Tuple[int, int]] = 224, clip_limit: float = 1.5,
                 tile_size: Tuple[int, int] = (8, 8), grayscale: bool = True,
                 device: Union[str, torch.device] = "cuda"):
        self.img_size = img_size
        self.size = (img_size, img_size) if isinstance(img_size, int) else tuple(img_size)
        self.clip_limit = clip_limit
        self.tile_size = tile_size
        self.grayscale = grayscale
        self.device = torch.device(device)
        self.transform = self.__call__      # the reference's Compose pipeline attribute (:26-41)

    def __call__(self, img) -> torch.Tensor:
        if isinstance(img, torch.Tensor):
            t = img
        else:   # PIL image or array-like
            a = np.asarray(img.convert("RGB") if hasattr(img, "convert") and getattr(img, "mode", "RGB")
                           not in ("RGB", "L") else img)
            t = torch.from_numpy(np.array(a, dtype=np.uint8, copy=True))
        if t.dtype != torch.uint8:
            raise TypeError("ITransform expects 8-bit images")
        t = t.to(self.device, non_blocking=True)
        if self.grayscale:
            flags = FLAG_CLAHE | FLAG_EDGES | (FLAG_GRAY if t.dim() == 3 and t.shape[2] == 3 else 0)
            return preprocess(t, self.size, (0.5,), (0.5,), flags, self.clip_limit, self.tile_size)
        if t.dim() == 2:
            t = t[:, :, None].expand(-1, -1, 3)
        return preprocess(t, self.size, IMAGENET_MEAN, IMAGENET_STD, FLAG_CLAHE | FLAG_BLUR, self.clip_limit,
                          self.tile_size)
