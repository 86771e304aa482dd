"""CPU oracle for the preprocessing path.

TEST INFRASTRUCTURE ONLY: imported by tests/ and never by the product path.

Reference: `ITransform` (dll/data/transforms.py:9-113) = an OpenCV stage
(`to_rgb_clahe` :80-108 / `to_grayscale_clahe` :43-78) -> torchvision
`Resize((s, s))` on a PIL image -> `ToTensor()` -> `Normalize(mean, std)`.

* `pil_resize_bilinear` restates Pillow's `ImagingResample` for 8-bit images
  (Pillow `src/libImaging/Resample.c`: `precompute_coeffs`,
  `normalize_coeffs_8bpc`, horizontal pass first with the intermediate rounded
  to uint8, PRECISION_BITS = 22).  **Pinned**: checked bit-exact against the
  real Pillow 12.2 in this container (tests/golden/make_preprocess_golden.py
  commits the vectors).
* `to_tensor_normalize` is torchvision's `ToTensor` (uint8 / 255 in fp32) then
  `Normalize` ((x - mean) / std in fp32).  Pinned by the same vectors.
* `clahe_u8` restates OpenCV's `cv::CLAHE` for CV_8U (imgproc/src/clahe.cpp:
  reflect-101 padding to a tile multiple, per-tile 256-bin histogram, clip at
  max(int(clip * area / 256), 1) with batch + strided residual redistribution,
  LUT = saturate_cast<uchar>(cumsum * 255 / area), bilinear blend of the four
  neighbouring tile LUTs).  OpenCV is absent from this image and from the GPU
  box, so this restatement is **parity unpinned** against OpenCV itself.
* `gaussian_blur3_u8` (the RGB pipeline's `GaussianBlur((3, 3), 0.5)`) is a
  float separable restatement, also **parity unpinned** (OpenCV's 8-bit
  fixed-point path may differ by one grey level at rounding ties).
"""
import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _bilinear(x):
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


def pil_coeffs(in_size: int, out_size: int):
    """Pillow precompute_coeffs + normalize_coeffs_8bpc for the bilinear
    filter (support 1): bounds [out][2] (xmin, count) and int32 fixed-point
    weights [out][ksize]."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(np.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_bilinear((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = sum(w)
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(v):
    out = np.where(v >= (1 << PRECISION_BITS << 8), 255, np.where(v <= 0, 0, v >> PRECISION_BITS))
    return out.astype(np.uint8)


def pil_resize_bilinear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """uint8 [H,W] or [H,W,C] -> uint8 [out_h,out_w(,C)] exactly as
    PIL.Image.resize((out_w, out_h), BILINEAR)."""
    a = img if img.ndim == 3 else img[:, :, None]
    H, W, C = a.shape
    if (H, W) == (out_h, out_w):
        return img.copy()
    a = a.astype(np.int64)
    bh, kh = pil_coeffs(W, out_w)
    bv, kv = pil_coeffs(H, out_h)
    need_h, need_v = out_w != W, out_h != H
    if need_h:
        y0 = int(bv[0, 0])
        y1 = int(bv[-1, 0] + bv[-1, 1])
        if not need_v:
            y0, y1 = 0, H
        src = a[y0:y1]
        tmp = np.empty((y1 - y0, out_w, C), np.uint8)
        for xx in range(out_w):
            xmin, n = bh[xx]
            acc = np.full((y1 - y0, C), 1 << (PRECISION_BITS - 1), np.int64)
            for x in range(n):
                acc += src[:, xmin + x, :] * kh[xx, x]
            tmp[:, xx, :] = _clip8(acc)
        a = tmp.astype(np.int64)
        bv = bv.copy()
        bv[:, 0] -= y0
    if need_v:
        out = np.empty((out_h, a.shape[1], C), np.uint8)
        for yy in range(out_h):
            ymin, n = bv[yy]
            acc = np.full((a.shape[1], C), 1 << (PRECISION_BITS - 1), np.int64)
            for y in range(n):
                acc += a[ymin + y] * kv[yy, y]
            out[yy] = _clip8(acc)
        a = out
    a = a.astype(np.uint8)
    return a if img.ndim == 3 else a[:, :, 0]


def to_tensor_normalize(img: np.ndarray, mean, std) -> np.ndarray:
    """torchvision ToTensor + Normalize: uint8 HWC -> fp32 CHW."""
    a = img if img.ndim == 3 else img[:, :, None]
    x = a.astype(np.float32) / np.float32(255)
    x = x.transpose(2, 0, 1)
    m = np.asarray(mean, np.float32).reshape(-1, 1, 1)
    s = np.asarray(std, np.float32).reshape(-1, 1, 1)
    return ((x - m) / s).astype(np.float32)


def rgb_to_gray_cv(img: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(RGB2GRAY) for 8U: (R*4899 + G*9617 + B*1868 + 2^13) >> 14."""
    a = img.astype(np.int64)
    return ((a[..., 0] * 4899 + a[..., 1] * 9617 + a[..., 2] * 1868 + (1 << 13)) >> 14).astype(np.uint8)


def _reflect101(i, n):
    if n == 1:
        return 0
    while i < 0 or i >= n:
        i = -i if i < 0 else 2 * n - 2 - i
    return i


def clahe_u8(img: np.ndarray, clip_limit: float, tiles_x: int, tiles_y: int) -> np.ndarray:
    """OpenCV cv::CLAHE(clipLimit, (tiles_x, tiles_y)).apply on one uint8 plane."""
    H, W = img.shape
    if W % tiles_x == 0 and H % tiles_y == 0:
        ext = img
    else:
        Hp = H + (tiles_y - H % tiles_y if H % tiles_y else 0)
        Wp = W + (tiles_x - W % tiles_x if W % tiles_x else 0)
        ys = np.array([_reflect101(y, H) for y in range(Hp)])
        xs = np.array([_reflect101(x, W) for x in range(Wp)])
        ext = img[ys][:, xs]
    tw, th = ext.shape[1] // tiles_x, ext.shape[0] // tiles_y
    area = tw * th
    lut_scale = np.float32(255.0) / np.float32(area)
    clip = 0
    if clip_limit > 0.0:
        clip = max(int(clip_limit * area / 256), 1)
    luts = np.zeros((tiles_y, tiles_x, 256), np.uint8)
    for ty in range(tiles_y):
        for tx in range(tiles_x):
            tile = ext[ty * th:(ty + 1) * th, tx * tw:(tx + 1) * tw]
            hist = np.bincount(tile.ravel(), minlength=256).astype(np.int64)
            if clip_limit > 0.0:
                clipped = int(np.maximum(hist - clip, 0).sum())
                hist = np.minimum(hist, clip)
                batch = clipped // 256
                residual = clipped - batch * 256
                hist += batch
                if residual:
                    step = max(256 // residual, 1)
                    i = 0
                    while i < 256 and residual > 0:
                        hist[i] += 1
                        i += step
                        residual -= 1
            csum = np.cumsum(hist).astype(np.float32) * lut_scale
            luts[ty, tx] = np.clip(np.rint(csum), 0, 255).astype(np.uint8)   # saturate_cast: round half even
    out = np.empty_like(img)
    inv_tw, inv_th = np.float32(1.0) / np.float32(tw), np.float32(1.0) / np.float32(th)
    for y in range(H):
        tyf = np.float32(y) * inv_th - np.float32(0.5)
        ty1 = int(np.floor(tyf))
        ya = np.float32(tyf - np.float32(ty1))
        ya1 = np.float32(1.0) - ya
        ty2 = min(ty1 + 1, tiles_y - 1)
        ty1 = max(ty1, 0)
        for x in range(W):
            txf = np.float32(x) * inv_tw - np.float32(0.5)
            tx1 = int(np.floor(txf))
            xa = np.float32(txf - np.float32(tx1))
            xa1 = np.float32(1.0) - xa
            tx2 = min(tx1 + 1, tiles_x - 1)
            tx1 = max(tx1, 0)
            v = img[y, x]
            l11, l12 = np.float32(luts[ty1, tx1, v]), np.float32(luts[ty1, tx2, v])
            l21, l22 = np.float32(luts[ty2, tx1, v]), np.float32(luts[ty2, tx2, v])
            r = (l11 * xa1 + l12 * xa) * ya1 + (l21 * xa1 + l22 * xa) * ya
            out[y, x] = np.uint8(min(max(int(np.rint(r)), 0), 255))
    return out


def gaussian_kernel(ksize: int, sigma: float) -> np.ndarray:
    """cv::getGaussianKernel (sigma > 0): exp(-(i - c)^2 / (2 sigma^2)), normalised."""
    c = (ksize - 1) / 2.0
    k = [float(np.exp(-((i - c) ** 2) / (2.0 * sigma * sigma))) for i in range(ksize)]
    s = 0.0
    for v in k:          # accumulated in index order, as getGaussianKernel does
        s += v
    return np.array([v / s for v in k])


def gaussian_blur3_u8(img: np.ndarray, sigma: float) -> np.ndarray:
    """Separable 3x3 Gaussian on uint8 planes, reflect-101 border, fp32 with
    round-half-even to uint8 (parity unpinned vs OpenCV's fixed-point path)."""
    k = gaussian_kernel(3, sigma).astype(np.float32)
    a = img if img.ndim == 3 else img[:, :, None]
    H, W, C = a.shape
    ys = [np.array([_reflect101(y + d, H) for y in range(H)]) for d in (-1, 0, 1)]
    xs = [np.array([_reflect101(x + d, W) for x in range(W)]) for d in (-1, 0, 1)]
    f = a.astype(np.float32)
    h = k[0] * f[:, xs[0]] + k[1] * f[:, xs[1]] + k[2] * f[:, xs[2]]
    v = k[0] * h[ys[0]] + k[1] * h[ys[1]] + k[2] * h[ys[2]]
    out = np.clip(np.rint(v), 0, 255).astype(np.uint8)
    return out if img.ndim == 3 else out[:, :, 0]


def itransform_rgb(img: np.ndarray, size: int, clip_limit: float = 2.0, tiles=(8, 8)) -> np.ndarray:
    """ITransform(grayscale=False) (transforms.py:36-41,80-108) -> fp32 [3,s,s]."""
    planes = [clahe_u8(np.ascontiguousarray(img[..., c]), clip_limit, tiles[0], tiles[1]) for c in range(3)]
    x = gaussian_blur3_u8(np.stack(planes, -1), 0.5)
    x = pil_resize_bilinear(x, size, size)
    return to_tensor_normalize(x, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
