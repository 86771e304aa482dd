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
* `gaussian_blur_u8` restates cv::GaussianBlur's CV_8U fixed-point path
  (getGaussianKernelBitExact -> 8-bit error-diffused kernel, exact integer
  row/column sums, round half up); `median5_u8`, `canny_u8` (L1, aperture 3),
  `morph3_u8` and `add_weighted_u8` restate medianBlur / Canny / dilate /
  erode / addWeighted for the grayscale pipeline's edge blend
  (`edge_blend_u8`, transforms.py:55-73).  All **parity unpinned** against
  OpenCV (absent); median, morphology and Canny are integer algorithms whose
  only freedom is the documented border and tie rules.
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


def gaussian_kernel_bitexact(ksize: int, sigma: float) -> np.ndarray:
    """cv::getGaussianKernelBitExact (imgproc/src/smooth.dispatch.cpp): the
    fixed table for sigma <= 0 and ksize <= 7, else exp(x^2 * (-0.125 / s^2))
    over doubled coordinates x = 2i - (n - 1), normalised by 1 / sum with the
    centre tap exactly 1 * mul1."""
    n = ksize
    if sigma <= 0 and n in (1, 3, 5, 7):
        return np.array({1: [1.0], 3: [0.25, 0.5, 0.25], 5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
                         7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125]}[n])
    sig = sigma if sigma > 0 else n * 0.15 + 0.35
    scale2x = -0.125 / (sig * sig)
    n2 = (n - 1) // 2
    values, s = [], 0.0
    for i in range(n2):
        x = 2 * i + 1 - n
        t = float(np.exp(float(x * x) * scale2x))
        values.append(t)
        s += t
    s = s * 2.0 + 1.0
    mul1 = 1.0 / s
    r = np.zeros(n)
    for i in range(n2):
        r[i] = r[n - 1 - i] = values[i] * mul1
    r[n2] = mul1
    return r


def gaussian_kernel_fixed(ksize: int, sigma: float) -> np.ndarray:
    """getGaussianKernelFixedPoint_ED with 8 fraction bits (ufixedpoint16, the
    type cv::GaussianBlur uses for CV_8U): error-diffused cvRound of the outer
    taps, centre = 256 - sum of the others."""
    k = gaussian_kernel_bitexact(ksize, sigma)
    n2 = ksize // 2
    out = np.zeros(ksize, np.int64)
    err, s = 0.0, 0
    for i in range(n2):
        adj = k[i] * 256.0 + err
        v0 = int(np.rint(adj))            # cvRound: half to even
        err = adj - v0
        out[i] = out[ksize - 1 - i] = v0
        s += v0
    out[n2] = 256 - 2 * s
    return out


def gaussian_blur_u8(img: np.ndarray, ksize: int, sigma: float) -> np.ndarray:
    """cv::GaussianBlur on CV_8U via the fixed-point path (GaussianBlurFixedPoint):
    reflect-101 border; the row pass is the exact integer sum of kernel(8-bit
    fraction) x pixel, the column pass the exact sum of kernel x row value
    (16-bit fraction), rounded half up to uint8."""
    k = gaussian_kernel_fixed(ksize, sigma)
    a = img if img.ndim == 3 else img[:, :, None]
    H, W, C = a.shape
    r = ksize // 2
    ys = [np.array([_reflect101(y + d, H) for y in range(H)]) for d in range(-r, r + 1)]
    xs = [np.array([_reflect101(x + d, W) for x in range(W)]) for d in range(-r, r + 1)]
    f = a.astype(np.int64)
    h = sum(k[i] * f[:, xs[i]] for i in range(ksize))
    v = sum(k[i] * h[ys[i]] for i in range(ksize))
    out = np.minimum((v + (1 << 15)) >> 16, 255).astype(np.uint8)
    return out if img.ndim == 3 else out[:, :, 0]


def median5_u8(img: np.ndarray) -> np.ndarray:
    """cv::medianBlur(img, 5) for CV_8U (the sorting-network path, replicated border)."""
    p = np.pad(img, 2, mode="edge")
    win = np.lib.stride_tricks.sliding_window_view(p, (5, 5)).reshape(img.shape[0], img.shape[1], 25)
    return np.sort(win, axis=-1)[..., 12].astype(np.uint8)


CANNY_TG22 = int(0.4142135623730950488016887242097 * (1 << 15) + 0.5)


def canny_u8(img: np.ndarray, low: float, high: float) -> np.ndarray:
    """cv::Canny(img, low, high) with apertureSize 3 and the L1 gradient
    (imgproc/src/canny.cpp): 3x3 Sobel (replicated border) in int, magnitude
    |dx| + |dy| (zero outside the image), non-maximum suppression by the
    tan(22.5)/tan(67.5) fixed-point sector test (strict '>' toward the
    previous neighbour, '>=' toward the next; both strict on diagonals),
    candidates m > floor(low), seeds m > floor(high), 8-connected hysteresis.
    Returns 0/255."""
    lo, hi = int(np.floor(low)), int(np.floor(high))
    p = np.pad(img.astype(np.int64), 1, mode="edge")
    dx = (p[:-2, 2:] + 2 * p[1:-1, 2:] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[1:-1, :-2] + p[2:, :-2])
    dy = (p[2:, :-2] + 2 * p[2:, 1:-1] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[:-2, 1:-1] + p[:-2, 2:])
    mag = np.abs(dx) + np.abs(dy)
    M = np.pad(mag, 1)
    ax, ay = np.abs(dx), np.abs(dy) << 15
    tg22x = ax * CANNY_TG22
    tg67x = tg22x + (ax << 16)
    horiz = ay < tg22x
    vert = ~horiz & (ay > tg67x)
    diag = ~horiz & ~vert
    neg = (dx ^ dy) < 0
    c = M[1:-1, 1:-1]
    keep_h = (c > M[1:-1, :-2]) & (c >= M[1:-1, 2:])
    keep_v = (c > M[:-2, 1:-1]) & (c >= M[2:, 1:-1])
    keep_d = np.where(neg, (c > M[:-2, 2:]) & (c > M[2:, :-2]),      # s = -1: (y-1, x+1) and (y+1, x-1)
                      (c > M[:-2, :-2]) & (c > M[2:, 2:]))            # s = +1: (y-1, x-1) and (y+1, x+1)
    nms = (horiz & keep_h) | (vert & keep_v) | (diag & keep_d)
    cand = (mag > lo) & nms
    strong = cand & (mag > hi)
    from scipy import ndimage
    lab, nlab = ndimage.label(cand, structure=np.ones((3, 3), int))
    seeded = np.zeros(nlab + 1, bool)
    seeded[np.unique(lab[strong])] = True
    seeded[0] = False
    return np.where(seeded[lab], 255, 0).astype(np.uint8)


def morph3_u8(img: np.ndarray, dilate: bool) -> np.ndarray:
    """cv::dilate / cv::erode with np.ones((3, 3)), one iteration, default
    border (the out-of-image value never wins)."""
    p = np.pad(img, 1, constant_values=0 if dilate else 255)
    win = np.lib.stride_tricks.sliding_window_view(p, (3, 3))
    return (win.max(axis=(-1, -2)) if dilate else win.min(axis=(-1, -2))).astype(np.uint8)


def add_weighted_u8(a: np.ndarray, alpha: float, b: np.ndarray, beta: float) -> np.ndarray:
    """cv::addWeighted for CV_8U, gamma 0: fp32 fma(a, alpha, fma(b, beta, 0))
    (the SIMD path), cvRound half to even, saturate.  Evaluated in double,
    where both products and the sum are exact, then rounded once to fp32 --
    the same value the fused multiply-adds give."""
    al, be = float(np.float32(alpha)), float(np.float32(beta))
    inner = (b.astype(np.float64) * be).astype(np.float32).astype(np.float64)
    t = (a.astype(np.float64) * al + inner).astype(np.float32)
    return np.clip(np.rint(t), 0, 255).astype(np.uint8)


def edge_blend_u8(clahe_img: np.ndarray) -> np.ndarray:
    """The edge half of to_grayscale_clahe (transforms.py:55-73):
    GaussianBlur 5x5 s1.5 -> medianBlur 5 -> Canny(100, 200) -> (dilate,
    erode) x 2 with a 3x3 ones kernel -> GaussianBlur 3x3 s0 -> scale to max
    255 (float64, truncating astype) -> addWeighted(clahe 0.7, edges 0.3)."""
    d = median5_u8(gaussian_blur_u8(clahe_img, 5, 1.5))
    e = canny_u8(d, 100, 200)
    e = morph3_u8(morph3_u8(morph3_u8(morph3_u8(e, True), False), True), False)
    e = gaussian_blur_u8(e, 3, 0)
    mx = int(e.max())
    if mx > 0:
        e = (e.astype(np.float64) / mx * 255).astype(np.uint8)
    return add_weighted_u8(clahe_img, 0.7, e, 0.3)


def itransform_gray(img: np.ndarray, size, clip_limit: float = 1.5, tiles=(8, 8)) -> np.ndarray:
    """ITransform(grayscale=True) (transforms.py:28-33,43-78) -> fp32 [1,h,w]."""
    oh, ow = (size, size) if isinstance(size, int) else size
    gray = img if img.ndim == 2 else rgb_to_gray_cv(img)
    x = edge_blend_u8(clahe_u8(np.ascontiguousarray(gray), clip_limit, tiles[0], tiles[1]))
    x = pil_resize_bilinear(x, oh, ow)
    return to_tensor_normalize(x, [0.5], [0.5])


def itransform_rgb(img: np.ndarray, size: int, clip_limit: float = 2.0, tiles=(8, 8)) -> np.ndarray:
    """ITransform(grayscale=False) (transforms.py:36-41,80-108) -> fp32 [3,s,s]."""
    planes = [clahe_u8(np.ascontiguousarray(img[..., c]), clip_limit, tiles[0], tiles[1]) for c in range(3)]
    x = gaussian_blur_u8(np.stack(planes, -1), 3, 0.5)
    x = pil_resize_bilinear(x, size, size)
    return to_tensor_normalize(x, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
