"""Preprocessing path: the oracle against real-Pillow
golden vectors (CPU), and the HIP kernels (kpd_preprocess) against the golden
vectors and the oracle (GPU).

Tolerances: resize + ToTensor + Normalize bit-exact (uint8 fixed point and the
same fp32 ops as torchvision); CLAHE, gray conversion, blurs and the grayscale
edge blend (median, Canny, morphology, addWeighted) bit-exact vs the oracle
restatement (parity unpinned vs OpenCV, which is absent).
"""
import numpy as np
import pytest
import torch

from oracle import preprocess_oracle as O


def _golden(golden_dir):
    return np.load(golden_dir / "preprocess.npz", allow_pickle=False)


def test_oracle_resize_matches_pillow(golden_dir):
    g = _golden(golden_dir)
    for i in range(int(g["n"])):
        h, w, c, oh, ow = (int(v) for v in g[f"shape{i}"])
        r = O.pil_resize_bilinear(g[f"img{i}"], oh, ow)
        assert np.array_equal(r, g[f"resized{i}"]), i
        if f"norm{i}" in g:
            mean, std = ([0.485, 0.456, 0.406], [0.229, 0.224, 0.225]) if c == 3 else ([0.5], [0.5])
            assert np.array_equal(O.to_tensor_normalize(r, mean, std), g[f"norm{i}"]), i


def test_oracle_clahe_properties():
    rng = np.random.default_rng(7)
    flat = np.full((64, 48), 77, np.uint8)
    out = O.clahe_u8(flat, 2.0, 8, 8)
    assert (out == out[0, 0]).all()                       # a constant image stays constant
    img = rng.integers(0, 256, (50, 70), dtype=np.uint8)  # ragged: reflect-101 padding path
    a = O.clahe_u8(img, 2.0, 8, 8)
    b = O.clahe_u8(img, 2.0, 8, 8)
    assert np.array_equal(a, b) and a.shape == img.shape
    # monotone per tile centre: within one tile LUT, larger input never maps lower
    ramp = np.tile(np.arange(256, dtype=np.uint8), (16, 1))
    r = O.clahe_u8(ramp, 40.0, 1, 1)
    assert (np.diff(r[8].astype(int)) >= 0).all()


def test_oracle_opencv_restatements_kat():
    # fixed-point Gaussian taps (8 fraction bits, sum 256)
    assert O.gaussian_kernel_fixed(3, 0.5).tolist() == [27, 202, 27]
    assert O.gaussian_kernel_fixed(5, 1.5).tolist() == [31, 60, 74, 60, 31]
    assert O.gaussian_kernel_fixed(3, 0).tolist() == [64, 128, 64]
    assert O.CANNY_TG22 == 13573
    # a constant image is a fixed point of the blur and the median
    flat = np.full((9, 11), 93, np.uint8)
    assert (O.gaussian_blur_u8(flat, 5, 1.5) == 93).all() and (O.median5_u8(flat) == 93).all()
    # median removes isolated salt, keeps a 3-pixel-wide bar
    img = np.zeros((12, 12), np.uint8)
    img[3, 3] = 255
    img[:, 6:9] = 200
    m = O.median5_u8(img)
    assert m[3, 3] == 0 and (m[:, 6:9] == 200).all() and (m[:, :5] == 0).all()
    # morphology: dilate grows a point to 3x3, erode shrinks it back
    pt = np.zeros((7, 7), np.uint8)
    pt[3, 3] = 255
    d = O.morph3_u8(pt, True)
    assert d.sum() == 9 * 255 and np.array_equal(O.morph3_u8(d, False), pt)
    # Canny: a vertical step gives a one-pixel line; hysteresis keeps a weak
    # segment only when it touches a strong one
    step = np.zeros((20, 20), np.uint8)
    step[:, 10:] = 200
    e = O.canny_u8(step, 100, 200)
    assert set(np.unique(e)) == {0, 255} and (e[:, 9] == 255).all() and e.sum() == 20 * 255
    weak = np.zeros((20, 20), np.uint8)
    weak[:, 10:] = 30                                  # |grad| = 120: candidate, never a seed
    assert O.canny_u8(weak, 100, 200).sum() == 0
    mix = weak.copy()
    mix[:8, 10:] = 200                                 # strong upper half seeds the weak lower half
    e = O.canny_u8(mix, 100, 200)
    assert e[15, 9] == 255 or e[15, 10] == 255
    # addWeighted rounding: 0.7 * 255 + 0.3 * 255 == 255
    assert O.add_weighted_u8(np.array([255, 0, 10], np.uint8), 0.7, np.array([255, 0, 0], np.uint8), 0.3).tolist() \
        == [255, 0, 7]


def _edge_image(rng, h, w, c=3):
    yy, xx = np.mgrid[0:h, 0:w]
    base = rng.integers(0, 50, (h, w, c) if c > 1 else (h, w))
    shape = ((xx > w * 0.45) * 120 + (((yy - h / 2) ** 2 + (xx - w / 3) ** 2) < (min(h, w) / 4) ** 2) * 70
             + ((yy // 9) % 2) * (xx > w * 0.7) * 40)
    return ((base + (shape[..., None] if c > 1 else shape)) % 256).astype(np.uint8)


def test_oracle_itransform_gray_shape():
    img = _edge_image(np.random.default_rng(3), 60, 80)
    out = O.itransform_gray(img, 32, 1.5)
    assert out.shape == (1, 32, 32) and out.dtype == np.float32
    assert out.min() >= -1.0 and out.max() <= 1.0


def test_itransform_api_importable():
    from dll.data import ITransform
    t = ITransform(img_size=64, clip_limit=2.0, tile_size=(8, 8), grayscale=False, device="cpu")
    assert t.size == (64, 64) and t.grayscale is False


gpu = pytest.mark.gpu
DEV = torch.device("cuda:0")


@gpu
def test_gpu_resize_normalize_vs_pillow(golden_dir):
    from dll.data.transforms import preprocess
    g = _golden(golden_dir)
    for i in range(int(g["n"])):
        h, w, c, oh, ow = (int(v) for v in g[f"shape{i}"])
        img = torch.from_numpy(g[f"img{i}"]).to(DEV)
        mean, std = ([0.485, 0.456, 0.406], [0.229, 0.224, 0.225]) if c == 3 else ([0.5], [0.5])
        out = preprocess(img, (oh, ow), mean, std).cpu().numpy()
        want = O.to_tensor_normalize(g[f"resized{i}"], mean, std)
        assert np.array_equal(out, want), i
        if f"norm{i}" in g:
            assert np.array_equal(out, g[f"norm{i}"]), i


@gpu
def test_gpu_clahe_gray_blur_vs_oracle():
    from dll.data.transforms import FLAG_BLUR, FLAG_CLAHE, FLAG_GRAY, preprocess
    rng = np.random.default_rng(11)
    for (h, w) in ((96, 128), (101, 77)):                 # tile multiple and ragged (reflect-101)
        yy, xx = np.mgrid[0:h, 0:w]
        img = ((rng.integers(0, 80, (h, w, 3)) + ((yy * 2 + xx)[..., None] % 176)) % 256).astype(np.uint8)
        t = torch.from_numpy(img).to(DEV)
        # gray + CLAHE, no resize
        got = preprocess(t, (h, w), [0.0], [1.0 / 255.0], FLAG_GRAY | FLAG_CLAHE, 2.0, (8, 8)).cpu().numpy()[0]
        want = O.clahe_u8(O.rgb_to_gray_cv(img), 2.0, 8, 8).astype(np.float32)
        assert np.array_equal(np.rint(got).astype(np.int64), want.astype(np.int64))
        # RGB ITransform pipeline: CLAHE per channel + blur + resize + normalise
        got = preprocess(t, (64, 64), [0.485, 0.456, 0.406], [0.229, 0.224, 0.225], FLAG_CLAHE | FLAG_BLUR, 2.0,
                         (8, 8)).cpu().numpy()
        want = O.itransform_rgb(img, 64, 2.0, (8, 8))
        assert np.array_equal(got, want)


@gpu
def test_gpu_itransform_dropin_matches_oracle():
    from PIL import Image
    from dll.data import ITransform
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (120, 90, 3), dtype=np.uint8)
    t = ITransform(img_size=96, clip_limit=2.0, tile_size=(8, 8), grayscale=False, device=DEV)
    out = t(Image.fromarray(img)).cpu().numpy()
    assert out.shape == (3, 96, 96)
    assert np.array_equal(out, O.itransform_rgb(img, 96, 2.0, (8, 8)))


@gpu
def test_gpu_edge_blend_vs_oracle():
    from dll.data.transforms import FLAG_CLAHE, FLAG_EDGES, FLAG_GRAY, preprocess
    rng = np.random.default_rng(13)
    for (h, w) in ((120, 160), (97, 83)):
        img = _edge_image(rng, h, w)
        t = torch.from_numpy(img).to(DEV)
        got = preprocess(t, (h, w), [0.0], [1.0 / 255.0], FLAG_GRAY | FLAG_CLAHE | FLAG_EDGES, 1.5,
                         (8, 8)).cpu().numpy()[0]
        want = O.edge_blend_u8(O.clahe_u8(O.rgb_to_gray_cv(img), 1.5, 8, 8))
        assert np.array_equal(np.rint(got).astype(np.int64), want.astype(np.int64))
    # single-plane input, no CLAHE, no edges found (flat image): blend of the image with zeros
    flat = torch.full((40, 50), 90, dtype=torch.uint8, device=DEV)
    got = preprocess(flat, (40, 50), [0.0], [1.0 / 255.0], FLAG_EDGES).cpu().numpy()[0]
    assert (np.rint(got) == 63).all()                     # round(0.7 * 90) = 63


@gpu
def test_gpu_itransform_gray_dropin_matches_oracle():
    from PIL import Image
    from dll.data import ITransform
    img = _edge_image(np.random.default_rng(17), 150, 110)
    t = ITransform(img_size=96, clip_limit=1.5, tile_size=(8, 8), grayscale=True, device=DEV)
    out = t(Image.fromarray(img)).cpu().numpy()
    assert out.shape == (1, 96, 96)
    assert np.array_equal(out, O.itransform_gray(img, 96, 1.5, (8, 8)))
