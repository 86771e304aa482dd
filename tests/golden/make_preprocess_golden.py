#!/usr/bin/env python3
"""Golden vectors for the preprocessing path.

Runs the REAL Pillow (12.2, importable in the build container) on seeded
uint8 images: PIL.Image.resize(BILINEAR) -- what torchvision Resize does to a
PIL image in ITransform (dll/data/transforms.py:28-41) -- then ToTensor +
Normalize as torchvision defines them.  Writes tests/golden/preprocess.npz.
OpenCV (CLAHE / blur) is absent here, so those stages have no golden.
"""
from pathlib import Path

import numpy as np
from PIL import Image

OUT = Path(__file__).resolve().parent / "preprocess.npz"
CASES = [  # (H, W, C, out_h, out_w)
    (180, 240, 3, 128, 96),     # downscale both axes (antialiased support > 1)
    (100, 76, 3, 160, 160),     # upscale
    (97, 131, 1, 64, 48),       # odd sizes, grayscale
    (256, 192, 3, 256, 192),    # identity size (PIL returns a copy)
    (300, 100, 3, 300, 200),    # horizontal only
    (123, 77, 1, 37, 77),       # vertical only
]


def main():
    rng = np.random.default_rng(2024)
    data = {}
    for i, (h, w, c, oh, ow) in enumerate(CASES):
        img = rng.integers(0, 256, size=(h, w, c) if c > 1 else (h, w), dtype=np.uint8)
        # smooth structure + noise so rounding paths are exercised
        yy, xx = np.mgrid[0:h, 0:w]
        grad = ((yy * 3 + xx * 5) % 256).astype(np.uint8)
        img = (img // 2 + (grad[..., None] // 2 if c > 1 else grad // 2)).astype(np.uint8)
        pil = Image.fromarray(img, mode="RGB" if c == 3 else "L")
        out = np.asarray(pil.resize((ow, oh), Image.BILINEAR))
        data[f"img{i}"] = img
        data[f"resized{i}"] = out
        x = out.astype(np.float32)[..., None] if out.ndim == 2 else out.astype(np.float32)
        x = (x / np.float32(255)).transpose(2, 0, 1)
        if c == 3:
            m = np.array([0.485, 0.456, 0.406], np.float32).reshape(3, 1, 1)
            s = np.array([0.229, 0.224, 0.225], np.float32).reshape(3, 1, 1)
        else:
            m = np.array([0.5], np.float32).reshape(1, 1, 1)
            s = np.array([0.5], np.float32).reshape(1, 1, 1)
        if i < 3:   # ToTensor + Normalize reference values (fp32) for a few cases
            data[f"norm{i}"] = ((x - m) / s).astype(np.float32)
        data[f"shape{i}"] = np.array([h, w, c, oh, ow], np.int32)
    data["n"] = np.array(len(CASES), np.int32)
    np.savez_compressed(OUT, **data)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
