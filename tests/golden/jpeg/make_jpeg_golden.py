#!/usr/bin/env python3
"""JPEG fixtures for rtow_image_decode_jpeg (tests/test_jpeg.py).

Encodes small synthetic images with PIL (libjpeg) in the variants the
decoder has to cover -- 4:2:0 / 4:2:2 / 4:4:4 sampling, grayscale, CMYK,
progressive, restart markers, odd sizes, quality 100 -- and decodes each with
the REFERENCE's own stb_image (oracle/_ref/ref_harness `decode`: stbi_load(
path, .., 0) as scenes.h:140 calls it).  Writes <case>.jpg and <case>.img
(uint32 nx, ny, channels, then the pixels) plus manifest.json.

Usage: python3 tests/golden/jpeg/make_jpeg_golden.py   (after make -C oracle ref)
"""
import hashlib
import io
import json
import os
import subprocess
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")


def picture(w, h, seed):
    """smooth gradients + edges + noise: every coefficient range gets used"""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    r = 127 + 120 * np.sin(x / 7.0 + seed) * np.cos(y / 11.0)
    g = (x * 255 / max(w - 1, 1) + (y // 8 % 2) * 60) % 256
    b = 255 * ((x // 5 + y // 3) % 2) * 0.8 + rng.integers(0, 40, (h, w))
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


# name, size, PIL mode, save options
CASES = [
    ("yuv420_q75", (64, 48), "RGB", dict(quality=75, subsampling=2)),
    ("yuv422_q90", (48, 40), "RGB", dict(quality=90, subsampling=1)),
    ("yuv444_q100", (40, 32), "RGB", dict(quality=100, subsampling=0)),
    ("odd_37x23_420", (37, 23), "RGB", dict(quality=80, subsampling=2)),
    ("odd_1x9_420", (1, 9), "RGB", dict(quality=80, subsampling=2)),
    ("gray_q85", (45, 30), "L", dict(quality=85)),
    ("progressive_420", (64, 40), "RGB", dict(quality=85, subsampling=2, progressive=True)),
    ("progressive_444_gray", (33, 17), "L", dict(quality=95, progressive=True)),
    ("restart_420", (80, 48), "RGB", dict(quality=80, subsampling=2, restart_marker_blocks=3)),
    ("restart_rows_444", (40, 40), "RGB", dict(quality=70, subsampling=0, restart_marker_rows=1)),
    ("cmyk_q90", (32, 24), "CMYK", dict(quality=90)),
    ("q10_420", (64, 64), "RGB", dict(quality=10, subsampling=2)),
]


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the harness first: make -C oracle ref")
    manifest = {"generator": "PIL encode, oracle/_ref/ref_harness decode (the reference's stb_image.h)",
                "cases": []}
    for k, (name, (w, h), mode, opts) in enumerate(CASES):
        img = Image.fromarray(picture(w, h, k), "RGB").convert(mode)
        buf = io.BytesIO()
        img.save(buf, format="JPEG", **opts)
        jpg = os.path.join(HERE, name + ".jpg")
        with open(jpg, "wb") as f:
            f.write(buf.getvalue())
        out = os.path.join(HERE, name + ".img")
        subprocess.run([HARNESS, "decode", jpg, out], check=True)
        raw = open(out, "rb").read()
        nx, ny, n = np.frombuffer(raw[:12], np.uint32)
        manifest["cases"].append(dict(name=name, mode=mode, options={a: str(b) for a, b in opts.items()},
                                      width=int(nx), height=int(ny), channels=int(n),
                                      sha256=hashlib.sha256(raw[12:]).hexdigest()))
        print(f"{name}: {nx}x{ny}x{n}, {len(buf.getvalue())} B")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
