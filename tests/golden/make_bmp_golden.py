#!/usr/bin/env python3
"""Golden BMP files written by the REFERENCE's own writer.

oracle/_ref/ref_bmp (built by `make -C oracle ref` from winDIBbitmap.cpp under
/root/reference) writes test.bmp for each input buffer; the inputs (.raw) and
its outputs (.bmp) are committed under tests/golden/bmp/ so that
rtow_write_bmp is pinned byte for byte without the reference.

Cases: the golden random100_noimg frame as main.cpp:774 hands it over (BGRA,
32 bpp), plus small seeded buffers at 24 and 8 bpp whose rows need padding.

Usage: python3 tests/golden/make_bmp_golden.py
"""
import json
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "bmp")
REF_BMP = os.path.join(HERE, "..", "..", "oracle", "_ref", "ref_bmp")


def cases():
    frame = np.fromfile(os.path.join(HERE, "random100_noimg.bgra"), dtype=np.uint8)
    rng = np.random.default_rng(7)
    return [
        ("frame64x36_32bpp", frame, 64, 36, 32),
        ("ragged13x7_24bpp", rng.integers(0, 256, 13 * 7 * 3, dtype=np.uint8), 13, 7, 24),
        ("ragged5x3_8bpp", rng.integers(0, 256, 5 * 3, dtype=np.uint8), 5, 3, 8),
    ]


def main():
    os.makedirs(OUT, exist_ok=True)
    manifest = []
    for name, buf, w, h, bpp in cases():
        raw = os.path.join(OUT, name + ".raw")
        buf.tofile(raw)
        with tempfile.TemporaryDirectory() as d:
            subprocess.run([REF_BMP, d, raw, str(w), str(h), str(bpp)], check=True)
            with open(os.path.join(d, "test.bmp"), "rb") as f:
                bmp = f.read()
        with open(os.path.join(OUT, name + ".bmp"), "wb") as f:
            f.write(bmp)
        manifest.append({"name": name, "width": w, "height": h, "bpp": bpp, "bytes": len(bmp)})
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest))


if __name__ == "__main__":
    main()
