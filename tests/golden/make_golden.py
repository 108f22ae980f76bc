#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE ITSELF.

Runs oracle/_ref/ref_harness (built by `make -C oracle ref` from the
reference's own headers under /root/reference, with the counter RNG injected;
see oracle/ref_harness.cpp).  Only works where /root/reference exists; the
outputs are committed so the GPU box never needs the reference.

For every case it writes
  <case>.scn   the scene graph the reference built (texel bytes stripped; the
               manifest keeps their sha256 -- the texture is the synthetic
               stand-in of rtow_synthetic_image(), fed to the reference's
               stbi_load as a lossless PNG named input_images/1_earth_8k.jpg)
  <case>.lin   averaged linear RGB, float32, framebuffer order
  <case>.bgra  BGRA8 frame, main.cpp:982-989 layout
and cam_<W>x<H>.cam, plus manifest.json.

Usage: python3 tests/golden/make_golden.py
"""
import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")

sys.path.insert(0, os.path.dirname(HERE))
from scene_io import synthetic_image  # noqa: E402

# name, harness scene, n, image mode, W, H, spp, render seed
CASES = [
    ("three_sphere", "three_sphere", 100, "none", 200, 100, 8, 1),
    ("random100_noimg", "random_ned", 100, "none", 64, 36, 64, 1),
    ("random100_synth", "random_ned", 100, "synthetic", 64, 36, 64, 7),
    ("random487_synth", "random_ned", 487, "synthetic", 64, 36, 32, 1),
    ("random487_ragged", "random_ned", 487, "synthetic", 37, 23, 8, 3),
    ("cornell", "cornell", 100, "none", 48, 48, 64, 1),
    ("cornell_smoke", "cornell_smoke", 100, "none", 48, 48, 64, 1),
    ("final_ned", "final_ned", 100, "synthetic", 48, 48, 16, 5),
]
SCENE_SEED = 1


def write_png(path, rgb):
    from PIL import Image
    Image.fromarray(rgb, "RGB").save(path, format="PNG")


def strip_texels(src, dst):
    b = open(src, "rb").read()
    hdr = struct.unpack("<10I", b[8:48])
    (ntex,) = struct.unpack("<Q", b[48:56])
    body = b[: len(b) - ntex]
    texels = b[len(b) - ntex:]
    out = bytearray(body)
    out[48:56] = struct.pack("<Q", 0)
    open(dst, "wb").write(bytes(out))
    return hashlib.sha256(texels).hexdigest(), ntex, hdr


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the harness first: make -C oracle ref")
    tmp = tempfile.mkdtemp(prefix="rtow_golden_")
    dirs = {"none": os.path.join(tmp, "none"), "synthetic": os.path.join(tmp, "synth")}
    os.makedirs(dirs["none"])
    os.makedirs(os.path.join(dirs["synthetic"], "input_images"))
    write_png(os.path.join(dirs["synthetic"], "input_images", "1_earth_8k.jpg"),
              synthetic_image(2048, 1024))
    env = dict(os.environ, RTOW_SCENE_SEED=str(SCENE_SEED))
    manifest = {"scene_seed": SCENE_SEED, "generator": "oracle/_ref/ref_harness", "cases": []}
    cams = set()
    for name, scene, n, img, W, H, spp, seed in CASES:
        raw = os.path.join(tmp, name + ".scn")
        out = subprocess.run([HARNESS, "dump", scene, raw, "--n", str(n), "--cwd", dirs[img]],
                             env=env, check=True, capture_output=True, text=True).stdout
        draws = int(out.split()[1])
        sha, ntex, hdr = strip_texels(raw, os.path.join(HERE, name + ".scn"))
        subprocess.run([HARNESS, "render", scene, str(W), str(H), str(spp), os.path.join(HERE, name),
                        "--n", str(n), "--seed", str(seed), "--cwd", dirs[img]], env=env, check=True)
        if (W, H) not in cams:
            subprocess.run([HARNESS, "camera", str(W), str(H), os.path.join(HERE, f"cam_{W}x{H}.cam")],
                           env=env, check=True)
            cams.add((W, H))
        manifest["cases"].append(dict(name=name, scene=scene, n=n, image=img, width=W, height=H, spp=spp,
                                      seed=seed, scene_draws=draws, texel_bytes=ntex, texel_sha256=sha,
                                      n_hitables=hdr[2]))
        print(f"{name}: {hdr[2]} hitables, {draws} scene draws")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
