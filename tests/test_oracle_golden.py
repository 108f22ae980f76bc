"""The C oracle against the golden fixtures the reference itself produced
(tests/golden/make_golden.py runs oracle/_ref/ref_harness, which compiles the
reference's own headers).  Bit-exact: same float/double expression shapes,
same libm, same counter RNG."""
import os

import numpy as np
import pytest

import scene_io as sio

CASES = [c["name"] for c in sio.manifest()["cases"]]


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_bit_exact(name):
    c = sio.golden_case(name)
    W, H = c["width"], c["height"]
    scene = sio.with_synthetic_texels(sio.load_scene(os.path.join(sio.GOLDEN, name + ".scn")))
    arrays = sio.SceneArrays(scene)
    cam = sio.camera_from_file(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"))
    p = sio.default_params(W, H, c["spp"], seed=c["seed"])
    import ctypes

    lin, bgra, cnt = sio.oracle_render(ctypes.addressof(arrays.view), cam, p)
    glin, gbgra = sio.golden_image(name, W, H)
    assert np.array_equal(lin.reshape(H, W, 3).view(np.uint32), glin.view(np.uint32))
    assert np.array_equal(bgra.reshape(H, W, 4), gbgra)
    assert cnt.samples == W * H * c["spp"]
    assert cnt.segments >= cnt.samples


def test_synthetic_texture_hash():
    import hashlib

    for c in sio.manifest()["cases"]:
        if c["image"] == "synthetic":
            assert hashlib.sha256(sio.synthetic_image(2048, 1024).tobytes()).hexdigest() == c["texel_sha256"]


def test_oracle_pixel_subset_matches_full_frame():
    """Rendering a pixel list gives the same values as the full frame (the
    multi-rank and bounded-sample paths rely on this)."""
    import ctypes

    c = sio.golden_case("cornell_smoke")
    W, H = c["width"], c["height"]
    arrays = sio.SceneArrays(sio.load_scene(os.path.join(sio.GOLDEN, "cornell_smoke.scn")))
    cam = sio.camera_from_file(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"))
    p = sio.default_params(W, H, c["spp"], seed=c["seed"])
    pix = np.array([0, 5, W * H - 1, 17 * W + 3, 1000], np.uint32)
    lin, _, _ = sio.oracle_render(ctypes.addressof(arrays.view), cam, p, pixels=pix, threads=3)
    glin, _ = sio.golden_image("cornell_smoke", W, H)
    assert np.array_equal(lin, glin.reshape(-1, 3)[pix])
