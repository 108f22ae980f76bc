"""The depth-of-field camera path (RTOW_FLAG_CAMERA_DOF = CAMERA_DOF_EN 1,
camera.h:124-126: offset = _lensRadius * randomInUnitDisk() +
randomInUnitSphere(), mathUtilities.h:11-25), off in the reference's own build
(defines.h:26) and so in every other fixture.

Fixtures: tests/golden/make_extra_golden.py, rendered by oracle/_ref/
ref_harness_dof -- the reference's headers compiled with CAMERA_DOF_EN 1 --
so the draw order (the sphere point first: g++ evaluates operator+'s
arguments right to left) is the reference build's, not a guess.
CPU: the oracle bit-exact against them.  GPU: the HIP path within the
north-star RMS bar, and its segment count equal to the oracle's."""
import ctypes
import json
import os

import numpy as np
import pytest

import rtow
import scene_io as sio

MANIFEST = json.load(open(os.path.join(sio.GOLDEN, "manifest_extra.json")))
CASES = {c["name"]: c for c in MANIFEST["cases"] if c["flags"] & rtow.FLAG_CAMERA_DOF}


def _setup(name):
    c = CASES[name]
    W, H = c["width"], c["height"]
    scene = sio.load_scene(os.path.join(sio.GOLDEN, name + ".scn"))
    if c["image"] == "synthetic":
        scene = sio.with_synthetic_texels(scene)
    cam = sio.camera_from_file(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"))
    p = sio.default_params(W, H, c["spp"], seed=c["seed"])
    p.flags |= rtow.FLAG_CAMERA_DOF
    return c, sio.SceneArrays(scene), cam, p


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_dof_matches_reference_bit_exact(name):
    c, arrays, cam, p = _setup(name)
    W, H = c["width"], c["height"]
    lin, bgra, cnt = sio.oracle_render(ctypes.addressof(arrays.view), cam, p)
    glin, gbgra = sio.golden_image(name, W, H)
    assert np.array_equal(lin.reshape(H, W, 3).view(np.uint32), glin.view(np.uint32))
    assert np.array_equal(bgra.reshape(H, W, 4), gbgra)


def test_dof_changes_the_frame():
    """The flag is not a no-op: the same case without it differs."""
    c, arrays, cam, p = _setup("dof_three_sphere")
    p.flags &= ~rtow.FLAG_CAMERA_DOF
    lin, _, _ = sio.oracle_render(ctypes.addressof(arrays.view), cam, p)
    glin, _ = sio.golden_image("dof_three_sphere", c["width"], c["height"])
    assert not np.array_equal(lin.reshape(glin.shape), glin)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_dof_matches_reference(name, gpu_ctx):
    c, arrays, ocam, op = _setup(name)
    W, H = c["width"], c["height"]
    scene = rtow.Scene.build(c["scene"], n=c["n"], image=c["image"], scene_seed=MANIFEST["scene_seed"])
    gpu_ctx.upload(scene)
    p = rtow.params(W, H, c["spp"], seed=c["seed"])
    p.flags |= rtow.FLAG_CAMERA_DOF
    bgra, lin, st = gpu_ctx.render(rtow.camera_main(W, H), p)
    glin, gbgra = sio.golden_image(name, W, H)
    a = np.asarray(lin, np.float64).reshape(-1, 3)
    rms = np.sqrt(np.mean((a - glin.reshape(-1, 3)) ** 2, axis=0))
    print(f"DOF {name}: rms {rms} exact {float(np.mean(lin.reshape(glin.shape) == glin)):.4f}")
    assert (rms <= 1e-4).all(), rms
    assert np.mean(bgra != gbgra) < 0.01
    _, _, cnt = sio.oracle_render(ctypes.addressof(arrays.view), ocam, op)
    assert st.segments == cnt.segments
