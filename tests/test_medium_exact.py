"""Media the reference composes freely, from the reference's own classes
(tests/golden/make_extra_golden.py; ref_harness.cpp mediumNestedNed and
mediumBvhWrappedNed):

* medium_nested: a ConstantMedium whose boundary is another ConstantMedium,
  and one whose boundary is a HitableList holding a medium
  (constantMedium.h:26-31: `_boundary` is any Hitable, and asking it draws);
* medium_bvh_wrapped: media below a BvhNode behind a Translate, inside a list
  (handed the list's closest hit so far, hitableList.h:24-34) and behind
  RotateY(Translate(...)).

CPU: the oracle reproduces the reference's frames bit for bit.  GPU: the HIP
path (the exact-order kernel, MODE 6) within the north-star bar, with the
segment count equal to the oracle's."""
import ctypes
import json
import os

import numpy as np
import pytest

import rtow
import scene_io as sio

MANIFEST = {c["name"]: c for c in json.load(open(os.path.join(sio.GOLDEN, "manifest_extra.json")))["cases"]}
NAMES = ["medium_nested", "medium_bvh_wrapped"]


def _setup(name):
    c = MANIFEST[name]
    W, H = c["width"], c["height"]
    d = sio.load_scene(os.path.join(sio.GOLDEN, name + ".scn"))
    cam = sio.camera_from_file(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"))
    p = sio.default_params(W, H, c["spp"], seed=c["seed"])
    return c, d, cam, p


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_bit_exact(name):
    c, d, cam, p = _setup(name)
    W, H = c["width"], c["height"]
    arrays = sio.SceneArrays(d)
    lin, bgra, cnt = sio.oracle_render(ctypes.addressof(arrays.view), cam, p)
    glin, gbgra = sio.golden_image(name, W, H)
    assert np.array_equal(lin.reshape(H, W, 3).view(np.uint32), glin.view(np.uint32))
    assert np.array_equal(bgra.reshape(H, W, 4), gbgra)
    assert cnt.medium_calls > 0


@pytest.mark.parametrize("name", NAMES)
def test_scene_check_accepts(name):
    _, d, _, _ = _setup(name)
    world = sio.ArrayScene(d)
    stack_need, _ = sio.scene_check(world)
    assert 0 < stack_need <= 48  # the exact-order kernel's call frames (XDEPTH)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_matches_reference(gpu_ctx, name):
    c, d, ocam, op = _setup(name)
    W, H = c["width"], c["height"]
    world = sio.ArrayScene(d)
    gpu_ctx.upload(world)
    bgra, lin, st = gpu_ctx.render(rtow.camera_main(W, H), rtow.params(W, H, c["spp"], seed=c["seed"]))
    glin, gbgra = sio.golden_image(name, W, H)
    a = np.asarray(lin, np.float64).reshape(-1, 3)
    rms = np.sqrt(np.mean((a - glin.reshape(-1, 3)) ** 2, axis=0))
    exact = float(np.mean(lin.reshape(glin.shape) == glin))
    print(f"{name}: rms {rms} exact {exact:.4f}")
    assert (rms <= 1e-4).all(), rms
    assert np.mean(bgra != gbgra) < 0.01
    _, _, cnt = sio.oracle_render(world.view_ptr, ocam, op)
    assert st.segments == cnt.segments
