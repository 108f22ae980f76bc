"""Residual corner (ii) pinned by a fixture: an exact tie between a list item
and a BvhNode item whose box the ray enters exactly at the tied t
(tests/golden/make_extra_golden.py `tie_bvh_entry`, ref_harness.cpp
tieBvhEntryNed: a wall rectangle coplanar with the near faces of Boxes in a
BvhNode).  The reference asks the BvhNode with (tmin, t*) (hitableList.h:24-34)
and AABB::hit returns `tmax <= tmin` (aabb.h:22-43), so the wall keeps the
record; a third Box, in a BvhNode whose box starts before the plane, takes the
tie (closed rectangle interval, xy_rect.h).  CPU: the oracle reproduces the
reference bit for bit.  GPU: the culled traversal settles the tie by the tie
keys and marks it (the tie bits of the record); tie_unsettled finds the
Boxes' BvhNode entered at the tied t below the list where the paths part, and
the ray is settled by xhit, the reference's own recursion: the frame within
the bar (without that: 8 % of the pixels differed, RMS up to 3e-2)."""
import ctypes
import json
import os

import numpy as np
import pytest

import scene_io as sio

CASE = {c["name"]: c for c in json.load(open(os.path.join(sio.GOLDEN, "manifest_extra.json")))["cases"]}[
    "tie_bvh_entry"]


def setup():
    c = CASE
    W, H = c["width"], c["height"]
    d = sio.load_scene(os.path.join(sio.GOLDEN, "tie_bvh_entry.scn"))
    cam = sio.camera_from_file(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"))
    p = sio.default_params(W, H, c["spp"], seed=c["seed"])
    return c, d, cam, p


def test_oracle_matches_reference_bit_exact():
    c, d, cam, p = setup()
    W, H = c["width"], c["height"]
    arrays = sio.SceneArrays(d)
    lin, bgra, _ = sio.oracle_render(ctypes.addressof(arrays.view), cam, p)
    glin, gbgra = sio.golden_image("tie_bvh_entry", W, H)
    assert np.array_equal(lin.reshape(H, W, 3).view(np.uint32), glin.view(np.uint32))
    assert np.array_equal(bgra.reshape(H, W, 4), gbgra)


def test_fixture_holds_the_culled_tie():
    """The wall (red) shows where the Boxes' coplanar faces (blue) were never
    tested: some pixels of the frame are wall-red inside the Boxes' outline."""
    c, _, _, _ = setup()
    glin, _ = sio.golden_image("tie_bvh_entry", c["width"], c["height"])
    red = (glin[..., 0] > 1.5 * glin[..., 1]) & (glin[..., 0] > 1.5 * glin[..., 2])
    green = (glin[..., 1] > 1.5 * glin[..., 0]) & (glin[..., 1] > 1.2 * glin[..., 2])
    assert red.sum() > 50 and green.sum() > 3


@pytest.mark.gpu
def test_gpu_matches_reference(gpu_ctx):
    """Within the north-star bar, segment count equal."""
    import rtow

    c, d, ocam, op = setup()
    W, H = c["width"], c["height"]
    world = sio.ArrayScene(d)
    gpu_ctx.upload(world)
    bgra, lin, st = gpu_ctx.render(rtow.camera_main(W, H), rtow.params(W, H, c["spp"], seed=c["seed"]))
    glin, gbgra = sio.golden_image("tie_bvh_entry", W, H)
    a = np.asarray(lin, np.float64).reshape(-1, 3)
    rms = np.sqrt(np.mean((a - glin.reshape(-1, 3)) ** 2, axis=0))
    print(f"tie_bvh_entry: rms {rms} exact {float(np.mean(lin.reshape(glin.shape) == glin)):.4f}")
    assert (rms <= 1e-4).all(), rms
    _, _, cnt = sio.oracle_render(world.view_ptr, ocam, op)
    assert st.segments == cnt.segments
