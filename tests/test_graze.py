"""Residual corner (i) pinned by a fixture (tests/golden/make_graze_golden.py,
ref_harness.cpp grazeMediumNed): one exact primary ray grazes the edge of a
Box held by an n == 1 BvhNode -- the reference's AABB::hit (aabb.h:22-43)
never tests the Box, although its side's rectangle would take the edge point
-- then meets a ConstantMedium's boundary beyond that point and, first of
all, a sphere in front of both.  The reference asks the medium with the whole
interval and draws its scatter distance (constantMedium.h:26-74); a
traversal that took the grazed side hands the medium that side's t, skips the
draw and ends at the same sphere one draw behind, so every later bounce of
the sample differs.  The device notices the grazed rectangle when it asks the
medium (ref_skips_hit on the record) and settles the ray with xhit.

CPU: the oracle reproduces the reference bit for bit, and its path of the
sample shows the medium's two draws.  GPU: the sample's path segment for
segment as the oracle's (hits, materials, draw counts), the frame within the
bar with the segment count equal."""
import ctypes
import json
import os

import numpy as np
import pytest

import rtow
import scene_io as sio

CASE = {c["name"]: c for c in json.load(open(os.path.join(sio.GOLDEN, "manifest_extra.json")))["cases"]}[
    "graze_medium"]


def setup():
    c = CASE
    W, H = c["width"], c["height"]
    d = sio.load_scene(os.path.join(sio.GOLDEN, "graze_medium.scn"))
    cam = sio.camera_from_file(os.path.join(sio.GOLDEN, f"cam_{W}x{H}.cam"))
    p = sio.default_params(W, H, c["spp"], seed=c["seed"])
    return c, d, cam, p


def test_oracle_matches_reference_bit_exact():
    c, d, cam, p = setup()
    W, H = c["width"], c["height"]
    arrays = sio.SceneArrays(d)
    lin, bgra, _ = sio.oracle_render(ctypes.addressof(arrays.view), cam, p)
    glin, gbgra = sio.golden_image("graze_medium", W, H)
    assert np.array_equal(lin.reshape(H, W, 3).view(np.uint32), glin.view(np.uint32))
    assert np.array_equal(bgra.reshape(H, W, 4), gbgra)


def test_the_sample_draws_the_medium_scatter_distance():
    """Segment 0 of the sample ends at the sphere (the fixture's hitable 12's
    material) after 5 draws: jitter u, v, time, the medium's discarded draw
    and its scatter distance -- the reference asked the medium with the whole
    interval (the grazed Box was never tested)."""
    c, d, cam, p = setup()
    col, row, s = c["trace"]
    arrays = sio.SceneArrays(d)
    tr = sio.oracle_trace(ctypes.addressof(arrays.view), cam, p, col, c["height"] - 1 - row, s)
    assert tr[0, 0] == 1.0 and tr[0, 10] == 5.0


@pytest.mark.gpu
def test_gpu_follows_the_reference_path(gpu_ctx):
    c, d, ocam, op = setup()
    W, H = c["width"], c["height"]
    col, row, s = c["trace"]
    world = sio.ArrayScene(d)
    gpu_ctx.upload(world)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, c["spp"], seed=c["seed"])
    g = gpu_ctx.trace_sample(cam, p, col, H - 1 - row, s)
    o = sio.oracle_trace(world.view_ptr, ocam, op, col, H - 1 - row, s)
    print("gpu", g[:, [0, 2, 9, 10]].tolist(), "oracle", o[:, [0, 2, 9, 10]].tolist())
    assert g.shape == o.shape
    assert np.array_equal(g[:, [0, 1, 9, 10]], o[:, [0, 1, 9, 10]])  # hit, depth, material, draws
    assert np.allclose(g, o, rtol=1e-5, atol=1e-6)
    bgra, lin, st = gpu_ctx.render(cam, p)
    glin, _ = sio.golden_image("graze_medium", W, H)
    rms = np.sqrt(np.mean((np.asarray(lin, np.float64).reshape(-1, 3) - glin.reshape(-1, 3)) ** 2, axis=0))
    assert (rms <= 1e-4).all(), rms
    _, _, cnt = sio.oracle_render(world.view_ptr, ocam, op)
    assert st.segments == cnt.segments
