"""The sphere test's fast square root (rtow_device.hip sqrt_pos) on the one
kind of ray where it could differ from sqrtf.

sqrt_pos<FAST> skips sqrtf's rescaling of inputs below 2^-96, so for disc =
b*b - a*c in (0, 2^-96) its result can be off by more than an ulp.  A root
is accepted only above tmin = 0.001, and disc < 2^-96 forces |b| < 2^-35, so
that takes a = dot(d, d) < 2^-24: a ray with a vanishing direction.  The
simple-scene kernel therefore traces such rays with the exact variant (equal
to sqrtf for every positive float).  This test builds exactly that case and
compares the GPU's first segment with the oracle's (sqrtf, sphere.h:20-69)
bit for bit: a camera whose rays are d = (2^-37, 0, 0) from the origin
(a = 2^-74), inside a unit sphere centred at (0, 1 - 2^-24, 0), so
c = |oc|^2 - r^2 = -2^-23, b = 0 and disc = 2^-97; the far root is
sqrt(2^-97) / 2^-74 = 2^25.5, the hit point (2^-11.5, 0, 0).
"""
import numpy as np
import pytest

import rtow
import scene_io as sio

pytestmark = pytest.mark.gpu


def tangent_scene():
    d = sio.scene_dict(rtow.Scene.build("random_ned", n=100, image="none", wrap_world=False))
    h = d["hitables"]
    leaves = sio.bvh_leaves_in_order(d)
    target = next(k for k in leaves if h[k]["kind"] == sio.HIT_SPHERE and h[k]["f"][3] < 1.0)
    for j, k in enumerate(leaves):
        if k == target:
            h[k]["f"][:4] = np.array([0.0, 1.0 - 2.0 ** -24, 0.0, 1.0], np.float32)
        elif h[k]["kind"] == sio.HIT_SPHERE:
            h[k]["f"][:4] = np.array([5000.0 + 10 * j, 5000.0, 5000.0, 1.0], np.float32)
        else:  # a MovingSphere: both centers far away
            h[k]["f"][:3] = h[k]["f"][3:6] = np.array([5000.0 + 10 * j, 5000.0, -5000.0], np.float32)
    sio.refresh_bvh_boxes(d)
    return sio.ArrayScene(d)


def tiny_camera():
    c = rtow.Camera()
    c.origin[:] = (0.0, 0.0, 0.0)
    c.lower_left_corner[:] = (2.0 ** -37, 0.0, 0.0)
    c.horizontal[:] = (0.0, 0.0, 0.0)
    c.vertical[:] = (0.0, 0.0, 0.0)
    c.u[:] = (0.0, 1.0, 0.0)
    c.v[:] = (0.0, 0.0, -1.0)
    c.w[:] = (-1.0, 0.0, 0.0)
    c.lens_radius = 0.0
    c.time0, c.time1 = 0.0, 1.0
    return c


def test_tiny_direction_ray_takes_the_exact_sqrt(gpu_ctx):
    sc = tangent_scene()
    assert sio.scene_check(sc)[0] > 0
    gpu_ctx.upload(sc)
    cam = tiny_camera()
    W, H, spp = 4, 4, 2
    p = rtow.params(W, H, spp, seed=3)
    ocam = sio.RtowCamera.from_buffer_copy(bytes(cam))
    op = sio.RtowParams.from_buffer_copy(bytes(p))
    for (x, y, s) in [(0, 0, 0), (3, 2, 1)]:
        g = gpu_ctx.trace_sample(cam, p, x, y, s)
        o = sio.oracle_trace(sc.view_ptr, ocam, op, x, y, s)
        assert len(o) >= 1 and o[0, 0] == 1.0, "the constructed ray must hit the sphere"
        t_expect = np.float32(np.sqrt(np.float32(2.0 ** -97), dtype=np.float32) / np.float32(2.0 ** -74))
        assert o[0, 2] == t_expect, (o[0, 2], t_expect)
        print(f"SQRT tiny ray ({x},{y},{s}): oracle t {o[0, 2]!r} p {o[0, 3:6]} gpu t {g[0, 2]!r} p {g[0, 3:6]} "
              f"segments {len(g)} / {len(o)}")
        assert len(g) == len(o)
        assert np.array_equal(g[:, :11], o[:, :11])  # every segment: hit, t, point, normal, material, draws
    _, lin, st = gpu_ctx.render(cam, p)
    olin, _, oc = sio.oracle_render(sc.view_ptr, ocam, op)
    assert st.segments == oc.segments
    assert np.sqrt(np.mean((lin.reshape(-1, 3).astype(np.float64) - olin) ** 2)) <= 1e-4
