"""The look-at camera, setCamera_Euler (camera.h:271-313): w = unit(lookFrom -
lookAt), u = unit(cross(up, w)), v = cross(w, u), and the same lower-left /
horizontal / vertical as the quaternion form.  The reference's setCamera()
compiles it out (camera.h:344-350), so main.cpp never uses it; the C-ABI
offers it as rtow_camera_look_at.

Fixtures: the reference's own Camera with setCamera_Euler called on it
(oracle/_ref/ref_harness camera_euler, tests/golden/make_camera_golden.py),
including a degenerate up vector (unit_vector's zero branch, vec3.h:141-148).
CPU: byte-identical basis.  GPU: a frame through that camera within the bar
against the oracle, segment counts equal."""
import json
import os

import numpy as np
import pytest

import rtow
import scene_io as sio

CAMS = json.load(open(os.path.join(sio.GOLDEN, "cameras_euler.json")))


def _cam(c):
    return rtow.camera_look_at(c["look_from"], c["look_at"], c["up"], c["vfov"], c["aspect"], c["aperture"],
                               c["focus"], c["t0"], c["t1"])


@pytest.mark.parametrize("k", range(len(CAMS)))
def test_look_at_camera_matches_reference(k):
    c = CAMS[k]
    assert bytes(_cam(c)) == open(os.path.join(sio.GOLDEN, c["file"]), "rb").read()


def test_degenerate_up_gives_zero_u():
    c = _cam(CAMS[3])
    assert list(c.u) == [0.0, 0.0, 0.0] and list(c.horizontal) == [0.0, 0.0, 0.0]


@pytest.mark.gpu
def test_gpu_frame_through_look_at_camera(gpu_ctx):
    W, H, spp = 64, 36, 16
    c = dict(CAMS[1], aspect=W / H)
    cam = _cam(c)
    scene = rtow.Scene.build("random_ned", n=100, image="synthetic")
    p = rtow.params(W, H, spp, seed=23)
    gpu_ctx.upload(scene)
    _, lin, st = gpu_ctx.render(cam, p)
    olin, _, oc = sio.oracle_render(scene.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                    sio.RtowParams.from_buffer_copy(bytes(p)))
    rms = np.sqrt(np.mean((np.asarray(lin, np.float64).reshape(-1, 3) - olin.astype(np.float64)) ** 2, axis=0))
    print(f"look-at camera: rms {rms} segments gpu {st.segments} oracle {oc.segments}")
    assert (rms <= 1e-4).all(), rms
    assert st.segments == oc.segments
