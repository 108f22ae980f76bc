"""Edge cases of the boundary (include/rtow.h) and of the worlds the reference
allows but its own scenes never build:

* an empty HitableList (hitableList.h:20-38 returns no hit: every ray is sky,
  color.h:48-57), a world that is one bare Sphere (no list, no BvhNode), a
  BvhNode over ONE leaf (bvhNode.h:38-39: left == right, the leaf asked
  twice), and a world that is only an emitter;
* degenerate frames: 1 x 1, a one-pixel-wide column, a one-row strip, 1 spp,
  max_depth 0 and 1 (DEPTH_RECURSION, color.h:23);
* the argument checks: a frame beyond 2^31 pixels, rank >= world, spp 0.

CPU: the oracle renders every world (the reference's semantics, restated
bit-exactly elsewhere) and the layout builds; GPU: the HIP path against the
oracle, per-channel RMS <= 1e-4 and equal segment counts."""
import ctypes

import numpy as np
import pytest

import rtow
import scene_io as sio

HITABLE = sio.HITABLE


def _base():
    return sio.scene_dict(rtow.Scene.build("three_sphere", n=1, image="none"))


def _hit(kind, a=0, b=0, f=()):
    h = np.zeros(1, HITABLE)
    h[0]["kind"], h[0]["a"], h[0]["b"] = kind, a, b
    h[0]["f"][: len(f)] = f
    return h


def _world(name):
    d = dict(_base())
    mats = d["materials"]
    if name == "empty_list":
        d["hitables"] = _hit(sio.HIT_LIST, 0, 0)
        d["refs"] = np.zeros(0, np.uint32)
    elif name == "bare_sphere":
        d["hitables"] = _hit(sio.HIT_SPHERE, 1, 0, (10.0, 0.0, 0.0, 1.5))
        d["refs"] = np.zeros(0, np.uint32)
    elif name == "bvh_one_leaf":  # BvhNode(list, 1): left = right = the leaf
        c, r = np.float32([10.0, 0.5, -0.25]), np.float32(2.0)
        d["hitables"] = np.concatenate([_hit(sio.HIT_BVH_NODE, 1, 1, tuple(c - r) + tuple(c + r)),
                                        _hit(sio.HIT_SPHERE, 2, 0, tuple(c) + (float(r),))])
        d["refs"] = np.zeros(0, np.uint32)
    elif name == "emitter_only":  # a DiffuseLight sphere in a list: the light itself, sky around it
        light = mats[:1].copy()
        light[0]["kind"] = 4  # RTOW_MAT_DIFFUSE_LIGHT, texture 0
        d["materials"] = np.concatenate([mats, light])
        d["hitables"] = np.concatenate([_hit(sio.HIT_LIST, 0, 1),
                                        _hit(sio.HIT_SPHERE, len(mats), 0, (8.0, 0.0, 0.0, 3.0))])
        d["refs"] = np.array([1], np.uint32)
    else:
        raise ValueError(name)
    d["root"] = 0
    return sio.ArrayScene(d)


WORLDS = ["empty_list", "bare_sphere", "bvh_one_leaf", "emitter_only"]


def _oracle(scene, cam, p):
    return sio.oracle_render(scene.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                             sio.RtowParams.from_buffer_copy(bytes(p)))


@pytest.mark.parametrize("name", WORLDS)
def test_world_builds_and_oracle_renders(name):
    scene = _world(name)
    sio.scene_check(scene)
    W, H = 16, 9
    lin, _, oc = _oracle(scene, rtow.camera_main(W, H), rtow.params(W, H, 4, seed=3))
    assert np.isfinite(lin).all() and oc.samples == W * H * 4
    if name == "empty_list":
        assert oc.segments == oc.samples  # every ray is sky at once


def test_argument_checks():
    with pytest.raises(rtow.RtowError):
        rtow.plan(rtow.params(1 << 16, (1 << 15) + 1, 1))  # more than 2^31 pixels
    with pytest.raises(rtow.RtowError):
        rtow.plan(rtow.params(64, 64, 1, rank=2, world=2))
    with pytest.raises(rtow.RtowError):
        rtow.plan(rtow.params(64, 64, 0))
    pl = rtow.plan(rtow.params(1, 1, 1))
    assert pl.n_local_px == 64 and pl.n_items >= 1  # one 8x8 tile, one live pixel


def _gpu_vs_oracle(ctx, scene, W, H, spp, seed=5, **kw):
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=seed, **kw)
    ctx.upload(scene)
    bgra, lin, st = ctx.render(cam, p)
    olin, obgra, oc = _oracle(scene, cam, p)
    a = np.asarray(lin, np.float64).reshape(-1, 3)
    rms = np.sqrt(np.mean((a - olin.astype(np.float64)) ** 2, axis=0))
    return rms, st, oc, bgra, obgra


@pytest.mark.gpu
@pytest.mark.parametrize("name", WORLDS)
def test_gpu_edge_worlds(name, gpu_ctx):
    rms, st, oc, bgra, obgra = _gpu_vs_oracle(gpu_ctx, _world(name), 40, 24, 8)
    print(f"{name}: rms {rms} segments gpu {st.segments} oracle {oc.segments}")
    assert (rms <= 1e-4).all(), rms
    assert st.segments == oc.segments
    if name == "empty_list":
        assert np.array_equal(bgra.reshape(-1), obgra.reshape(-1))


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,spp,kw", [(1, 1, 1, {}), (1, 1, 1000, {}), (1, 37, 16, {}), (53, 1, 16, {}),
                                        (24, 16, 8, {"max_depth": 0}), (24, 16, 8, {"max_depth": 1})])
def test_gpu_degenerate_frames(W, H, spp, kw, gpu_ctx):
    scene = rtow.Scene.build("random_ned", n=100, image="synthetic")
    rms, st, oc, _, _ = _gpu_vs_oracle(gpu_ctx, scene, W, H, spp, **kw)
    print(f"{W}x{H}x{spp} {kw}: rms {rms} segments gpu {st.segments} oracle {oc.segments}")
    assert (rms <= 1e-4).all(), rms
    assert st.segments == oc.segments
    assert st.samples == W * H * spp
