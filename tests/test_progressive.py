"""Frame-loop pieces: the camera after the GUI loop's updates (pinned against
the reference's own Camera, tests/golden/make_camera_golden.py) and
progressive accumulation across frames (rtow_render_progressive)."""
import json
import os

import numpy as np
import pytest

import rtow
import scene_io as sio

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CAMS = json.load(open(os.path.join(GOLDEN, "cameras_oriented.json")))


@pytest.mark.parametrize("c", CAMS, ids=[c["file"] for c in CAMS])
def test_oriented_camera_matches_reference(c):
    cam = rtow.camera_oriented(c["width"], c["height"], c["look_from"], c["rows"])
    assert bytes(cam) == open(os.path.join(GOLDEN, c["file"]), "rb").read()


@pytest.mark.gpu
def test_progressive_frames_equal_one_render(gpu_ctx):
    """F frames of S spp == one render of F*S spp with samples_per_chunk S,
    bit for bit (the random streams continue; the sums add in the same order)."""
    W, H, S, F = 72, 40, 8, 4
    scene = rtow.Scene.build("random_ned", n=100, image="synthetic")
    gpu_ctx.upload(scene)
    cam = rtow.camera_main(W, H)
    ref_bgra, ref_lin, _ = gpu_ctx.render(cam, rtow.params(W, H, F * S, seed=3, samples_per_chunk=S))
    for f in range(F):
        bgra, lin, total, _ = gpu_ctx.render_progressive(cam, rtow.params(W, H, S, seed=3), reset=(f == 0))
        assert total == (f + 1) * S
    assert np.array_equal(lin.view(np.uint32), ref_lin.view(np.uint32))
    assert np.array_equal(bgra, ref_bgra)


@pytest.mark.gpu
def test_progressive_restarts_on_camera_change(gpu_ctx):
    W, H = 40, 24
    scene = rtow.Scene.build("three_sphere")
    gpu_ctx.upload(scene)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, 4, seed=1)
    gpu_ctx.render_progressive(cam, p, reset=True)
    _, _, total, _ = gpu_ctx.render_progressive(cam, p)
    assert total == 8
    c = CAMS[1]
    moved = rtow.camera_oriented(W, H, c["look_from"], c["rows"])
    _, lin, total, _ = gpu_ctx.render_progressive(moved, p)
    assert total == 4
    _, one, _ = gpu_ctx.render(moved, p)
    assert np.array_equal(lin, one)


@pytest.mark.gpu
def test_progressive_restarts_when_dof_turns_on(gpu_ctx):
    """RTOW_FLAG_CAMERA_DOF changes the image, so switching it restarts the
    running sums (pinhole and depth-of-field samples are never averaged into
    one frame); RTOW_FLAG_STATS does not."""
    W, H = 40, 24
    scene = rtow.Scene.build("three_sphere")
    gpu_ctx.upload(scene)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, 4, seed=1)
    gpu_ctx.render_progressive(cam, p, reset=True)
    pd = rtow.params(W, H, 4, seed=1)
    pd.flags |= rtow.FLAG_CAMERA_DOF
    _, lin, total, _ = gpu_ctx.render_progressive(cam, pd)
    assert total == 4
    _, one, _ = gpu_ctx.render(cam, pd)
    assert np.array_equal(lin, one)
    ps = rtow.params(W, H, 4, seed=1)
    ps.flags = pd.flags ^ rtow.FLAG_STATS
    _, _, total, _ = gpu_ctx.render_progressive(cam, ps)
    assert total == 8


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["random_ned", "cornell"])
def test_oriented_camera_render_matches_oracle(scene, gpu_ctx):
    c = CAMS[2]
    W, H, spp = c["width"], c["height"], 8
    sc = rtow.Scene.build(scene, n=100, image="synthetic")
    gpu_ctx.upload(sc)
    cam = rtow.camera_oriented(W, H, c["look_from"], c["rows"])
    p = rtow.params(W, H, spp, seed=2)
    _, lin, _ = gpu_ctx.render(cam, p)
    olin, _, _ = sio.oracle_render(sc.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                   sio.RtowParams.from_buffer_copy(bytes(p)))
    rms = np.sqrt(np.mean((lin.reshape(-1, 3).astype(np.float64) - olin) ** 2, axis=0))
    assert (rms <= 1e-4).all(), rms


@pytest.mark.gpu
def test_progressive_restarts_on_scene_upload(gpu_ctx):
    """Running sums belong to the scene they were rendered from: after a new
    upload, a progressive frame without reset equals a fresh render of the
    new scene (not a mix of both scenes)."""
    W, H = 40, 24
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, 4, seed=1)
    gpu_ctx.upload(rtow.Scene.build("three_sphere"))
    gpu_ctx.render_progressive(cam, p, reset=True)
    gpu_ctx.render_progressive(cam, p)
    b = rtow.Scene.build("random_ned", n=100, image="synthetic")
    gpu_ctx.upload(b)
    _, lin, total, _ = gpu_ctx.render_progressive(cam, p)
    assert total == 4
    _, one, _ = gpu_ctx.render(cam, p)
    assert np.array_equal(lin.view(np.uint32), one.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_progressive_tiles_assemble_to_progressive_frame(world, gpu_ctx):
    """Multi-GPU progressive frames: every rank (its own context, as on its own
    GPU) adds F frames of S spp of its tiles (rtow_render_progressive_tiles_device);
    the assembled BGRA and linear frames equal rtow_render_progressive's after
    the same F calls, bit for bit."""
    import torch

    W, H, S, F = 61, 45, 4, 3
    scene = rtow.Scene.build("random_ned", n=100, image="synthetic")
    gpu_ctx.upload(scene)
    cam = rtow.camera_main(W, H)
    for f in range(F):
        ref_bgra, ref_lin, _, _ = gpu_ctx.render_progressive(cam, rtow.params(W, H, S, seed=5), reset=(f == 0))
    stride = rtow.rank_tile_count(W, H, 0, world) * 64
    bgra = torch.zeros((world, stride * 4), dtype=torch.uint8, device="cuda")
    lin = torch.zeros((world, stride * 3), dtype=torch.float32, device="cuda")
    ctxs = [rtow.Context(0) for _ in range(world)]
    try:
        for r, ctx in enumerate(ctxs):
            ctx.upload(scene)
            for f in range(F):
                total, _ = ctx.render_progressive_tiles_device(cam, rtow.params(W, H, S, seed=5, rank=r, world=world),
                                                               bgra[r].data_ptr(), lin[r].data_ptr(), reset=(f == 0))
                assert total == (f + 1) * S
    finally:
        for ctx in ctxs:
            ctx.close()
    fb = rtow.assemble(bgra.cpu().numpy().reshape(world, stride, 4), W, H, world)
    fl = rtow.assemble(lin.cpu().numpy().reshape(world, stride, 3), W, H, world)
    assert np.array_equal(fb, ref_bgra)
    assert np.array_equal(fl.view(np.uint32), ref_lin.view(np.uint32))


@pytest.mark.gpu
def test_progressive_tiles_restart_on_partition_change(gpu_ctx):
    """The running sums belong to one rank's tiles: a call for another rank or
    world restarts them."""
    import torch

    W, H, S = 40, 24, 4
    gpu_ctx.upload(rtow.Scene.build("three_sphere"))
    cam = rtow.camera_main(W, H)
    slab = torch.zeros(rtow.rank_tile_count(W, H, 0, 2) * 64 * 4, dtype=torch.uint8, device="cuda")
    total, _ = gpu_ctx.render_progressive_tiles_device(cam, rtow.params(W, H, S, rank=0, world=2), slab.data_ptr(),
                                                       reset=True)
    total, _ = gpu_ctx.render_progressive_tiles_device(cam, rtow.params(W, H, S, rank=0, world=2), slab.data_ptr())
    assert total == 2 * S
    total, _ = gpu_ctx.render_progressive_tiles_device(cam, rtow.params(W, H, S, rank=1, world=2), slab.data_ptr())
    assert total == S
    with pytest.raises(rtow.RtowError):
        gpu_ctx.render_progressive_tiles_device(cam, rtow.params(W, H, S, rank=2, world=2), slab.data_ptr())
