"""Bright emitters.  The reference sums its samples in float with no range
limit (main.cpp:939-955: outputColor += color(...)); the pixel sums here are
signed 192-bit fixed point (rtow_device.hip fx_add), so any emitter whose
samples stay finite in float renders.  cornell with its light scaled to 1e6
(only limb 0 of the sums, as every reference scene) and to 1e30 (sums beyond
2^64: the carries into limbs 1 and 2) against the C oracle: segment counts
equal, and the frame within 1e-6 relative RMS (the absolute 1e-4 bar of the
north star is for the reference scenes' [0, ~20] radiance)."""
import numpy as np
import pytest

import rtow
import scene_io as sio

MAT_DIFFUSE_LIGHT = 4


def _bright_cornell(radiance):
    d = sio.scene_dict(rtow.Scene.build("cornell"))
    for m in d["materials"]:
        if m["kind"] == MAT_DIFFUSE_LIGHT:
            d["textures"][int(m["texture"])]["f"][:3] = radiance
    return d


def test_bright_scene_is_accepted():
    d = _bright_cornell(1e30)
    world = sio.ArrayScene(d)
    sio.scene_check(world)  # no range refusal at the scene level


@pytest.mark.gpu
@pytest.mark.parametrize("radiance", [1e6, 1e30])
def test_gpu_bright_emitter_matches_oracle(gpu_ctx, radiance):
    W, H, spp = 48, 48, 64
    world = sio.ArrayScene(_bright_cornell(radiance))
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=2)
    gpu_ctx.upload(world)
    _, lin, st = gpu_ctx.render(cam, p)
    olin, _, cnt = sio.oracle_render(world.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                     sio.RtowParams.from_buffer_copy(bytes(p)))
    assert st.segments == cnt.segments
    a = lin.reshape(-1, 3).astype(np.float64)
    b = olin.astype(np.float64)
    assert np.isfinite(a).all() and b.max() > radiance * 1e-3
    rel = np.sqrt(np.mean((a - b) ** 2)) / np.sqrt(np.mean(b ** 2))
    print(f"radiance {radiance:g}: relative rms {rel:.3e}")
    assert rel <= 1e-6
