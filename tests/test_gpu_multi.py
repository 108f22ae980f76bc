"""rtow_multi (include/rtow.h): several GPUs from one process -- device i
renders rank i of n (its 8x8 tiles into a slab, rtow_render_tiles_device), one
RCCL gather (ncclCommInitAll + grouped ncclSend/ncclRecv) to the first device,
which assembles the frame.  The reference's counterpart is its N worker
threads over a column interleave (main.cpp:182-195, 936).

The test box has one GPU, so n = 1 here: device 0's slab still goes through
RCCL (a send to itself), the assemble kernels run, and the frame must equal
rtow_render's bit for bit.  n > 1 needs several GPUs (unmeasured here; the
same code with more communicators)."""
import numpy as np
import pytest

import rtow

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scene,W,H,spp", [("random_ned", 61, 45, 8), ("cornell_smoke", 40, 24, 16),
                                           ("final_ned", 37, 23, 4)])
def test_multi_n1_equals_render_bitwise(scene, W, H, spp, gpu_ctx):
    sc = rtow.Scene.build(scene, n=100, image="synthetic")
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=3)
    gpu_ctx.upload(sc)
    bgra, lin, st = gpu_ctx.render(cam, p)
    m = rtow.Multi([0])
    try:
        m.upload(sc)
        mb, ml, mst, dst = m.render(cam, p)
        assert np.array_equal(mb, bgra)
        assert np.array_equal(ml.view(np.uint32), lin.view(np.uint32))
        assert mst.segments == st.segments and mst.samples == st.samples == W * H * spp
        assert mst.pixels == W * H and len(dst) == 1 and dst[0].segments == st.segments
        assert mst.total_ms >= mst.kernel_ms > 0
        # again, at another size (buffers re-sized), BGRA only
        W2, H2 = 96, 54
        cam2, p2 = rtow.camera_main(W2, H2), rtow.params(W2, H2, 2, seed=4)
        mb2, none, _, _ = m.render(cam2, p2, linear=False)
        assert none is None
        ref2, _, _ = gpu_ctx.render(cam2, p2, linear=False)
        assert np.array_equal(mb2, ref2)
    finally:
        m.close()


def test_render_devices_one_call_and_bad_device(gpu_ctx):
    import ctypes

    L = rtow.lib()
    W, H, spp = 32, 18, 4
    sc = rtow.Scene.build("three_sphere")
    cam, p = rtow.camera_main(W, H), rtow.params(W, H, spp, seed=5)
    gpu_ctx.upload(sc)
    ref, _, _ = gpu_ctx.render(cam, p, linear=False)
    out = np.zeros((H, W, 4), np.uint8)
    st = rtow.Stats()
    devs = (ctypes.c_int * 1)(0)
    rc = L.rtow_render_devices(devs, 1, sc.view_ptr, ctypes.byref(cam), ctypes.byref(p), out.ctypes.data, None,
                               ctypes.byref(st))
    assert rc == rtow.OK, L.rtow_last_error()
    assert np.array_equal(out, ref) and st.samples == W * H * spp
    n = rtow.device_count()
    with pytest.raises(rtow.RtowError) as e:
        rtow.Multi([n])  # one past the last device
    assert e.value.code == rtow.E_INVALID
