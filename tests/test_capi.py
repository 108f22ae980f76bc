"""C-ABI surface: the library loads, exports every function include/rtow.h
declares, and the host-only entry points behave (no GPU compute here)."""
import ctypes

import numpy as np
import pytest

import rtow


def test_exports_every_declared_symbol():
    names = rtow.header_functions()
    assert len(names) >= 20
    L = ctypes.CDLL(rtow.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_abi_version_and_errors():
    L = rtow.lib()
    assert L.rtow_abi_version() == 1
    for code in range(-7, 1):
        assert L.rtow_error_string(code)
    assert L.rtow_error_string(-99) == b"unknown error"


def test_params_default_reproduce_defines():
    p = rtow.params(800, 800, 64)
    assert (p.max_depth, p.gi_enable, p.world) == (50, 1, 1)
    assert p.sky_gain == pytest.approx(1.0) and p.gi_gain == np.float32(0.3)


@pytest.mark.parametrize("W,H,world", [(1920, 1080, 1), (1920, 1080, 8), (37, 23, 3), (1, 1, 2), (4096, 4096, 8)])
def test_tile_partition_covers_every_tile_once(W, H, world):
    n = rtow.tile_count(W, H)
    assert n == ((W + 7) // 8) * ((H + 7) // 8)
    counts = [rtow.rank_tile_count(W, H, r, world) for r in range(world)]
    assert sum(counts) == n
    assert max(counts) - min(counts) <= 1


def test_bad_arguments_fail_loudly():
    L = rtow.lib()
    assert L.rtow_build_scene(99, None, ctypes.byref(ctypes.c_void_p())) == rtow.E_INVALID
    assert L.rtow_camera_main(0, 10, ctypes.byref(rtow.Camera())) == rtow.E_INVALID
    with pytest.raises(rtow.RtowError):
        rtow.Scene.load("/nonexistent/file.scn")
    with pytest.raises(rtow.RtowError):
        rtow.Scene.build("random_ned", n=2)


@pytest.mark.parametrize("W,H,spp,rank,world,spc,n_big,tail,n_tail", [
    (1920, 1080, 1024, 0, 1, 128, 7, 128, 8),   # the bench's config-2 frame on one GPU
    (1920, 1080, 1024, 0, 2, 128, 7, 128, 8),
    (1920, 1080, 1024, 0, 4, 64, 15, 64, 7),
    (1920, 1080, 1024, 3, 8, 32, 31, 32, 6),    # one rank of the 8-GPU config-2 frame
    (4096, 4096, 8192, 0, 8, 128, 63, 128, 8),  # config 5: rank 0 of 8
    (4096, 4096, 512, 0, 8, 128, 3, 128, 8),    # the config-5 share the GPU parity test renders
    (800, 800, 4096, 0, 1, 128, 31, 128, 8),    # configs 3/4
    (64, 36, 16, 0, 1, 16, 1, 0, 0),            # small frames: one 16-sample chunk, no tail
])
def test_render_plan_matches_the_documented_chunking(W, H, spp, rank, world, spc, n_big, tail, n_tail):
    """rtow_render_plan (no context: a 256-CU MI355X) exposes the automatic
    chunking the kernels run: 128/64/32/16-sample items leaving >= 30 items per
    lane, then the halving tail (DevParams, rtow_device.hip)."""
    pl = rtow.plan(rtow.params(W, H, spp, rank=rank, world=world))
    assert (pl.samples_per_chunk, pl.n_big, pl.tail_samples, pl.n_tail) == (spc, n_big, tail, n_tail)
    assert pl.n_chunks == n_big + n_tail and pl.cus == 256
    assert pl.n_local_px == rtow.rank_tile_count(W, H, rank, world) * 64
    assert pl.n_items == pl.n_chunks * pl.n_local_px
    # the chunks cover every sample once: n_big full chunks, then the tail
    assert n_big * spc + tail == spp or (n_tail == 0 and (n_big - 1) * spc < spp <= n_big * spc)
    fixed = rtow.plan(rtow.params(W, H, spp, rank=rank, world=world, samples_per_chunk=16))
    assert (fixed.samples_per_chunk, fixed.n_tail) == (16, 0) and fixed.n_big == (spp + 15) // 16
    with pytest.raises(rtow.RtowError):
        rtow.plan(rtow.params(W, H, 0))


def test_device_count_without_gpu_is_not_a_crash():
    # here (no GPU) this returns 0; on the GPU box >= 1
    assert rtow.device_count() >= 0


def test_multi_gpu_arguments_are_validated_before_any_gpu_call():
    """rtow_multi_create / rtow_render_devices (several GPUs from one process,
    one RCCL gather): bad device lists fail with E_INVALID before HIP or RCCL
    is touched; a valid list on a machine without a GPU is E_NO_DEVICE."""
    L = rtow.lib()
    h = ctypes.c_void_p()
    i32 = ctypes.c_int
    assert L.rtow_multi_create(None, 1, ctypes.byref(h)) == rtow.E_INVALID
    assert L.rtow_multi_create((i32 * 1)(0), 0, ctypes.byref(h)) == rtow.E_INVALID
    assert L.rtow_multi_create((i32 * 2)(0, -1), 2, ctypes.byref(h)) == rtow.E_INVALID
    assert L.rtow_multi_create((i32 * 1)(0), 1, None) == rtow.E_INVALID
    assert h.value is None
    assert L.rtow_multi_destroy(None) == rtow.OK
    assert L.rtow_multi_device_count(None) == 0
    assert L.rtow_multi_upload(None, None) == rtow.E_INVALID
    assert L.rtow_multi_render(None, None, None, None, None, None, None) == rtow.E_INVALID
    cam, p = rtow.camera_main(16, 8), rtow.params(16, 8, 1)
    assert L.rtow_render_devices((i32 * 1)(0), 1, None, ctypes.byref(cam), ctypes.byref(p), None, None,
                                 None) == rtow.E_INVALID
    if rtow.device_count() == 0:
        rc = L.rtow_multi_create((i32 * 2)(0, 1), 2, ctypes.byref(h))
        assert rc == rtow.E_NO_DEVICE and h.value is None
        # a device listed twice is two ranks sharing it (no RCCL): still a device call
        assert L.rtow_multi_create((i32 * 2)(0, 0), 2, ctypes.byref(h)) == rtow.E_NO_DEVICE
    assert L.rtow_error_string(rtow.E_RCCL) == b"RCCL error"


def test_library_loads_without_rccl():
    """librtow_hip.so does not link RCCL: rtow_multi opens librccl.so.1 at the
    first rtow_multi_create that needs it, so single-GPU callers
    load the library (and the ctypes binding) without RCCL present."""
    import subprocess

    out = subprocess.run(["readelf", "-d", rtow.LIB_PATH], capture_output=True, text=True, check=True).stdout
    needed = [line for line in out.splitlines() if "NEEDED" in line]
    assert needed and not any("rccl" in line for line in needed), needed


@pytest.mark.parametrize("W,H,spp,world", [(1920, 1080, 1024, 8), (1920, 1080, 256, 2), (4096, 4096, 8192, 8),
                                           (800, 800, 4096, 4), (61, 45, 8, 3)])
def test_frame_plan_flag_gives_every_rank_the_whole_frames_chunks(W, H, spp, world):
    """RTOW_FLAG_FRAME_PLAN: a rank of any world cuts its samples as rtow_render
    cuts the whole frame's (rank 0 of 1), so chunk float sums -- and the
    assembled frame -- do not depend on the world size; without it a rank's
    share plans for its own pixel count (config 2 at 8 ranks: 32-sample items
    against the frame's 128)."""
    whole = rtow.plan(rtow.params(W, H, spp))
    for rank in range(world):
        pl = rtow.plan(rtow.params(W, H, spp, rank=rank, world=world, flags=rtow.FLAG_FRAME_PLAN))
        assert (pl.samples_per_chunk, pl.n_big, pl.tail_samples, pl.n_tail, pl.n_chunks) == \
               (whole.samples_per_chunk, whole.n_big, whole.tail_samples, whole.n_tail, whole.n_chunks)
        assert pl.n_local_px == rtow.rank_tile_count(W, H, rank, world) * 64
    own = rtow.plan(rtow.params(W, H, spp, rank=0, world=world))
    if (W, H, spp, world) in ((1920, 1080, 1024, 8), (1920, 1080, 256, 2)):
        assert own.samples_per_chunk < whole.samples_per_chunk  # the flag matters here
