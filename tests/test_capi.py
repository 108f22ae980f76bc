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
    for code in range(-6, 1):
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


def test_device_count_without_gpu_is_not_a_crash():
    # here (no GPU) this returns 0; on the GPU box >= 1
    assert rtow.device_count() >= 0
