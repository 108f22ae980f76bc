"""The reference-side binding (include/rtow_reference.hpp): compiled in the
reference's own translation unit, it flattens the Hitable* world the
reference's scenes.h builds and reads its Camera, for rtow_scene_upload /
rtow_render.

CPU (only where /root/reference and the harness build exist): the harness
now flattens through this header, and for every golden case its dump is
byte-identical to the committed fixture (generated in round 1 by the
harness's own walker) -- which the product's builders also reproduce
(tests/test_scene_graph.py); the camera read through the public getters is
byte-identical to the Camera's private basis, for the main camera and after
the frame loop's updates.

GPU: oracle/_ref/ref_dropin (the harness built with its `dropin` command and
linked against librtow_hip.so -- built here, it travels to the GPU box)
renders the reference's own world through the header and the C-ABI; its
frame equals the product path's (rtow.Scene.build + render) bit for bit."""
import hashlib
import json
import os
import struct
import subprocess

import numpy as np
import pytest

import rtow
import scene_io as sio

REF = "/root/reference/rayTracingOneWeekend"
HARNESS = os.path.join(sio.REPO, "oracle", "_ref", "ref_harness")
DROPIN = os.path.join(sio.REPO, "oracle", "_ref", "ref_dropin")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _stage(tmp_path, image):
    """cwd for the reference's scene builders: the synthetic earth texture
    staged as ./input_images/1_earth_8k.jpg (a lossless PNG; stbi_load reads it)."""
    d = tmp_path / image
    os.makedirs(d / "input_images", exist_ok=True)
    if image == "synthetic":
        from PIL import Image

        Image.fromarray(rtow.synthetic_image(2048, 1024), "RGB").save(d / "input_images" / "1_earth_8k.jpg",
                                                                      format="PNG")
    return str(d)


needs_ref = pytest.mark.skipif(not (os.path.isdir(REF) and os.path.exists(HARNESS)),
                               reason="reference or its harness build not present")


@needs_ref
@pytest.mark.parametrize("name", [c["name"] for c in sio.manifest()["cases"]])
def test_header_flattens_reference_world_as_golden(name, tmp_path):
    c = sio.golden_case(name)
    env = dict(os.environ, RTOW_SCENE_SEED=str(sio.manifest()["scene_seed"]))
    out = str(tmp_path / "w.scn")
    subprocess.run([HARNESS, "dump", c["scene"], out, "--n", str(c["n"]), "--cwd", _stage(tmp_path, c["image"])],
                   env=env, check=True, capture_output=True)
    b = open(out, "rb").read()
    (ntex,) = struct.unpack("<Q", b[48:56])
    body, texels = bytearray(b[:len(b) - ntex]), b[len(b) - ntex:]
    body[48:56] = struct.pack("<Q", 0)
    assert bytes(body) == open(os.path.join(GOLDEN, name + ".scn"), "rb").read()
    assert ntex == c["texel_bytes"] and hashlib.sha256(texels).hexdigest() == c["texel_sha256"]


@needs_ref
@pytest.mark.parametrize("W,H", [(200, 100), (1920, 1080), (48, 48)])
def test_header_camera_equals_private_basis(W, H):
    cams = json.load(open(os.path.join(GOLDEN, "cameras_oriented.json")))
    for c in cams:
        args = [str(v) for v in list(c["look_from"]) + list(c["rows"])]
        r = subprocess.run([HARNESS, "camera_check", str(W), str(H), *args], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/ref_dropin not built (needs /root/reference)")
@pytest.mark.parametrize("scene,n,image", [("cornell", 1, "none"), ("random_ned", 487, "synthetic"),
                                           ("final_ned", 1, "synthetic")])
def test_reference_world_renders_as_product_path(scene, n, image, tmp_path, gpu_ctx):
    W, H, spp, seed = 96, 64, 8, 13
    env = dict(os.environ, RTOW_SCENE_SEED="1")
    pre = str(tmp_path / "d")
    r = subprocess.run([DROPIN, "dropin", scene, str(W), str(H), str(spp), pre, "--n", str(n), "--seed", str(seed),
                        "--cwd", _stage(tmp_path, image)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lin_d = np.fromfile(pre + ".lin", np.float32).reshape(H, W, 3)
    bgra_d = np.fromfile(pre + ".bgra", np.uint8).reshape(H, W, 4)
    sc = rtow.Scene.build(scene, n=n, image=image, scene_seed=1)
    gpu_ctx.upload(sc)
    bgra, lin, st = gpu_ctx.render(rtow.camera_main(W, H), rtow.params(W, H, spp, seed=seed))
    assert json.loads(r.stdout.strip().splitlines()[-1])["segments"] == st.segments
    assert np.array_equal(lin_d.view(np.uint32), lin.reshape(H, W, 3).view(np.uint32))
    assert np.array_equal(bgra_d, bgra.reshape(H, W, 4))


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/ref_dropin not built (needs /root/reference)")
@pytest.mark.parametrize("scene,n,image,ranks", [("random_ned", 487, "synthetic", 0), ("final_ned", 1, "synthetic", 0),
                                                 ("cornell_smoke", 1, "none", 3)])
def test_reference_multi_gpu_binding(scene, n, image, ranks, tmp_path, gpu_ctx):
    """INTEGRATION.md's multi-GPU binding run from inside the reference's own
    translation unit (oracle/_ref/ref_dropin `dropin_multi`): rtow_render_devices
    over every visible device (ranks 0: the RCCL gather, ncclCommInitAll over
    the devices) or over device 0 listed `ranks` times (device-copy gather).
    No torch in that process, so the RCCL it opens is ROCm's own librccl.so.1
    (it prints the mapped path).  The frame equals the product path's
    rtow_render bit for bit."""
    W, H, spp, seed = 120, 72, 8, 29
    env = dict(os.environ, RTOW_SCENE_SEED="1")
    pre = str(tmp_path / "m")
    cmd = [DROPIN, "dropin_multi", scene, str(W), str(H), str(spp), pre, "--n", str(n), "--seed", str(seed),
           "--cwd", _stage(tmp_path, image)]
    if ranks:
        cmd += ["--ranks", str(ranks)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    print("dropin_multi", scene, info)
    if ranks:
        assert info["ranks"] == ranks
    else:
        assert info["ranks"] == info["devices_visible"] >= 1
        assert info["librccl"].endswith("librccl.so") and "torch" not in info["librccl"], info
    sc = rtow.Scene.build(scene, n=n, image=image, scene_seed=1)
    gpu_ctx.upload(sc)
    bgra, lin, st = gpu_ctx.render(rtow.camera_main(W, H), rtow.params(W, H, spp, seed=seed))
    assert info["segments"] == st.segments
    assert np.array_equal(np.fromfile(pre + ".lin", np.float32).view(np.uint32), lin.reshape(-1).view(np.uint32))
    assert np.array_equal(np.fromfile(pre + ".bgra", np.uint8), bgra.reshape(-1))
