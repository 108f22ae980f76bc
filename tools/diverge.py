"""Find pixels where library builds disagree on a large frame and check each
build against the C oracle on exactly those pixels (diagnostic)."""
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import scene_io as sio  # noqa: E402

RTOW_PY = os.path.join(HERE, "..", "ray-tracing-one-weekend_amd", "rtow.py")
THR = float(os.environ.get("DV_THR", "1e-3"))  # DV_SCENE, DV_W, DV_H, DV_SPP, DV_THR


def load(name, lib):
    os.environ["RTOW_LIB"] = os.path.abspath(lib)
    spec = importlib.util.spec_from_file_location(name, RTOW_PY)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    m.lib()
    return m


def main():
    import torch

    torch.cuda.init()
    libs = [a for a in sys.argv[1:] if a.endswith(".so")]
    W, H, spp = int(os.environ.get("DV_W", 1920)), int(os.environ.get("DV_H", 1080)), int(os.environ.get("DV_SPP", 32))
    mods = [load(f"m{i}", l) for i, l in enumerate(libs)]
    lins = []
    scene = None
    for m in mods:
        scene = m.Scene.build(os.environ.get("DV_SCENE", "random_ned"), n=487, image="synthetic")
        ctx = m.Context(0)
        ctx.upload(scene)
        cam = m.camera_main(W, H)
        p = m.params(W, H, spp, seed=1)
        _, lin, _ = ctx.render(cam, p)
        lins.append(lin.reshape(-1, 3))
        ctx.close()
    diff = np.zeros(W * H, bool)
    for l in lins[1:]:
        diff |= (l != lins[0]).any(axis=1)
    big = np.zeros(W * H, bool)
    for l in lins[1:]:
        big |= np.abs(l - lins[0]).max(axis=1) > THR
    pix = np.nonzero(big)[0].astype(np.uint32)
    print(f"{diff.sum()} pixels differ in any bit, {big.sum()} by > {THR}")
    m = mods[0]
    cam = m.camera_main(W, H)
    p = m.params(W, H, spp, seed=1)
    olin, _, _ = sio.oracle_render(scene.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                   sio.RtowParams.from_buffer_copy(bytes(p)), pixels=pix, threads=16)
    for i, l in enumerate(lins):
        d = np.abs(l[pix] - olin).max(axis=1)
        print(f"{os.path.basename(libs[i])}: on those pixels, {int((d > THR).sum())} differ from the oracle by > {THR}; "
              f"full-frame rms vs oracle restricted to them: {float(np.sqrt(np.sum((l[pix]-olin)**2)/(W*H*3))):.3g}")
    print("pixels", pix[:32].tolist())
    np.save(os.path.join(HERE, "..", "gpurun_out", "diverge_pix.npy"), pix)


if __name__ == "__main__":
    main()
