"""Cost of the texture kinds in the config-2 frame: the same scene with one
texture kind at a time replaced by a constant, kernel time compared.
(Images differ, of course; this measures where shading time goes.)"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

TEX_CONSTANT, TEX_CHECKER, TEX_NOISE, TEX_IMAGE = 1, 2, 3, 4


def main():
    W, H, spp = 1920, 1080, int(os.environ.get("SC_SPP", "16"))
    d = sio.scene_dict(rtow.Scene.build("random_ned", n=487, image="synthetic"))
    ctx = rtow.Context(0)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=1)
    variants = [("original", None), ("noise->const", TEX_NOISE), ("checker->const", TEX_CHECKER),
                ("image->const", TEX_IMAGE)]
    for name, kind in variants:
        e = {k: (v.copy() if hasattr(v, "copy") else v) for k, v in d.items()}
        if kind:
            t = e["textures"]
            for i in range(len(t)):
                if t[i]["kind"] == kind:
                    t[i]["kind"] = TEX_CONSTANT
                    t[i]["f"][:3] = (0.5, 0.5, 0.5)
        sc = sio.ArrayScene(e)
        ctx.upload(sc)
        ctx.render(cam, p, linear=False)
        best = min(ctx.render(cam, p, linear=False)[2].kernel_ms for _ in range(2))
        _, _, st = ctx.render(cam, p, linear=False)
        print(f"{name:16s} kernel {best:7.1f} ms  segments {st.segments}  {st.segments / best / 1e3:.0f} Mray/s",
              flush=True)


if __name__ == "__main__":
    main()
