"""A/B of builds on the general-path scenes (cornell, cornell_smoke, final_ned).
  python tools/ab_general.py A.so B.so ...   (AB_SPP, AB_ROUNDS)"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ab  # noqa: E402


def main():
    import torch

    torch.cuda.init()
    libs = [a for a in sys.argv[1:] if ".so" in a]
    spp = int(os.environ.get("AB_SPP", "16"))
    rounds = int(os.environ.get("AB_ROUNDS", "2"))
    mods = [ab.load(f"rtow_g{i}", l) for i, l in enumerate(libs)]
    for name, W, H in [("cornell", 800, 800), ("cornell_smoke", 800, 800), ("final_ned", 1024, 1024)]:
        runs = []
        for m in mods:
            ctx = m.Context(0)
            ctx.upload(m.Scene.build(name, image="synthetic"))
            runs.append((ctx, m.camera_main(W, H), m.params(W, H, spp, seed=1)))
        imgs = [c.render(cam, p)[1] for c, cam, p in runs]
        same = all((im == imgs[0]).all() for im in imgs)
        line = [f"{name} {W}x{H}x{spp} identical={same}"]
        for (c, cam, p), l in zip(runs, libs):
            best = min(c.render(cam, p, linear=False)[2].kernel_ms for _ in range(rounds))
            segs = c.render(cam, p, linear=False)[2].segments
            line.append(f"{os.path.basename(l)}: {best:.1f} ms {segs / best / 1e3:.0f} Mray/s")
        print(" | ".join(line), flush=True)
        for c, _, _ in runs:
            c.close()


if __name__ == "__main__":
    main()
