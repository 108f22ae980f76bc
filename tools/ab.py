"""A/B two builds of librtow_hip.so in ONE process, interleaved rounds.

  python tools/ab.py A.so B.so [C.so ...]   (AB_SPP, AB_ROUNDS, AB_SPC, AB_SCENES)
Each build is loaded through its own copy of rtow.py (RTOW_LIB), renders the
same frames; images must be identical; the kernel times are compared."""
import importlib.util
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
EARTH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "input_images", "1_earth_8k.jpg")  # the benched scenes' texture (scenes.h:140)
RTOW_PY = os.path.join(HERE, "..", "ray-tracing-one-weekend_amd", "rtow.py")


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
    # each variant: path/to/lib.so[:ENV=VAL[,ENV=VAL]] (env applied while its contexts are created and the scene uploaded)
    specs = [a for a in sys.argv[1:] if ".so" in a]
    libs = [a.split(":")[0] for a in specs]
    envs = [dict(kv.split("=") for kv in a.split(":")[1].split(",")) if ":" in a else {} for a in specs]
    spp = int(os.environ.get("AB_SPP", "32"))
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    mods = [load(f"rtow_{i}", l) for i, l in enumerate(libs)]
    names = [os.path.basename(sp) for sp in specs]
    spc = int(os.environ.get("AB_SPC", "16"))
    configs = [("random_ned", 487, 1920, 1080, spp), ("cornell_smoke", 100, 800, 800, spp),
               ("cornell", 100, 800, 800, spp), ("final_ned", 100, 1024, 1024, spp)]
    only = os.environ.get("AB_SCENES", "random_ned,cornell_smoke").split(",")
    configs = [c for c in configs if c[0] in only]
    for name, n, W, H, s in configs:
        runs = []
        for m, env in zip(mods, envs):
            sc = m.Scene.build(name, n=n, image="jpeg", image_path=EARTH)
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            ctx = m.Context(0)
            ctx.upload(sc)  # scene-layout knobs (RTOW_BVH) are read at upload
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            runs.append((m, sc, ctx, m.camera_main(W, H), m.params(W, H, s, seed=1, samples_per_chunk=spc)))
        imgs = [r[2].render(r[3], r[4], linear=True)[1] for r in runs]
        same = all((im == imgs[0]).all() for im in imgs)
        if not same:
            import numpy as np
            for i in range(1, len(imgs)):
                d = np.abs(imgs[i] - imgs[0]).max(axis=-1)
                print(f"  {name}: {names[i]} vs {names[0]}: "
                      f"{int((d > 0).sum())} pixels differ, max {d.max():.3g}, "
                      f"rms {float(np.sqrt(np.mean((imgs[i] - imgs[0]) ** 2))):.3g}", flush=True)
        t = [[] for _ in runs]
        for _ in range(rounds):
            for i, (m, sc, ctx, cam, p) in enumerate(runs):
                _, _, st = ctx.render(cam, p, linear=False)
                t[i].append((st.kernel_ms, st.segments))
        line = [f"{name} {W}x{H}x{s} identical={same}"]
        for i, l in enumerate(names):
            ms = sorted(k for k, _ in t[i])
            line.append(f"{l}: min {ms[0]:.1f} med {ms[len(ms)//2]:.1f} ms "
                        f"{t[i][0][1] / ms[0] / 1e3:.0f} Mray/s")
        print(" | ".join(line), flush=True)
        for r in runs:
            r[2].close()


if __name__ == "__main__":
    main()
