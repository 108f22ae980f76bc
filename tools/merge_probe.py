"""Does splitting final_ned's top-level list at its media cost traversal
efficiency?  Renders final_ned (a) as is and (b) with its two media dropped
(then the top list becomes ONE tree: treeRuns has no barrier), with the
instrumented kernel when RTOW_PROFILE=1 (SIMD efficiency per variant).
  python tools/merge_probe.py [W H SPP]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import isolate_ground as ig  # noqa: E402
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402


def main():
    W, H, spp = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (1024, 1024, 16)
    d = sio.scene_dict(rtow.Scene.build("final_ned", image="synthetic"))
    h = d["hitables"]
    lst = int(h[d["root"]]["a"]) if h[d["root"]]["kind"] == sio.HIT_TRANSLATE else int(d["root"])
    first, count = int(h[lst]["a"]), int(h[lst]["b"])
    items = [int(r) for r in d["refs"][first:first + count]]
    media = [it for it in items if int(h[it]["kind"]) == 12]
    ctx = rtow.Context(0)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=1)
    for name, keep in [("as is", items), ("no media", [it for it in items if it not in media]),
                       ("media first", media + [it for it in items if it not in media])]:
        ctx.upload(sio.ArrayScene(ig.with_items(d, lst, keep)))
        ctx.render(cam, p, linear=False)
        st = min((ctx.render(cam, p, linear=False)[2] for _ in range(2)), key=lambda s: s.kernel_ms)
        print(f"{name:12s}: {st.kernel_ms:7.2f} ms {st.segments / 1e6:7.2f} M segments "
              f"{st.segments / st.kernel_ms / 1e3:6.0f} Mray/s {st.kernel_ms / st.segments * 1e9:6.2f} ns/segment",
              flush=True)


if __name__ == "__main__":
    main()
