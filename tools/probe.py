"""Quick A/B of trace-kernel variants in ONE process (interleaved rounds)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-one-weekend_amd"))
import rtow  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
variants = [int(v) for v in os.environ.get("PROBE_WAVES", "0,3,4,5").split(",")]
rounds = int(os.environ.get("PROBE_ROUNDS", "2"))
configs = [("random_ned", 487, 1920, 1080, int(os.environ.get("PROBE_SPP", "32"))), ("cornell_smoke", 100, 800, 800, 32),
           ("cornell", 100, 800, 800, 32), ("final_ned", 100, 1024, 1024, 16)]
if os.environ.get("PROBE_ONLY"):
    configs = [c for c in configs if c[0] in os.environ["PROBE_ONLY"].split(",")]
ctxs = {}
for w in variants:
    os.environ["RTOW_TRACE_WAVES"] = str(w)
    ctxs[w] = rtow.Context(0)
for name, n, W, H, spp in configs:
    scene = rtow.Scene.build(name, n=n, image="synthetic")
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=1)
    res = {w: [] for w in variants}
    ref = None
    for w in variants:
        ctxs[w].upload(scene)
        b, _, _ = ctxs[w].render(cam, p, linear=False)  # warm
        if ref is None:
            ref = b
        assert (b == ref).all(), f"variant {w} differs"
    for r in range(rounds):
        for w in variants:
            _, _, st = ctxs[w].render(cam, p, linear=False)
            res[w].append((st.kernel_ms, st.segments))
    for w in variants:
        ms = min(k for k, _ in res[w])
        segs = res[w][0][1]
        print(f"{name} {W}x{H}x{spp} waves={w}: kernel {ms:.1f} ms  {segs / ms / 1e3:.1f} Mray/s", flush=True)
