"""One render of a config's scene (for PMC passes over the trace kernel of
another config than bench.py's): SCENE W H SPP; prints segments and time.
  rocprofv3 --pmc ... -- python3 tools/pmc_scene.py final_ned 1024 1024 64"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ray-tracing-one-weekend_amd"))
import rtow  # noqa: E402

scene, W, H, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
ctx = rtow.Context(0)
ctx.upload(rtow.Scene.build(scene, n=487, image="synthetic"))
_, _, st = ctx.render(rtow.camera_main(W, H), rtow.params(W, H, spp, seed=1), linear=False)
print(f"{scene} {W}x{H}x{spp}: segments {st.segments} kernel_ms {st.kernel_ms:.2f}", flush=True)
