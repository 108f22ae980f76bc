"""The instrumented trace kernel (RTOW_PROFILE=1: per-lane/per-wave step
counters and s_memtime split of wave cycles, printed by the library to
stderr) on a config's frame at reduced spp.
  python tools/prof_counters.py [SCENE] [SPP]"""
import os
import sys

os.environ["RTOW_PROFILE"] = "1"
HERE = os.path.dirname(os.path.abspath(__file__))
EARTH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "input_images", "1_earth_8k.jpg")  # the benched scenes' texture (scenes.h:140)
sys.path.insert(0, os.path.join(HERE, "..", "ray-tracing-one-weekend_amd"))
import rtow  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "random_ned"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 32
sizes = {"random_ned": (1920, 1080), "cornell": (800, 800), "cornell_smoke": (800, 800), "final_ned": (1024, 1024)}
W, H = sizes.get(scene, (1920, 1080))
ctx = rtow.Context(0)
ctx.upload(rtow.Scene.build(scene, n=487, image="jpeg", image_path=EARTH))
_, _, st = ctx.render(rtow.camera_main(W, H), rtow.params(W, H, spp, seed=1), linear=False)
print(f"{scene} {W}x{H}x{spp}: segments {st.segments} kernel {st.kernel_ms:.1f} ms", flush=True)
