"""The tie_bvh_entry fixture on the GPU against the reference's golden frame:
per-channel RMS, the share of differing pixels (quantised) and where they
lie (diagnostic for tests/test_tie_entry.py)."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

c = {x["name"]: x for x in json.load(open(os.path.join(sio.GOLDEN, "manifest_extra.json")))["cases"]}["tie_bvh_entry"]
W, H = c["width"], c["height"]
world = sio.ArrayScene(sio.load_scene(os.path.join(sio.GOLDEN, "tie_bvh_entry.scn")))
ctx = rtow.Context(0)
ctx.upload(world)
bgra, lin, st = ctx.render(rtow.camera_main(W, H), rtow.params(W, H, c["spp"], seed=c["seed"]))
glin, gbgra = sio.golden_image("tie_bvh_entry", W, H)
rms = np.sqrt(np.mean((lin.astype(np.float64) - glin) ** 2, axis=(0, 1)))
diff = np.any(bgra != gbgra, axis=-1)
print(json.dumps({"rms": rms.tolist(), "bgra_differ_frac": float(diff.mean()), "segments": int(st.segments),
                  "max_abs": float(np.abs(lin - glin).max())}))
for y in range(0, H, 3):
    print("".join("X" if diff[y, x] else "." for x in range(W)))
