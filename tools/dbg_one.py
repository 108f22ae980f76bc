import os, sys
HERE = os.path.join(os.environ["GRAFT_REPO_ROOT"], "tools")
sys.path[:0] = [HERE, os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow, scene_io as sio
from trace_diff import fmt
sc = rtow.Scene.build("cornell_smoke", image="synthetic")
ctx = rtow.Context(0); ctx.upload(sc)
W, H, spp = 64, 64, 4
cam, p = rtow.camera_main(W, H), rtow.params(W, H, spp, seed=1)
g = ctx.trace_sample(cam, p, 32, 32, 0)
o = sio.oracle_trace(sc.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)), sio.RtowParams.from_buffer_copy(bytes(p)), 32, 32, 0)
for i in range(max(len(g), len(o))):
    if i < len(g): print("gpu", i, fmt(g[i]))
    if i < len(o): print("ora", i, fmt(o[i]))
