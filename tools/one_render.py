"""One render on cuda:0, timing and segment count, next to the oracle's count
for small frames.  python tools/one_render.py SCENE W H SPP  (RTOW_N: random-scene sphere count, default 487)"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

sc = rtow.Scene.build(sys.argv[1], n=int(os.environ.get("RTOW_N", "487")), image="synthetic")
ctx = rtow.Context(0)
ctx.upload(sc)
W, H, spp = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
cam, p = rtow.camera_main(W, H), rtow.params(W, H, spp, seed=1)
t = time.time()
_, _, st = ctx.render(cam, p, linear=False)
line = f"{sys.argv[1:]} kernel_ms {st.kernel_ms:.2f} segments {st.segments} wall {time.time() - t:.3f}"
if W * H * spp <= 1 << 16:
    _, _, oc = sio.oracle_render(sc.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                 sio.RtowParams.from_buffer_copy(bytes(p)))
    line += f" oracle segments {oc.segments}"
print(line, flush=True)
