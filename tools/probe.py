import sys, time
sys.path.insert(0, 'ray-tracing-one-weekend_amd')
import rtow, torch
torch.cuda.init()
ctx = rtow.Context(0)
for name, n, W, H, spp in [("random_ned", 487, 1920, 1080, 16), ("cornell", 100, 800, 800, 64)]:
    s = rtow.Scene.build(name, n=n, image="synthetic")
    ctx.upload(s)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=1)
    ctx.render(cam, p, linear=False)
    t = time.time(); b, l, st = ctx.render(cam, p, linear=False); dt = time.time() - t
    print(f"{name} {W}x{H}x{spp}: kernel {st.kernel_ms:.1f} ms resolve {st.resolve_ms:.2f} ms total {st.total_ms:.1f} ms "
          f"segments {st.segments} -> {st.segments/st.kernel_ms/1e3:.1f} Mray/s {st.samples/st.kernel_ms/1e3:.1f} Msample/s", flush=True)
