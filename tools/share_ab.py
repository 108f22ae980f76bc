"""A/B one rank's share of a frame across builds (same process): python tools/_share_ab.py A.so B.so"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ab
import torch
torch.cuda.init()
libs = sys.argv[1:]
SCENE = os.environ.get("SA_SCENE", "final_ned")
W, H, SPP = [int(v) for v in os.environ.get("SA_FRAME", "4096,4096,8192").split(",")]
RANK, WORLD = [int(v) for v in os.environ.get("SA_RANK", "0,8").split(",")]
mods = [ab.load(f"rtow_{i}", l) for i, l in enumerate(libs)]
ctxs, scs = [], []
for m in mods:
    sc = m.Scene.build(SCENE, n=487 if SCENE == "random_ned" else 1, image="jpeg", image_path=ab.EARTH, scene_seed=1)
    c = m.Context(0)
    c.upload(sc)
    ctxs.append(c); scs.append(sc)
slab = torch.zeros(mods[0].rank_tile_count(W, H, RANK, WORLD) * 64 * 4, dtype=torch.uint8, device="cuda")
outs = [None] * len(mods)
for r in range(int(os.environ.get("SA_ROUNDS", "2"))):
    for i, (m, c) in enumerate(zip(mods, ctxs)):
        p = m.params(W, H, SPP, seed=1, rank=RANK, world=WORLD)
        st = c.render_tiles_device(m.camera_main(W, H), p, slab.data_ptr())
        torch.cuda.synchronize()
        cur = slab.cpu().numpy().copy()
        same = outs[i] is None or (cur == outs[i]).all()
        outs[i] = cur
        print(f"round {r} {os.path.basename(libs[i])}: {SCENE} {W}x{H}x{SPP} rank {RANK}/{WORLD}: kernel {st.kernel_ms:.1f} ms "
              f"{st.segments / st.kernel_ms / 1e3:.1f} Mray/s", flush=True)
print("identical across builds:", all((o == outs[0]).all() for o in outs))
