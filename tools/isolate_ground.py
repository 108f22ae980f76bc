"""Divergence hunt on final_ned's ground (BvhNode of 400 Boxes): variants of
that one item, GPU vs oracle; writes a diff image of the first variant."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

HIT_LIST, HIT_BOX = 9, 10
OUT = os.path.join(HERE, "..", "gpurun_out")


def copy(d):
    return {k: (v.copy() if hasattr(v, "copy") else v) for k, v in d.items()}


def with_items(d, lst, items):
    e = copy(d)
    e["hitables"][lst]["a"] = len(e["refs"])
    e["hitables"][lst]["b"] = len(items)
    e["refs"] = np.concatenate([e["refs"], np.array(items, np.uint32)])
    return e


def add_list(d, members):
    """append a HitableList hitable over `members`; returns (dict, its index)"""
    e = copy(d)
    h = np.zeros(1, dtype=sio.HITABLE)
    h[0]["kind"] = HIT_LIST
    h[0]["a"] = len(e["refs"])
    h[0]["b"] = len(members)
    e["refs"] = np.concatenate([e["refs"], np.array(members, np.uint32)])
    e["hitables"] = np.concatenate([e["hitables"], h])
    return e, len(e["hitables"]) - 1


def leaves(h, i):
    if h[i]["kind"] == sio.HIT_BVH_NODE:
        out = leaves(h, h[i]["a"])
        if h[i]["b"] != h[i]["a"]:
            out += leaves(h, h[i]["b"])
        return out
    return [int(i)]


def main():
    W, H, spp = 48, 48, 16
    d = sio.scene_dict(rtow.Scene.build("final_ned", image="synthetic"))
    h = d["hitables"]
    lst = int(h[d["root"]]["a"])
    first = int(h[lst]["a"])
    ground = int(d["refs"][first])
    boxes = leaves(h, ground)
    variants = [("bvh of 400 boxes", with_items(d, lst, [ground]))]
    e, L = add_list(d, boxes[:40])
    variants.append(("list of 40 boxes", with_items(e, lst, [L])))
    variants.append(("40 boxes at top level", with_items(d, lst, boxes[190:230])))
    # BvhNode subtrees of the ground tree by leaf count
    subs = {}
    for i in range(len(h)):
        if h[i]["kind"] == sio.HIT_BVH_NODE and i != ground:
            n = len(leaves(h, i))
            subs.setdefault(n, i)
    picks = [n for n in sorted(subs) if n >= 20]
    for n in picks[:: max(1, len(picks) // 8)]:
        variants.append((f"bvh subtree of {n} boxes", with_items(d, lst, [subs[n]])))
    root_l, root_r = int(h[ground]["a"]), int(h[ground]["b"])
    variants.append(("root left half", with_items(d, lst, [root_l])))
    variants.append(("root right half", with_items(d, lst, [root_r])))
    ctx = rtow.Context(0)
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=5)
    for k, (name, e) in enumerate(variants):
        sc = sio.ArrayScene(e)
        ctx.upload(sc)
        _, lin, st = ctx.render(cam, p)
        olin, _, oc = sio.oracle_render(sc.view_ptr, sio.RtowCamera.from_buffer_copy(bytes(cam)),
                                        sio.RtowParams.from_buffer_copy(bytes(p)))
        lin = lin.reshape(-1, 3).astype(np.float64)
        diff = np.abs(lin - olin).max(axis=1)
        rms = np.sqrt(np.mean((lin - olin) ** 2, axis=0))
        print(f"{name}: rms {rms} pixels>1e-3 {int((diff > 1e-3).sum())} segs gpu {st.segments} "
              f"oracle {oc.segments}", flush=True)
        if k == 0:
            np.save(os.path.join(OUT, "ground_gpu.npy"), lin.reshape(H, W, 3))
            np.save(os.path.join(OUT, "ground_oracle.npy"), olin.reshape(H, W, 3))


if __name__ == "__main__":
    main()
