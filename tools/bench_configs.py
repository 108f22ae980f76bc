"""Every BASELINE.json config at its full size on ONE MI355X (bench.py times
config 2 only, as the driver's contract asks): Mray/s and Msample/s of the
HIP path, next to the C oracle (the reference loop restated, kind "port") on
a bounded random pixel sample of the same frame.  Config 5 is quoted for
8 GPUs, so one GPU renders rank 0's share of the 8-rank tile split (the other
ranks' shares are the same size, interleaved tiles).

  python tools/bench_configs.py [--configs 1,2,3,4,5] [--out FILE] [--cpu-seconds S]
Writes one JSON line per config to stdout (and FILE).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
EARTH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "input_images", "1_earth_8k.jpg")  # the benched scenes' texture (scenes.h:140)
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "ray-tracing-one-weekend_amd")]
import rtow  # noqa: E402
import scene_io as sio  # noqa: E402

sys.path.insert(0, os.path.join(HERE, ".."))
import bench  # noqa: E402


def pmc_roofline(scene, W, H, segments, kernel_ms, src_hash, spp=None, world=1):
    """The VALU-issue roofline of this config's trace kernel (bench.py's
    definition), from the newest PMC summary of the same workload and frame
    size (profiles/*/pmc_summary.json, this build's source hash preferred).
    One number from one launch: when the summary profiled this
    very launch (same frame, spp and world), its VALU count per ray x this
    launch's rays / this launch's kernel time, as bench.py prices its line;
    otherwise (config 5: the summary is a 256-spp whole frame, this launch an
    8192-spp share) the summary's own launch -- its VALU count / its own kernel
    time -- with `pmc_config` naming that launch."""
    import glob

    best = None
    # (gpurun_out/prof_*: the summaries tools/round_check.sh wrote earlier in
    # the same GPU call, before they are copied into profiles/)
    for f in (glob.glob(os.path.join(HERE, "..", "profiles", "*", "pmc_summary.json")) +
              glob.glob(os.path.join(HERE, "..", "gpurun_out", "prof_*", "pmc_summary.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload", "random_ned") != scene or d.get("config", [0, 0])[:2] != [W, H]:
            continue
        if "SQ_INSTS_VALU" not in d:
            continue
        key = (d.get("source_hash") == src_hash, d.get("created", 0), os.path.getmtime(f))
        if best is None or key > best[0]:
            best = (key, f, d)
    if best is None:
        return None
    _, f, d = best
    vpr = d["SQ_INSTS_VALU"] / d["rays_per_launch"]
    same_launch = spp is not None and d.get("config", [None] * 5)[2] == spp and (d.get("config") + [1])[4] == world
    if same_launch or not d.get("kernel_ms_pmc"):
        achieved = vpr * segments / (kernel_ms * 1e-3) / 1e9
    else:
        achieved = d["SQ_INSTS_VALU"] / (d["kernel_ms_pmc"] * 1e-3) / 1e9
    lane = d["SQ_THREAD_CYCLES_VALU"] / (d["SQ_ACTIVE_INST_VALU"] * 64) if "SQ_THREAD_CYCLES_VALU" in d else None
    out = {"bound": "valu", "achieved": round(achieved, 1), "peak": bench.VALU_PEAK_G, "unit": "Gwave-instr/s",
           "frac": round(achieved / bench.VALU_PEAK_G, 4), "valu_per_ray": round(vpr, 3),
           "lane_util": round(lane, 4) if lane is not None else None,
           "useful_lane_frac": round(achieved / bench.VALU_PEAK_G * lane, 4) if lane is not None else None,
           "pmc": os.path.relpath(f, os.path.join(HERE, "..")), "pmc_config": d.get("config"),
           "priced_on": "this launch" if (same_launch or not d.get("kernel_ms_pmc")) else
                        "the PMC summary's own launch (pmc_config)",
           "pmc_matches_build": d.get("source_hash") == src_hash}
    if "WRITE_SIZE" in d:
        out["write_bytes_per_ray"] = round(d["WRITE_SIZE"] * 1024 / d["rays_per_launch"], 2)
    return out

CONFIGS = {
    1: ("three-sphere lambertian scene 200x100x8spp", "three_sphere", 0, 200, 100, 8, 1),
    2: ("book-1 random_scene (n=487) 1920x1080x1024spp", "random_ned", 487, 1920, 1080, 1024, 1),
    3: ("cornell_box 800x800x4096spp", "cornell", 0, 800, 800, 4096, 1),
    4: ("cornell_smoke 800x800x4096spp", "cornell_smoke", 0, 800, 800, 4096, 1),
    5: ("book-2 final_scene 4096x4096x8192spp over 8 GPUs (rank 0's share on this GPU)", "final_ned", 0, 4096,
        4096, 8192, 8),
}


def cpu_rate(scene, cam, W, H, spp, seconds, threads):
    """Oracle Mray/s on random pixels, sized from a short probe to ~`seconds`."""
    rng = np.random.default_rng(7)
    p = sio.default_params(W, H, spp, seed=1)
    ocam = sio.RtowCamera.from_buffer_copy(bytes(cam))
    n = 16
    while True:
        pix = rng.choice(W * H, size=min(n, W * H), replace=False).astype(np.uint32)
        t0 = time.perf_counter()
        _, _, c = sio.oracle_render(scene.view_ptr, ocam, p, pixels=pix, threads=threads)
        dt = time.perf_counter() - t0
        if dt >= seconds or n >= W * H:
            return {"value": round(c.segments / dt / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
                    "msample_per_s": round(c.samples / dt / 1e6, 4), "seconds": round(dt, 2),
                    "sample": f"{len(pix)} random pixels x {spp} spp of the same frame"}
        n = int(n * max(2.0, min(16.0, seconds / max(dt, 1e-3))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3,4,5")
    ap.add_argument("--out", default=None)
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    args = ap.parse_args()
    torch.cuda.init()
    threads, _ = rtow.host_threads()  # the CPUs this process may use (affinity, cgroup quota)
    ctx = rtow.Context(0)
    lines = []
    for k in [int(v) for v in args.configs.split(",")]:
        desc, name, n, W, H, spp, world = CONFIGS[k]
        scene = rtow.Scene.build(name, n=max(n, 1), image="jpeg", image_path=EARTH, scene_seed=1)  # as bench.py
        ctx.upload(scene)
        cam = rtow.camera_main(W, H)
        slab = torch.zeros(rtow.rank_tile_count(W, H, 0, world) * 64 * 4, dtype=torch.uint8, device="cuda")
        ctx.render_tiles_device(cam, rtow.params(W, H, 2, seed=1, rank=0, world=world), slab.data_ptr())  # warm
        p = rtow.params(W, H, spp, seed=1, rank=0, world=world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = ctx.render_tiles_device(cam, p, slab.data_ptr())
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        out = {"config": k, "workload": desc, "scene": name, "width": W, "height": H, "spp": spp,
               "ranks": world, "rank_rendered": 0, "pixels": st.pixels, "samples": st.samples,
               "segments": st.segments, "rays_per_sample": round(st.segments / max(st.samples, 1), 4),
               "seconds": round(wall, 3), "kernel_ms": round(st.kernel_ms, 2),
               "mray_per_s": round(st.segments / wall / 1e6, 2), "msample_per_s": round(st.samples / wall / 1e6, 3),
               "roofline": pmc_roofline(name, W, H, st.segments, st.kernel_ms, rtow.source_hash(), spp, world),
               "cpu_baseline": cpu_rate(scene, cam, W, H, spp, args.cpu_seconds, threads)}
        if world > 1:
            out["note"] = (f"one GPU rendered rank 0's 1/{world} share; {world} GPUs render the frame in about "
                           f"{wall:.1f} s")
        print(json.dumps(out), flush=True)
        lines.append(out)
    if args.out:
        with open(args.out, "w") as f:
            for o in lines:
                f.write(json.dumps(o) + "\n")
    ctx.close()


if __name__ == "__main__":
    main()
