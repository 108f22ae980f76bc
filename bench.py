#!/usr/bin/env python3
"""Benchmark: BASELINE.json config 2 -- the book-1 random scene
(randomScene_NED with n = 487, 488 hitables under one BvhNode) at
1920x1080x1024spp, depth 50, on N MI355X.

One step = one full frame: every rank renders its share of the frame's 8x8
tiles (rank r takes tiles r, r+N, ...) with the HIP path in librtow_hip.so,
then one RCCL gather (torch.distributed, backend "nccl") brings the tile
slabs to rank 0, which assembles the BGRA frame on its GPU.  Total work is
the fixed frame, so scaling is "strong".

  python bench.py [--gpus N] [--steps K] [--warmup W] [--spp S] [--no-cpu]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Rank 0 prints ONE JSON line (value = whole-job Mray/s; Msample/s beside it).

roofline: the bound that limits this kernel is VALU issue, not HBM (the scene
is LDS/L2-resident; measured HBM traffic is ~7 GB/s).  achieved = VALU
wave-instructions per second of the trace kernel = (wave-instructions per ray,
SQ_INSTS_VALU from the committed rocprofv3 PMC pass of this exact build and
config, profiles/<round>_*/pmc_summary.json) x the rays this launch traced /
the kernel's mean duration from HIP events on the render stream.  peak = 1024
SIMDs x 2.4 GHz x 0.5 (a wave64 VALU instruction occupies a SIMD-32 for two
cycles, MI355X_MICROARCH.md).  lane_util = the active-lane fraction of those
instructions (SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64), calibrated on
gfx950 by tools/valu_calib.hip), so frac x lane_util is the useful-lane share
of the chip's VALU throughput.  The measured HBM bytes (FETCH_SIZE x 2 +
WRITE_SIZE of the same PMC run) and the reference-equivalent record bytes per
ray are informational fields.  cpu_baseline = the reference's
own code (oracle/_ref/ref_harness) on all the host cores this process may use
over a bounded random pixel sample, rays counted by the C oracle on the same
pixels (the oracle alone, kind "port", when the harness was not built).
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-one-weekend_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMD-32, a wave64 VALU instruction takes two
# cycles of its SIMD, 2.4 GHz max clock (MI355X_MICROARCH.md) -> G wave-instr/s
N_SIMD, CLOCK_GHZ = 1024, 2.4
VALU_PEAK_G = N_SIMD * CLOCK_GHZ * 0.5
# algorithmic record bytes per reference traversal event
BYTES_BVH, BYTES_SPHERE, BYTES_MSPHERE, BYTES_RECT, BYTES_MEDIUM = 32, 20, 40, 24, 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--n", type=int, default=487)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-pixels", type=int, default=40000)
    ap.add_argument("--cpu-spp", type=int, default=1024)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-kind", choices=["auto", "port"], default="auto",
                    help="auto: the reference's own code when oracle/_ref was built, else the oracle")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every host CPU this process may use")
    ap.add_argument("--pmc-json", default=None,
                    help="PMC summary to use (default: the newest profiles/*/pmc_summary.json of this build+config)")
    return ap.parse_args()


def reference_run(pix, args, threads):
    """The reference's own code (oracle/_ref/ref_harness, compiled from
    /root/reference's headers in the build container; its render loop body is
    main.cpp:938-951) on the same pixels: (seconds, checksum) or None when the
    harness was not built.  The random scene loads its earth texture from
    ./input_images/1_earth_8k.jpg (scenes.h:140): the synthetic texture the GPU
    uses is staged there as a lossless PNG."""
    import subprocess
    import tempfile

    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.access(harness, os.X_OK):
        return None
    try:
        from PIL import Image

        import rtow
    except ImportError:
        return None
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "input_images"))
        Image.fromarray(rtow.synthetic_image(2048, 1024), "RGB").save(
            os.path.join(d, "input_images", "1_earth_8k.jpg"), format="PNG")
        pf = os.path.join(d, "pix.u32")
        pix.tofile(pf)
        env = dict(os.environ, RTOW_SCENE_SEED="1")
        out = subprocess.run([harness, "bench", "random_ned", str(args.width), str(args.height), str(args.cpu_spp), pf,
                              "--n", str(args.n), "--seed", str(args.seed), "--threads", str(threads), "--cwd", d],
                             env=env, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return None
    r = json.loads(out.stdout.strip().splitlines()[-1])
    return r["seconds"], r["checksum"]


def find_pmc(args, world, src_hash):
    """The PMC summary (tools/profile_bench.sh) that describes this run: the
    newest one under profiles/ recorded for this config and this build's
    source hash; failing that the newest for this config, flagged stale."""
    import glob

    cands = [args.pmc_json] if args.pmc_json else sorted(glob.glob(os.path.join(REPO, "profiles", "*", "pmc_summary.json")))
    want = [args.width, args.height, args.spp, args.n, world]
    fresh, stale = None, None
    for f in cands:
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config") != want or "SQ_INSTS_VALU" not in d:
            continue
        if d.get("source_hash") == src_hash:
            fresh = (f, d)
        else:
            stale = (f, d)
    return fresh or stale


def roofline(args, world, launch_rays, mean_kms, bpr, src_hash):
    """VALU-issue roofline of the trace kernel (see the module docstring)."""
    found = find_pmc(args, world, src_hash)
    if found is None:
        return {"bound": "valu", "achieved": None, "peak": VALU_PEAK_G, "unit": "Gwave-instr/s", "frac": None,
                "traffic": None, "kernel_ms": round(mean_kms, 2), "note": "no PMC summary for this config under profiles/"}
    path, d = found
    rays_pmc = d["rays_per_launch"]
    valu_per_ray = d["SQ_INSTS_VALU"] / rays_pmc
    achieved = valu_per_ray * launch_rays / (mean_kms * 1e-3) / 1e9
    lane_util = d["SQ_THREAD_CYCLES_VALU"] / (d["SQ_ACTIVE_INST_VALU"] * 64) if "SQ_THREAD_CYCLES_VALU" in d else None
    traffic = None
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:  # KB; FETCH_SIZE reads half the bytes on gfx950
        traffic = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024 / rays_pmc * launch_rays
    frac = achieved / VALU_PEAK_G
    roof = {"bound": "valu", "achieved": round(achieved, 1), "peak": VALU_PEAK_G, "unit": "Gwave-instr/s",
            "frac": round(frac, 4),
            "lane_util": round(lane_util, 4) if lane_util is not None else None,
            "useful_lane_frac": round(frac * lane_util, 4) if lane_util is not None else None,
            "traffic": round(traffic) if traffic is not None else None,
            "valu_per_ray": round(valu_per_ray, 3), "kernel_ms": round(mean_kms, 2),
            "pmc": os.path.relpath(path, REPO), "pmc_source_hash": d.get("source_hash"),
            "pmc_matches_build": d.get("source_hash") == src_hash,
            "peak_def": f"{N_SIMD} SIMD-32 x {CLOCK_GHZ} GHz x 0.5 wave64 VALU instr/cycle"}
    if "GRBM_GUI_ACTIVE" in d and d.get("kernel_ms_pmc"):
        roof["clock_ghz_under_pmc"] = round(d["GRBM_GUI_ACTIVE"] / 8 / (d["kernel_ms_pmc"] * 1e-3) / 1e9, 3)
    if traffic is not None:
        roof["hbm_gbps"] = round(traffic / (mean_kms * 1e-3) / 1e9, 2)
        roof["hbm_frac"] = round(traffic / (mean_kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5)
    if bpr is not None:
        roof["reference_bytes_per_ray"] = round(bpr, 1)
        roof["reference_equiv_gbps"] = round(bpr * launch_rays / (mean_kms * 1e-3) / 1e9, 1)
    return roof


def cpu_baseline(scene, cam, args, threads):
    """The CPU render of a bounded random pixel sample of the same frame: the
    reference's own code (kind "reference", oracle/_ref) when it was built, the
    oracle otherwise (kind "port": the reference's render loop restated in C,
    bit-exact with the reference build).  The oracle always runs: its traversal
    counts give the ray count (the same paths: the two agree bit for bit, and
    the checksum of the pixel sums shows it) and bytes/ray."""
    import scene_io as sio

    rng = np.random.default_rng(1234)
    W, H = args.width, args.height
    pix = rng.choice(W * H, size=min(args.cpu_pixels, W * H), replace=False).astype(np.uint32)
    ocam = sio.RtowCamera.from_buffer_copy(bytes(cam))
    p = sio.default_params(W, H, args.cpu_spp, seed=args.seed)
    t0 = time.perf_counter()
    lin, _, c = sio.oracle_render(scene.view_ptr, ocam, p, pixels=pix, threads=threads)
    dt = time.perf_counter() - t0
    bytes_per_ray = (c.bvh_visits * BYTES_BVH + c.sphere_tests * BYTES_SPHERE + c.moving_sphere_tests * BYTES_MSPHERE
                     + c.rect_tests * BYTES_RECT + c.medium_calls * BYTES_MEDIUM) / max(c.segments, 1)
    sample = f"{len(pix)} random pixels of the {W}x{H} frame x {args.cpu_spp} spp (same scene/seed), {threads} threads"
    port = {"value": round(c.segments / dt / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "msample_per_s": round(c.samples / dt / 1e6, 4), "seconds": round(dt, 2),
            "sample": sample + ", oracle/librtow_oracle.so"}
    base = port
    ref = reference_run(pix, args, threads) if args.cpu_kind != "port" else None
    if ref is not None:
        rs, checksum = ref
        osum = float(lin.astype(np.float64).sum())
        base = {"value": round(c.segments / rs / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "reference",
                "msample_per_s": round(c.samples / rs / 1e6, 4), "seconds": round(rs, 2),
                "sample": sample + ", oracle/_ref/ref_harness (the reference's headers); rays counted by the oracle",
                "same_result_as_oracle": bool(abs(checksum - osum) <= 1e-6 * max(1.0, abs(osum))),
                "port": {k: port[k] for k in ("value", "msample_per_s", "seconds")}}
    counts = {"segments_per_sample": c.segments / max(c.samples, 1),
              "bvh_visits_per_ray": c.bvh_visits / max(c.segments, 1),
              "sphere_tests_per_ray": c.sphere_tests / max(c.segments, 1),
              "moving_sphere_tests_per_ray": c.moving_sphere_tests / max(c.segments, 1)}
    return base, bytes_per_ray, counts


def frame_step(render, assemble, slab, gathered, rank, world, dist=None):
    """One bench step: this rank renders its 8x8-tile slab (`render(slab)`),
    one gather brings every rank's slab to rank 0 (torch.distributed: RCCL
    over xGMI on the GPUs, gloo in tests/test_distributed.py), rank 0
    assembles the frame (`assemble(gathered)`).  Returns render's stats."""
    st = render(slab)
    if world > 1:
        dist.gather(slab, list(gathered.unbind(0)) if rank == 0 else None, dst=0)
    else:
        gathered[0].copy_(slab)
    if rank == 0:
        assemble(gathered)
    return st


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import rtow

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"# note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    distributed = world > 1
    if distributed:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if distributed:
            dist.barrier()

    W, H, spp = args.width, args.height, args.spp
    scene = rtow.Scene.build("random_ned", n=args.n, image="synthetic", scene_seed=1)
    cam = rtow.camera_main(W, H)
    ctx = rtow.Context(local)
    ctx.upload(scene)
    stride = rtow.rank_tile_count(W, H, 0, world) * 64  # rank 0 holds the most tiles
    slab = torch.zeros(stride * 4, dtype=torch.uint8, device="cuda")
    gathered = torch.zeros((world, stride * 4), dtype=torch.uint8, device="cuda") if rank == 0 else None
    frame = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") if rank == 0 else None
    stream = torch.cuda.current_stream().cuda_stream
    p = rtow.params(W, H, spp, seed=args.seed, rank=rank, world=world)

    def step():
        return frame_step(lambda sl: ctx.render_tiles_device(cam, p, sl.data_ptr(), None, stream),
                          lambda g: ctx.assemble_device(W, H, world, g.data_ptr(), stride, frame.data_ptr(), stream),
                          slab, gathered, rank, world, dist)

    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    segs, samples, kms = 0, 0, []
    for _ in range(args.steps):
        st = step()
        segs += st.segments
        samples += st.samples
        kms.append(st.kernel_ms)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    tot = torch.tensor([float(segs), float(samples)], dtype=torch.float64, device="cuda")
    el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if distributed:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    segs_all, samples_all, elapsed = float(tot[0]), float(tot[1]), float(el[0])

    if rank == 0:
        threads, cpu_info = rtow.host_threads()
        if args.cpu_threads:
            threads = args.cpu_threads
        if args.no_cpu:
            base, bpr, counts = None, None, {}
        elif world == 1:
            base, bpr, counts = cpu_baseline(scene, cam, args, threads)
            base.update(cpu_info)
        else:  # the CPU baseline is quoted at N=1 only; bytes/ray from a smaller oracle sample
            args.cpu_pixels = max(1, args.cpu_pixels // 10)
            args.cpu_kind = "port"
            _, bpr, counts = cpu_baseline(scene, cam, args, threads)
            base = None
        mean_kms = float(np.mean(kms))
        launch_rays = segs / max(args.steps, 1)
        roof = roofline(args, world, launch_rays, mean_kms, bpr, rtow.source_hash())
        out = {
            "metric": "Mray/s + Msample/s, random_scene 1920×1080×1024spp at 1/2/4/8 MI355X",
            "value": round(segs_all / elapsed / 1e6, 2),
            "unit": "Mray/s",
            "msample_per_s": round(samples_all / elapsed / 1e6, 3),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"randomScene_NED n={args.n} ({args.n + 1} hitables under one BvhNode), "
                                   f"{W}x{H}x{spp}spp, depth 50, synthetic 2048x1024 earth texture",
                       "width": W, "height": H, "spp": spp, "n": args.n, "scene_seed": 1, "render_seed": args.seed,
                       "parallelism": f"tiles8x8 interleaved over {world} rank(s) + RCCL gather to rank 0"},
            "rays_per_sample": round(segs_all / max(samples_all, 1), 4),
            "rays_per_step": int(segs_all / max(args.steps, 1)),
            "roofline": roof,
            "cpu_baseline": base,
            "oracle_counts": {k: round(v, 3) for k, v in counts.items()},
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
