"""rtow_multi (include/rtow.h): several GPUs from one process -- device i
renders rank i of n (its 8x8 tiles into a slab, rtow_render_tiles_device), one
RCCL gather (ncclCommInitAll + grouped ncclSend/ncclRecv) to the first device,
which assembles the frame.  The reference's counterpart is its N worker
threads over a column interleave (main.cpp:182-195, 936).

The test box has one GPU.  With distinct devices that is n = 1: device 0's
slab still goes through RCCL (a send to itself), the assemble kernels run, and
the frame must equal rtow_render's bit for bit.  The n-rank code -- one host
thread per rank, the world-n slab offsets, the assembly -- runs with device 0
listed several times (ranks sharing it, gathered by device copies) and with k
contexts rendering ranks of world k at once; every rank chunks as the whole
frame (RTOW_FLAG_FRAME_PLAN), so those frames equal rtow_render's bit for bit
too.  n > 1 distinct devices (the RCCL gather between GPUs) is skipped below
two visible GPUs."""
import numpy as np
import pytest

import rtow

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scene,W,H,spp", [("random_ned", 61, 45, 8), ("cornell_smoke", 40, 24, 16),
                                           ("final_ned", 37, 23, 4)])
def test_multi_n1_equals_render_bitwise(scene, W, H, spp, gpu_ctx):
    sc = rtow.Scene.build(scene, n=100, image="synthetic")
    cam = rtow.camera_main(W, H)
    p = rtow.params(W, H, spp, seed=3)
    gpu_ctx.upload(sc)
    bgra, lin, st = gpu_ctx.render(cam, p)
    m = rtow.Multi([0])
    try:
        m.upload(sc)
        mb, ml, mst, dst = m.render(cam, p)
        assert np.array_equal(mb, bgra)
        assert np.array_equal(ml.view(np.uint32), lin.view(np.uint32))
        assert mst.segments == st.segments and mst.samples == st.samples == W * H * spp
        assert mst.pixels == W * H and len(dst) == 1 and dst[0].segments == st.segments
        assert mst.total_ms >= mst.kernel_ms > 0
        # again, at another size (buffers re-sized), BGRA only
        W2, H2 = 96, 54
        cam2, p2 = rtow.camera_main(W2, H2), rtow.params(W2, H2, 2, seed=4)
        mb2, none, _, _ = m.render(cam2, p2, linear=False)
        assert none is None
        ref2, _, _ = gpu_ctx.render(cam2, p2, linear=False)
        assert np.array_equal(mb2, ref2)
    finally:
        m.close()


def test_render_devices_one_call_and_bad_device(gpu_ctx):
    import ctypes

    L = rtow.lib()
    W, H, spp = 32, 18, 4
    sc = rtow.Scene.build("three_sphere")
    cam, p = rtow.camera_main(W, H), rtow.params(W, H, spp, seed=5)
    gpu_ctx.upload(sc)
    ref, _, _ = gpu_ctx.render(cam, p, linear=False)
    out = np.zeros((H, W, 4), np.uint8)
    st = rtow.Stats()
    devs = (ctypes.c_int * 1)(0)
    rc = L.rtow_render_devices(devs, 1, sc.view_ptr, ctypes.byref(cam), ctypes.byref(p), out.ctypes.data, None,
                               ctypes.byref(st))
    assert rc == rtow.OK, L.rtow_last_error()
    assert np.array_equal(out, ref) and st.samples == W * H * spp
    n = rtow.device_count()
    with pytest.raises(rtow.RtowError) as e:
        rtow.Multi([n])  # one past the last device
    assert e.value.code == rtow.E_INVALID


# ---- n > 1 on one GPU: several ranks share device 0 ---------------------------------------------
# The box has one GPU, so the multi-rank paths run with every rank on device 0:
# each rank its own rtow_context (stream, scene copy, buffers), all rendering at
# once from their own host threads -- the fan-out of rtow_multi_render -- then
# the gather (device copies; RCCL allows one rank per device) and the world-n
# assembly.  With RTOW_FLAG_FRAME_PLAN every rank chunks its samples as
# rtow_render does, so the frame must equal rtow_render's bit for bit (VERDICT
# r4 "what's weak" 4).

def _render_ranks(ctxs, cam, W, H, spp, world, seed, concurrent=True):
    """Ranks 0..world-1 of world (rank r on ctxs[r % len(ctxs)]), each
    rtow_render_tiles_device into its own device slab, from one host thread
    per rank when `concurrent`; returns (bgra slabs, linear slabs, stride, stats)."""
    import threading

    import torch

    stride = rtow.rank_tile_count(W, H, 0, world) * 64
    bgra = torch.zeros((world, stride * 4), dtype=torch.uint8, device="cuda")
    lin = torch.zeros((world, stride * 3), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    stats, errs = [None] * world, [None] * world

    def work(r):
        try:
            p = rtow.params(W, H, spp, seed=seed, rank=r, world=world, flags=rtow.FLAG_FRAME_PLAN)
            stats[r] = ctxs[r % len(ctxs)].render_tiles_device(cam, p, bgra[r].data_ptr(), lin[r].data_ptr())
        except Exception as e:  # noqa: BLE001 (re-raised below)
            errs[r] = e

    if concurrent:
        ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in ts)
    else:
        for r in range(world):
            work(r)
    for e in errs:
        if e is not None:
            raise e
    return bgra, lin, stride, stats


def _assemble(ctx, bgra, lin, stride, W, H, world):
    import torch

    fb = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    fl = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
    ctx.assemble_device(W, H, world, bgra.data_ptr(), stride, fb.data_ptr())
    ctx.assemble_linear_device(W, H, world, lin.data_ptr(), stride, fl.data_ptr())
    torch.cuda.synchronize()
    return fb.cpu().numpy(), fl.cpu().numpy()


@pytest.mark.parametrize("k", [2, 4])
def test_concurrent_contexts_on_one_device_assemble_to_render(k, gpu_ctx):
    """k contexts on device 0 render ranks 0..k-1 of world k from k host threads
    at once (rtow_multi_render's fan-out, rtow_multi.cpp), the slabs are
    assembled, and the frame equals rtow_render's bit for bit.  1920x1080x256
    of the random scene: here automatic chunking WOULD differ by world (64-
    sample items for the frame, 32 for a rank of 2), so the frame plan flag is
    what keeps the float chunk sums rtow_render's."""
    W, H, spp, seed = 1920, 1080, 256, 21
    whole = rtow.plan(rtow.params(W, H, spp))
    assert rtow.plan(rtow.params(W, H, spp, rank=0, world=k)).samples_per_chunk < whole.samples_per_chunk
    sc = rtow.Scene.build("random_ned", n=487, image="synthetic")
    cam = rtow.camera_main(W, H)
    gpu_ctx.upload(sc)
    ref_b, ref_l, ref_st = gpu_ctx.render(cam, rtow.params(W, H, spp, seed=seed))
    ctxs = [rtow.Context(0) for _ in range(k)]
    try:
        for c in ctxs:
            c.upload(sc)
        bgra, lin, stride, st = _render_ranks(ctxs, cam, W, H, spp, k, seed, concurrent=True)
        fb, fl = _assemble(ctxs[0], bgra, lin, stride, W, H, k)
    finally:
        for c in ctxs:
            c.close()
    assert sum(s.segments for s in st) == ref_st.segments
    assert sum(s.pixels for s in st) == W * H
    assert np.array_equal(fl.view(np.uint32), ref_l.view(np.uint32))
    assert np.array_equal(fb, ref_b)


@pytest.mark.parametrize("scene,W,H,spp", [("cornell_smoke", 203, 117, 64), ("final_ned", 61, 45, 16)])
def test_eight_ranks_on_one_gpu_assemble_to_render(scene, W, H, spp, gpu_ctx):
    """ranks 0..7 of world 8 rendered one after another with
    rtow_render_tiles_device, assembled by rtow_assemble_device and
    rtow_assemble_linear_device (ragged frames: partial edge tiles, unequal
    rank slabs), equal rtow_render's frame bit for bit."""
    sc = rtow.Scene.build(scene, n=1, image="synthetic")
    cam = rtow.camera_main(W, H)
    gpu_ctx.upload(sc)
    ref_b, ref_l, ref_st = gpu_ctx.render(cam, rtow.params(W, H, spp, seed=5))
    bgra, lin, stride, st = _render_ranks([gpu_ctx], cam, W, H, spp, 8, 5, concurrent=False)
    fb, fl = _assemble(gpu_ctx, bgra, lin, stride, W, H, 8)
    assert sum(s.segments for s in st) == ref_st.segments
    assert np.array_equal(fl.view(np.uint32), ref_l.view(np.uint32))
    assert np.array_equal(fb, ref_b)
    # the numpy mirror of the assembly agrees with the kernel
    assert np.array_equal(rtow.assemble(lin.cpu().numpy().reshape(8, stride, 3), W, H, 8), fl)


@pytest.mark.parametrize("k,scene,W,H,spp", [(2, "random_ned", 1920, 1080, 256), (3, "final_ned", 37, 23, 4),
                                             (8, "cornell", 96, 54, 16)])
def test_multi_ranks_sharing_device_equal_render(k, scene, W, H, spp, gpu_ctx):
    """rtow_multi with device 0 listed k times: k ranks, each its own context
    and stream on device 0, rendered at once by rtow_multi_render's host
    threads, gathered by device copies into the world-k slots, assembled on
    the first rank's context.  BGRA and linear frames equal rtow_render's."""
    sc = rtow.Scene.build(scene, n=487 if scene == "random_ned" else 1, image="synthetic")
    cam, p = rtow.camera_main(W, H), rtow.params(W, H, spp, seed=9)
    gpu_ctx.upload(sc)
    bgra, lin, st = gpu_ctx.render(cam, p)
    m = rtow.Multi([0] * k)
    try:
        m.upload(sc)
        mb, ml, mst, dst = m.render(cam, p)
    finally:
        m.close()
    assert np.array_equal(ml.view(np.uint32), lin.view(np.uint32))
    assert np.array_equal(mb, bgra)
    assert mst.segments == st.segments and mst.pixels == W * H and len(dst) == k
    assert sum(d.pixels for d in dst) == W * H
    assert max(d.kernel_ms for d in dst) == mst.kernel_ms


def test_multi_all_devices_equal_render(gpu_ctx):
    """rtow_multi over every visible device (distinct devices: the RCCL gather
    of rtow_multi.cpp, ncclCommInitAll + grouped ncclSend/ncclRecv): the frame
    equals one GPU's rtow_render bit for bit."""
    n = rtow.device_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs visible to one process")
    W, H, spp = 640, 360, 64
    sc = rtow.Scene.build("random_ned", n=487, image="synthetic")
    cam, p = rtow.camera_main(W, H), rtow.params(W, H, spp, seed=11)
    gpu_ctx.upload(sc)
    bgra, lin, st = gpu_ctx.render(cam, p)
    m = rtow.Multi(list(range(n)))
    try:
        m.upload(sc)
        mb, ml, mst, dst = m.render(cam, p)
    finally:
        m.close()
    assert np.array_equal(ml.view(np.uint32), lin.view(np.uint32)) and np.array_equal(mb, bgra)
    assert mst.segments == st.segments and len(dst) == n


def test_bench_multiprocess_ranks_sharing_the_gpu(tmp_path, gpu_ctx):
    """bench.py's own N > 1 path with the real kernels on the one-GPU box:
    `--gpus 2 --share-device` starts two rank processes (torch.distributed.run),
    both render their tile slabs on cuda:0 at the same time, the slabs are
    gathered (gloo through host memory: RCCL allows one rank per device) and
    rank 0 assembles the frame on the GPU.  With --frame-plan the dumped frame
    equals one GPU's rtow_render bit for bit, and the line's ray count equals
    that render's (the one-process-per-GPU path the driver times at N > 1,
    minus the RCCL gather)."""
    import json
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    W, H, spp = 320, 180, 16
    out = str(tmp_path / "frame.bgra")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--share-device", "--frame-plan",
           "--width", str(W), "--height", str(H), "--spp", str(spp), "--steps", "2", "--warmup", "1", "--no-cpu",
           "--dump-frame", out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][-1]
    print("share-device bench:", {k: line[k] for k in ("value", "n_gpus", "ranks", "rays_per_step", "rank_kernel_ms")})
    assert line["ranks"] == 2 and line["n_gpus"] == 1 and len(line["rank_kernel_ms"]["per_rank"]) == 2
    sc = rtow.Scene.build("random_ned", n=487, image="jpeg", scene_seed=1,  # the bench's earth texture
                          image_path=os.path.join(repo, "input_images", "1_earth_8k.jpg"))
    gpu_ctx.upload(sc)
    bgra, _, st = gpu_ctx.render(rtow.camera_main(W, H), rtow.params(W, H, spp, seed=1), linear=False)
    assert line["rays_per_step"] == st.segments
    assert np.array_equal(np.fromfile(out, np.uint8).reshape(H, W, 4), bgra)
