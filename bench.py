#!/usr/bin/env python3
"""bench.py — Msamples/s of the HIP path-tracing hot path (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W] [--config C2|C3|C4|C5]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU)

A step renders one full frame of the workload (every pixel x every stratum x up
to 8 bounces).  With N ranks (default --shard tiles) tile t of the frame is
rendered by rank t % N in stratum-chunked work units and one RCCL gather over
xGMI brings the compact tile sums to rank 0; --shard strata splits the strata
instead and combines full-frame sums with an RCCL reduce(sum).  Strong scaling:
the frame is fixed, N varies.

Output: ONE JSON line on rank 0 (driver contract) with a roofline object (the
render kernel's algorithmic bytes / HIP-event duration vs HBM peak), a "valu"
object (the kernel's real ceiling: fp64 FLOP/s and VALU issue occupancy from the
committed PMC pass, profiles/pmc_<config>.json) and a CPU baseline (the
reference's own code on the host cores, bounded sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "real-time-ray-tracing-engine_amd")
sys.path.insert(0, PKG)

BASELINE = json.load(open(os.path.join(ROOT, "BASELINE.json")))
SCENES = os.path.join(PKG, "scenes")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
F64_PEAK_TFS = 78.6    # MI355X fp64 vector peak (AMD spec): 16 FMA lanes/clk/SIMD at 2.4 GHz

# BASELINE.json configs
CONFIGS = {
    "C1": ("three_spheres", 400, 10, 8),
    "C2": ("three_spheres", 1920, 64, 8),
    "C3": ("bouncing_seed42", 1920, 256, 8),
    "C4": ("cornell_fog", 1920, 1024, 8),
    "C5": ("bouncing_seed42", 3840, 4096, 8),
}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def algorithmic_bytes(st, info, n_pixels):
    """Bytes the kernel must fetch/store per launch under the device layout
    (SURVEY §8d formula): node fetches x node size + primitive tests x (item +
    primitive record) + medium tests x (item + medium + boundary records) +
    light-pdf primitive tests x (light leaf + record) + material/texture per
    shading event + the fp64 accumulator store per pixel."""
    item, light_leaf, mat_tex = 32, 48, 96
    b = st["node_visits"] * info["node_bytes"]
    b += st["sphere_tests"] * (item + info["sphere_bytes"])
    b += st["quad_tests"] * (item + info["quad_bytes"])
    b += st["other_tests"] * (item + 1024)  # medium: record + boundary items
    b += st["light_tests"] * (light_leaf + info["quad_bytes"])
    b += st["shade_events"] * mat_tex
    b += n_pixels * 24
    return b


def cpu_baseline(scene, cam_full, threads):
    """The reference's own C++ path (oracle/_ref, built from /root/reference/src)
    with its -p decomposition over `threads` host threads, on a bounded sample:
    the full frame at 5x5 strata (same scene, depth, resolution; ~15 s)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    from rtx.scene import camera_desc  # noqa: F401
    spp = 25
    cam = scene.camera_desc(image_width=cam_full.image_width, samples_per_pixel=spp,
                            max_depth=cam_full.max_depth)
    if O.ref_available():
        t = time.time()
        n, _ = O.ref_trace_parallel(scene, cam, threads)
        dt = time.time() - t
        kind = "reference"
    else:  # reference build absent: the oracle restatement, same decomposition
        t = time.time()
        O.oracle_render(scene, cam, O.MODE_COUNTER, 1, threads=threads)
        dt = time.time() - t
        n = cam.image_width * max(1, int(cam.image_width / cam.aspect_ratio)) * spp
        kind = "port"
    return {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": kind,
            "sample": "%dx%d @ %d spp, depth %d, %s, %.1f s" % (
                cam.image_width, max(1, int(cam.image_width / cam.aspect_ratio)), spp,
                cam.max_depth, scene_name_of(scene), dt)}


def scene_name_of(scene):
    return getattr(scene, "_name", "scene")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    # rehearsal of the N>1 path on one GPU: every rank on cuda:0, gloo all_reduce
    # instead of RCCL reduce (the driver's 8-GPU runs use the defaults)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--share-device", action="store_true")
    ap.add_argument("--shard", default="tiles", choices=["tiles", "strata"],
                    help="N>1: tiles round-robin + gather (default) or strata + reduce")
    ap.add_argument("--n1-layout", default="frame", choices=["frame", "tiles"],
                    help="N=1: render straight into the frame (default) or in 8x8 tile "
                         "work units + chunk sum + tile->frame reorder, as the N>1 path")
    ap.add_argument("--check", action="store_true",
                    help="rank 0 compares the reduced frame with a 1-device render")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    import torch
    from rtx import abi
    from rtx.render import Renderer, camera_frame
    from rtx.scene import load_scene

    if ws != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, ws), file=sys.stderr)
    if args.share_device:
        local = 0
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if ws > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    name, width, spp, depth = CONFIGS[args.config]
    width = args.width or width
    spp = args.spp or spp
    scene = load_scene(os.path.join(SCENES, name + ".json"))
    scene._name = name
    cam = scene.camera_desc(image_width=width, samples_per_pixel=spp, max_depth=depth)
    frame = camera_frame(cam)
    W, H, sq = frame.image_width, frame.image_height, frame.sqrt_spp
    n_strata = sq * sq
    s0 = rank * n_strata // ws
    s1 = (rank + 1) * n_strata // ws
    tiles_mode = (ws > 1 and args.shard == "tiles") or (ws == 1 and args.n1_layout == "tiles")

    from rtx.dist import ShardedRenderer, TileShardedRenderer, max_over_ranks
    R = Renderer(scene, device=local)
    info = R.info()
    stream = torch.cuda.current_stream(dev)  # the null stream: ordered with RCCL's waits

    def render_fn(fr, acc, seed, strata):
        # overwrite the partial sums (no memset, no read-modify-write)
        R.render_device(fr, acc.data_ptr(), stream.cuda_stream, seed=seed, samples=strata,
                        output=abi.RT_OUT_SUM, accumulate=0)

    def tile_render_fn(fr, buf, seed, tiles, chunks):
        R.render_device(fr, buf.data_ptr(), stream.cuda_stream, seed=seed, samples=(0, -1),
                        output=abi.RT_OUT_SUM, accumulate=0, tiles=tiles,
                        layout=abi.RT_LAYOUT_TILES, chunks=chunks)

    if tiles_mode:
        shard = TileShardedRenderer(tile_render_fn, frame, rank, ws)
        bufs = [shard.buffer(dev) for _ in range(2)]
        gath = [shard.gather_buffer(dev) if rank == 0 else None for _ in range(2)]
        tsum = [None, None]  # per-tile sums (chunk sum) of each buffer

        def launch_work(seed, b):
            tsum[b] = shard.render(bufs[b], seed)
    else:
        shard = ShardedRenderer(render_fn, frame, rank, ws)
        assert shard.strata == (s0, s1)
        bufs = [torch.zeros((H, W, 3), dtype=torch.float64, device=dev) for _ in range(2)]
        launch_work = lambda seed, b: render_fn(frame, bufs[b], seed, (s0, s1 - s0))  # noqa: E731
    final = {}      # rank 0: the last completed frame's raw sums, by step
    inflight = []   # (step, buffer, work handle) in step order
    kernel_ms = []

    def complete(k, b, work):
        if work is not None:
            work.wait()
        if rank == 0:
            if tiles_mode:
                # reorder the gathered tiles (N=1: this rank's own tile sums)
                final["frame"] = shard.frame_sums(gath[b] if ws > 1 else tsum[b].unsqueeze(0))
            else:
                final["frame"] = bufs[b]
            final["step"] = k

    def exchange(b):
        if ws == 1:
            return None
        if tiles_mode:
            if args.backend == "nccl":
                return shard.gather(tsum[b], gath[b], async_op=True)
            torch.cuda.synchronize(dev)  # gloo: host-staged, no CUDA gather
            cpu = tsum[b].cpu()
            parts = [torch.empty_like(cpu) for _ in range(ws)] if rank == 0 else None
            dist.gather(cpu, gather_list=parts, dst=0)
            if rank == 0:
                gath[b].copy_(torch.stack(parts))
            return None
        if args.backend == "nccl":
            return dist.reduce(bufs[b], dst=0, op=dist.ReduceOp.SUM, async_op=True)
        torch.cuda.synchronize(dev)  # gloo has no CUDA reduce
        return dist.all_reduce(bufs[b], op=dist.ReduceOp.SUM, async_op=True)

    def step(k, seed):
        b = k % 2
        while inflight and inflight[0][1] == b:  # this buffer's exchange (step k-2) first
            complete(*inflight.pop(0))
        launch_work(seed, b)
        inflight.append((k, b, exchange(b)))

    def drain():
        while inflight:
            complete(*inflight.pop(0))

    for w in range(args.warmup):
        step(w, 1000 + w)
    drain()
    torch.cuda.synchronize(dev)

    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, k)
        if ws == 1:
            kernel_ms.append(R.last_kernel_ms())  # HIP events around the kernel, launch stream
    drain()
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    check = None
    if args.check and rank == 0:  # the last timed frame on rank 0 vs one device, all strata
        assert final["step"] == args.steps - 1
        last = final["frame"].clone()
        ref = torch.empty_like(last)
        render_fn(frame, ref, args.steps - 1, (0, n_strata))
        torch.cuda.synchronize(dev)
        err = (last - ref).abs().max().item()
        scale = max(1.0, ref.abs().max().item())
        check = {"max_abs_diff": err, "ok": bool(err <= 1e-9 * scale)}

    if ws > 1:  # kernel time measured after the timed region (no sync inside it)
        for k in range(min(2, args.steps)):
            launch_work(5000 + k, 0)
            kernel_ms.append(R.last_kernel_ms())

    samples_per_step = W * H * n_strata  # whole frame, all ranks together
    value = samples_per_step * args.steps / elapsed / 1e6

    # roofline of the dominant (render) kernel on this rank, one launch
    if tiles_mode:
        st = R.stats(frame, seed=0, tiles=(rank, ws), layout=abi.RT_LAYOUT_TILES,
                     chunks=shard.chunks)
    else:
        st = R.stats(frame, seed=0, samples=(s0, s1 - s0))
    px_launch = shard.tiles_per_rank * shard.chunks * 64 if tiles_mode else W * H
    bytes_launch = algorithmic_bytes(st, info, px_launch)
    avg_ms = sum(kernel_ms) / len(kernel_ms)
    achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
    traffic = None
    pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            traffic = pmc.get("hbm_bytes_per_launch")
        except Exception:
            pmc = {}
    valu = None
    if pmc.get("f64_flops_per_launch") and ws == 1:
        # fp64 work per launch is a property of the workload (PMC pass on the same
        # command); divided by this run's live HIP-event kernel time
        tfs = pmc["f64_flops_per_launch"] / (avg_ms * 1e-3) / 1e12
        valu = {"bound": "valu_f64", "achieved": round(tfs, 3), "peak": F64_PEAK_TFS,
                "unit": "TFLOP/s", "frac": round(tfs / F64_PEAK_TFS, 4),
                "valu_busy": pmc.get("valu_busy"),
                "valu_insts_per_launch": pmc.get("valu_insts_per_launch"),
                "f64_insts_per_launch": pmc.get("f64_insts_per_launch"),
                "note": "f64 FLOP = 64 x (ADD+MUL+TRANS) + 128 x FMA wave-instructions "
                        "(PMC, every lane counted); valu_busy = SQ_ACTIVE_INST_VALU x 4 / "
                        "(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the share of SIMD cycles "
                        "issuing VALU — the bound this kernel runs against"}

    out = {
        "metric": BASELINE["metric"],
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: JSON scene %s, seeded Philox sample stream" % name,
        "config": {"workload": "%s %s %dx%d spp%d depth%d" % (args.config, name, W, H, n_strata, depth),
                   "scene": name, "width": W, "height": H, "spp": n_strata, "max_depth": depth,
                   "parallelism": (("1 GPU, tile work units x%d chunks" % shard.chunks
                                    if tiles_mode else "1 GPU") if ws == 1 else
                                   "tile-shard x%d (tile t on rank t %% %d, %d stratum chunks) + %s gather" % (
                                       ws, ws, shard.chunks,
                                       "RCCL" if args.backend == "nccl" else "gloo")
                                   if tiles_mode else
                                   "stratum-shard x%d + %s reduce(sum)" % (
                                       ws, "RCCL" if args.backend == "nccl" else "gloo"))},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                     "traffic": traffic, "kernel_ms": round(avg_ms, 3),
                     "note": "achieved = SURVEY 8d algorithmic bytes / kernel time; the scene "
                             "is L1/L2-resident, so it can exceed HBM peak; traffic = PMC "
                             "FETCH_SIZE x2 + WRITE_SIZE per launch (the accumulator)",
                     "bytes_per_launch": int(bytes_launch),
                     "bytes_per_sample": round(bytes_launch / max(1, st["samples"]), 1),
                     "counters": st},
    }
    if valu is not None:
        out["valu"] = valu
    if check is not None:
        out["check"] = check
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(scene, cam, min(args.cpu_threads, os.cpu_count() or 1))
    if rank == 0:
        print(json.dumps(out), flush=True)
    R.close()
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
