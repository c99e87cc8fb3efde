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

Output: ONE JSON line on rank 0 (driver contract) with
  * a roofline object for the render kernel: bound "valu" (the kernel issues
    vector instructions most cycles; the scene is cache/LDS-resident), frac =
    VALU-busy from rocprofv3 PMC passes that bench.py runs on this build and
    workload before the timed run; physical HBM bytes per launch (traffic) and
    GB/s, fp64 TFLOP/s, and SURVEY §8(d)'s algorithmic bytes as the
    cache-served figure beside it;
  * a CPU baseline: the reference's own StaticCamera::render -p (ThreadPool of
    hardware_concurrency() workers) on the host cores, bounded sample.
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


PMC_PASSES = {  # one rocprofv3 --pmc run each (TCC slots: FETCH_SIZE 3, WRITE_SIZE 2 of 4)
    "valu": ["SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
             "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64", "GRBM_GUI_ACTIVE"],
    "fetch": ["FETCH_SIZE"],
    "write": ["WRITE_SIZE"],
}


def pmc_counters(path_glob_root, kernel_tag="render_tiles<false"):
    """Per-launch averages of every counter in the rocprofv3 counter-collection
    CSVs under `path_glob_root`, over the render kernel's plain instance."""
    import csv
    import glob
    sums, counts = {}, {}
    for f in glob.glob(os.path.join(path_glob_root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel_tag not in r.get("Kernel_Name", ""):
                continue
            k = r["Counter_Name"]
            sums[k] = sums.get(k, 0.0) + float(r["Counter_Value"])
            counts[k] = counts.get(k, 0) + 1
    return {k: sums[k] / counts[k] for k in sums}, max(counts.values()) if counts else 0


def pmc_live(args):
    """rocprofv3 PMC passes over THIS build and workload, run by bench.py itself
    before it touches the GPU (each pass: a child `bench.py --pmc off` of the
    same config, 1 warmup + 2 steps; counters averaged over the plain render
    kernel's launches).  Returns the summary dict or None (no rocprofv3 / a pass
    failed: the caller falls back to the committed profiles/pmc_<config>.json)."""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    tmp = tempfile.mkdtemp(prefix="rtx_pmc_")
    child = [sys.executable, os.path.abspath(__file__), "--config", args.config, "--steps", "2",
             "--warmup", "1", "--no-cpu-baseline", "--pmc", "off", "--no-other-configs"]
    if args.width:
        child += ["--width", str(args.width)]
    if args.spp:
        child += ["--spp", str(args.spp)]
    res = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for name, ctrs in PMC_PASSES.items():
        d = os.path.join(tmp, name)
        cmd = ["timeout", "-s", "KILL", "240", prof, "--pmc"] + ctrs + [
            "--output-format", "csv", "-d", d, "-o", name, "--"] + child
        print("bench: PMC pass %s (%s)" % (name, " ".join(ctrs)), file=sys.stderr, flush=True)
        try:
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env,
                               timeout=260)
        except subprocess.TimeoutExpired:
            return None
        if r.returncode != 0:
            print("bench: PMC pass %s failed (rc %d): %s" % (name, r.returncode,
                                                               r.stderr.decode()[-400:]),
                  file=sys.stderr)
            return None
        c, n = pmc_counters(d)
        if not n or any(k not in c for k in ctrs):
            return None
        res.update(c)
        res["launches_" + name] = n
    f64 = sum(res[k] for k in PMC_PASSES["valu"][2:6])
    return {
        "source": "live: rocprofv3 --pmc passes run by bench.py on this build and workload",
        "hbm_read_bytes_per_launch": int(2 * res["FETCH_SIZE"] * 1024),
        "hbm_write_bytes_per_launch": int(res["WRITE_SIZE"] * 1024),
        "hbm_bytes_per_launch": int(2 * res["FETCH_SIZE"] * 1024 + res["WRITE_SIZE"] * 1024),
        "valu_insts_per_launch": int(res["SQ_INSTS_VALU"]),
        "f64_insts_per_launch": int(f64),
        "f64_flops_per_launch": int(64 * (f64 - res["SQ_INSTS_VALU_FMA_F64"])
                                    + 128 * res["SQ_INSTS_VALU_FMA_F64"]),
        "valu_busy": round(4 * res["SQ_ACTIVE_INST_VALU"] / (res["GRBM_GUI_ACTIVE"] / 8 * 1024), 4),
        "launches": [res["launches_" + k] for k in PMC_PASSES],
    }


def host_cpu_info():
    """Host cores as the reference sees them (std::thread::hardware_concurrency()
    == os.cpu_count()), the cores this process may run on, the cgroup CPU quota
    and the CPU model."""
    info = {"hardware_concurrency": os.cpu_count() or 1}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def grow(run, target_s):
    """Run run(spp) at square sample counts 1, 4, 9, ... (up to 256) until one
    run takes at least half of target_s; returns (spp, seconds) of the last run.
    Each step is sized from the previous run's rate, which per-row overhead
    makes look slow at low spp."""
    sq, dt = 1, run(1)
    while dt < 0.5 * target_s and sq < 16:
        nxt = int(sq * (target_s / max(dt, 1e-3)) ** 0.5)
        sq = max(sq + 1, min(16, nxt))
        dt = run(sq * sq)
    return sq * sq, dt


def cpu_baseline(scene, cam_full):
    """The reference's OWN multithreaded CPU path: StaticCamera::render with -p
    (use_parallelism), i.e. render_cpu's ThreadPool of
    std::thread::hardware_concurrency() workers, one task per pixel, a barrier per
    row, and its PPM writer (StaticCamera.cpp:32-100, ThreadPool.hpp:6-174),
    compiled from /root/reference/src into oracle/_ref.

    Bounded sample: the same scene and depth at 960x540 (the reference pool's
    1024-slot Chase-Lev deque overflows on rows wider than 1023 pixels and
    corrupts the heap -- measured: `malloc(): unaligned fastbin chunk detected`
    at 1920 wide, WorkStealingDeque.hpp:29-43 vs :72-85 -- so the sample keeps
    rows short), at the square sample count grow() reaches from 1 spp for a
    timed run of ~8-15 s of CPU work."""
    import ctypes as C
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    host = host_cpu_info()
    width = 960
    h = max(1, int(width / cam_full.aspect_ratio))

    def run(spp):
        cam = scene.camera_desc(image_width=width, samples_per_pixel=spp,
                                max_depth=cam_full.max_depth)
        d = scene.desc()
        cwd = os.getcwd()
        tmp = tempfile.mkdtemp(prefix="rtx_cpu_")
        err = os.dup(2)
        try:
            os.chdir(tmp)  # the reference writes output/<file> under the cwd
            with open(os.path.join(tmp, "clog.txt"), "w") as f:
                os.dup2(f.fileno(), 2)  # its "Scanlines remaining" progress (std::clog)
                t = time.perf_counter()
                if O.ref_available():
                    O.ref().ref_render_static(C.byref(d), C.byref(cam), 1, int(scene.use_bvh), 1,
                                              b"cpu_baseline.ppm")
                else:  # reference build absent: the oracle restatement, same decomposition
                    O.oracle_render(scene, cam, O.MODE_COUNTER, 1, threads=host["hardware_concurrency"])
                dt = time.perf_counter() - t
        finally:
            os.dup2(err, 2)
            os.close(err)
            os.chdir(cwd)
        return dt

    spp, dt = grow(run, 15.0)
    n = width * h * spp
    out = {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s",
           "cores": host["hardware_concurrency"],
           "kind": "reference" if O.ref_available() else "port",
           "sample": "StaticCamera::render -p (ThreadPool, hardware_concurrency() = %d workers), "
                     "%s %dx%d @ %d spp, depth %d, %.1f s" % (
                         host["hardware_concurrency"], scene_name_of(scene), width, h, spp,
                         cam_full.max_depth, dt)}
    out.update({k: v for k, v in host.items() if k != "hardware_concurrency"})
    # The box may cap this process below hardware_concurrency() (cgroup CPU
    # quota): the reference's pool then oversubscribes the quota with spinning
    # workers.  Beside the primary figure, the same -p loop on the reference's
    # ThreadPool sized to the quota.
    quota = host.get("cgroup_cpu_quota") or host.get("affinity_cpus")
    if O.ref_available() and quota and int(quota) < host["hardware_concurrency"]:
        nt = max(1, int(quota))

        def run_pool(spp):
            cam = scene.camera_desc(image_width=width, samples_per_pixel=spp,
                                    max_depth=cam_full.max_depth)
            t = time.perf_counter()
            O.ref_trace_pool(scene, cam, nt)
            return time.perf_counter() - t
        spp2, dt2 = grow(run_pool, 10.0)
        out["quota_sized_pool"] = {
            "value": round(width * h * spp2 / dt2 / 1e6, 4), "unit": "Msamples/s", "cores": nt,
            "sample": "render_cpu -p loop on the reference ThreadPool with %d workers, "
                      "%dx%d @ %d spp, %.1f s" % (nt, width, h, spp2, dt2)}
    return out


def scene_name_of(scene):
    return getattr(scene, "_name", "scene")


def other_configs(args, torch, dev, skip):
    """The other single-GPU BASELINE configs at their full size (C3: 486-sphere BVH
    scene at spp 256; C4: Cornell + fog + Perlin at spp 1024), timed like the
    headline (device-resident frame buffer, barrier-free single rank, K steps
    bracketed by device syncs) so the bench line carries every 1080p config."""
    from rtx import abi
    from rtx.render import Renderer, camera_frame
    from rtx.scene import load_scene
    res = {}
    for c in ("C3", "C4"):
        if c == skip:
            continue
        name, width, spp, depth = CONFIGS[c]
        S = load_scene(os.path.join(SCENES, name + ".json"))
        f = camera_frame(S.camera_desc(image_width=width, samples_per_pixel=spp, max_depth=depth))
        buf = torch.empty((f.image_height, f.image_width, 3), dtype=torch.float64, device=dev)
        steps = 2 if c == "C4" else 4
        with Renderer(S, device=dev.index or 0) as R:
            def go(seed):
                R.render_device(f, buf.data_ptr(), 0, seed=seed, output=abi.RT_OUT_SUM, accumulate=0)
            go(999)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            ms = []
            for k in range(steps):
                go(k)
                ms.append(R.last_kernel_ms())
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
        n = f.image_width * f.image_height * f.sqrt_spp ** 2 * steps
        res[c] = {"workload": "%s %s %dx%d spp%d depth%d" % (c, name, f.image_width, f.image_height,
                                                             f.sqrt_spp ** 2, depth),
                  "value": round(n / dt / 1e6, 3), "unit": "Msamples/s", "steps": steps,
                  "ms_per_step": round(dt * 1e3 / steps, 3),
                  "kernel_ms": round(sum(ms) / len(ms), 3)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="N=1: skip timing C3 and C4 beside the headline config")
    # rehearsal of the N>1 path on one GPU: every rank on cuda:0, gloo all_reduce
    # instead of RCCL reduce (the driver's 8-GPU runs use the defaults)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--share-device", action="store_true")
    ap.add_argument("--shard", default="tiles", choices=["tiles", "strata"],
                    help="N>1: tiles round-robin + gather (default) or strata + reduce")
    ap.add_argument("--n1-layout", default="frame", choices=["frame", "tiles"],
                    help="N=1: render straight into the frame (default) or in 8x8 tile "
                         "work units + chunk sum + tile->frame reorder, as the N>1 path")
    ap.add_argument("--pg-rehearsal", action="store_true",
                    help="N=1: still create the process group and run the N>1 exchange "
                         "(RCCL gather/reduce over a world of one) -- exercises the "
                         "collective path the driver's multi-GPU runs take on one GPU")
    ap.add_argument("--check", action="store_true",
                    help="rank 0 compares the reduced frame with a 1-device render")
    ap.add_argument("--pmc-save", default="",
                    help="write the live PMC summary (the pmc_<config>.json format) here")
    ap.add_argument("--pmc", default="auto", choices=["auto", "file", "off"],
                    help="N=1 roofline counters: auto = rocprofv3 PMC passes of this build "
                         "run before the timed run (fallback: the committed "
                         "profiles/pmc_<config>.json), file = the committed file only")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    pmc = None
    if ws == 1 and args.pmc == "auto":  # before this process initialises the GPU
        pmc = pmc_live(args)
        if pmc and args.pmc_save:
            with open(args.pmc_save, "w") as fh:
                json.dump(dict(pmc, config=args.config), fh, indent=1)
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
    use_pg = ws > 1 or args.pg_rehearsal
    if use_pg:
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
    tiles_mode = (use_pg and args.shard == "tiles") or (ws == 1 and args.n1_layout == "tiles")

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
                final["frame"] = shard.frame_sums(gath[b] if use_pg else tsum[b].unsqueeze(0))
            else:
                final["frame"] = bufs[b]
            final["step"] = k

    def exchange(b):
        if not use_pg:
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

    if use_pg:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, k)
        if ws == 1:
            kernel_ms.append(R.last_kernel_ms())  # HIP events around the kernel, launch stream
    drain()
    torch.cuda.synchronize(dev)
    if use_pg:
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
    pmc_path = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if pmc is None and ws == 1 and args.pmc != "off" and os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            pmc["source"] = "committed file profiles/pmc_%s.json (an earlier PMC run)" % args.config
        except (OSError, ValueError):
            pmc = None
    kernel_s = avg_ms * 1e-3
    # The binding roof is vector-ALU issue: the scene is
    # L1/L2/LDS-resident, so HBM carries only the accumulator.  frac = VALU-busy,
    # SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (GRBM_GUI_ACTIVE / 8 XCDs x 1024
    # SIMDs), from the PMC passes; physical HBM traffic (FETCH_SIZE x 2 +
    # WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction) is reported beside it.
    roof = {"bound": "valu", "unit": "fraction of SIMD cycles issuing VALU", "peak": 1.0,
            "achieved": None, "frac": None, "traffic": None, "kernel_ms": round(avg_ms, 3)}
    if pmc and pmc.get("valu_busy") is not None:
        roof["achieved"] = roof["frac"] = pmc["valu_busy"]
    if pmc and pmc.get("hbm_bytes_per_launch"):
        tb = pmc["hbm_bytes_per_launch"]
        roof["traffic"] = tb
        roof["hbm"] = {"bytes_per_launch": tb, "read_bytes_per_launch": pmc.get("hbm_read_bytes_per_launch"),
                       "write_bytes_per_launch": pmc.get("hbm_write_bytes_per_launch"),
                       "achieved_gbs": round(tb / kernel_s / 1e9, 2), "peak_gbs": HBM_PEAK_GBS,
                       "frac": round(tb / kernel_s / 1e9 / HBM_PEAK_GBS, 5)}
    if pmc and pmc.get("f64_flops_per_launch"):
        tfs = pmc["f64_flops_per_launch"] / kernel_s / 1e12
        roof["f64"] = {"achieved_tflops": round(tfs, 3), "peak_tflops": F64_PEAK_TFS,
                       "frac": round(tfs / F64_PEAK_TFS, 4),
                       "valu_insts_per_launch": pmc.get("valu_insts_per_launch"),
                       "f64_insts_per_launch": pmc.get("f64_insts_per_launch")}
    if pmc:
        roof["pmc_source"] = pmc.get("source")
    # SURVEY §8(d)'s algorithmic bytes: what the traversal/shading reads from the
    # scene tables per launch.  Served by LDS/L1/L2, not HBM -- a cache-side
    # figure, never an HBM fraction.
    roof["cache_served"] = {"bytes_per_launch": int(bytes_launch),
                            "bytes_per_sample": round(bytes_launch / max(1, st["samples"]), 1),
                            "gbs": round(achieved, 1)}
    roof["counters"] = st
    if st.get("cyc_loop"):
        # STATS instance: shares of a wavefront's loop time per region (s_memtime)
        roof["phase_share"] = {k[4:]: round(st[k] / st["cyc_loop"], 4) for k in (
            "cyc_regen", "cyc_trace", "cyc_media", "cyc_shade", "cyc_lights")}
    roof["lane_utilisation"] = {
        "traversal": round(st["node_visits"] / max(1, 64 * st["wave_node_iters"]), 4),
        "leaf": round((st["sphere_tests"] + st["quad_tests"]) / max(1, 64 * st["wave_leaf_iters"]), 4),
        "shading": round(st["shade_events"] / max(1, 64 * st["wave_shade_iters"]), 4),
        "path_trips": round(st["segments"] / max(1, 64 * st["wave_trips"]), 4)}
    roof["note"] = ("VALU-issue bound; N>1 lines carry no PMC data (traffic null)"
                    if ws == 1 else "N>1: no PMC pass in multi-rank runs (traffic null)")

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
                                    if tiles_mode else "1 GPU") if not use_pg else
                                   "tile-shard x%d (tile t on rank t %% %d, %d stratum chunks) + %s gather" % (
                                       ws, ws, shard.chunks,
                                       "RCCL" if args.backend == "nccl" else "gloo")
                                   if tiles_mode else
                                   "stratum-shard x%d + %s reduce(sum)" % (
                                       ws, "RCCL" if args.backend == "nccl" else "gloo"))},
        "roofline": roof,
    }
    if check is not None:
        out["check"] = check
    if rank == 0 and ws == 1 and not args.no_other_configs and not args.width and not args.spp:
        out["other_configs"] = other_configs(args, torch, dev, args.config)
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(scene, cam)
    if rank == 0:
        print(json.dumps(out), flush=True)
    R.close()
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
