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
  * a roofline object for the render kernel: bound "valu" -- the kernel issues
    vector instructions most cycles and the scene is cache/LDS-resident, so the
    roof is the fp64 vector peak (78.6 TFLOP/s); achieved = fp64 FLOP per
    launch (rocprofv3 PMC passes bench.py runs on this build and workload
    before the timed run) / the live HIP-event kernel time.  VALU-busy, the
    fp64 share of the VALU instructions, physical HBM bytes per launch
    (traffic) and GB/s sit beside it, and SURVEY §8(d)'s algorithmic bytes as
    the cache-served figure;
  * the other single-GPU BASELINE configs (C3, C4, C5) timed the same way, C3
    with its own live PMC passes and roofline;
  * the host-output rate (rt_render: kernel + D2H into caller host memory,
    pinned and pageable) and the progressive ("real-time") frame rate per
    scene (one stratum per frame + device to-bytes, with and without the bytes
    copied to the host every frame);
  * a CPU baseline: the reference's own render_cpu -p loop on its ThreadPool
    sized to the CPUs this process may use (the as-shipped pool of
    hardware_concurrency() workers beside it), bounded sample.
  * N>1: per-rank kernel ms (min/mean/max over ranks) and rank 0's exchange
    wait, measured in serial diagnostic steps after the timed region.
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


def tuning_from_env():
    """A/B runs only (profiles/ab.sh NAME=VALUE variants): RTX_TUNING =
    "field=value,..." of rt_tuning fields (rtx.abi.Tuning) for the bench's
    scenes.  The library itself reads no environment (ABI 4); unset = the
    default plan."""
    spec = os.environ.get("RTX_TUNING", "").strip()
    if not spec:
        return None
    out = {}
    for kv in spec.split(","):
        k, v = kv.split("=")
        out[k.strip()] = float(v) if k.strip() == "tail_tiles" else int(v)
    return out


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def visible_devices():
    """GPUs this process could use, counted without initialising the GPU
    (torch.cuda.device_count() does not, on this image)."""
    import torch
    return torch.cuda.device_count()


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) with no launcher in the environment: this
    process becomes the launcher.  Before anything touches the GPU it checks
    that N devices are visible (unless --share-device / --device cpu), then
    starts N children of this same script with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set (torchrun's
    variables; one rank per GPU, rank r on cuda:r), relays rank 0's JSON line
    (rank 0 writes to this process's stdout, every other rank's stdout goes to
    stderr), and returns non-zero if any rank fails -- the others are then
    stopped, by their PIDs, rather than left waiting in a collective.  It never
    re-executes itself.  Returns the exit code."""
    import signal
    import socket
    import subprocess
    if args.gpus < 1:
        print("bench: --gpus must be >= 1", file=sys.stderr)
        return 2
    if args.device == "cuda" and not args.share_device:
        n_dev = visible_devices()
        if n_dev < args.gpus:
            print("bench: --gpus %d needs %d GPUs, %d visible (one rank per GPU; "
                  "--share-device puts every rank on cuda:0)" % (args.gpus, args.gpus, n_dev),
                  file=sys.stderr)
            return 2
    port = os.environ.get("MASTER_PORT")
    if not port:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
        s.close()
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    stopping = {"sig": None}

    def on_signal(signum, frame):
        stopping["sig"] = signum

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    try:
        for r in range(args.gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                       LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=port, RTX_BENCH_LAUNCHER="bench.py")
            procs.append(subprocess.Popen(cmd, env=env, stdout=None if r == 0 else sys.stderr))
        print("bench: launched %d ranks (pids %s), MASTER_PORT %s" % (
            args.gpus, " ".join(str(p.pid) for p in procs), port), file=sys.stderr, flush=True)
        live = set(range(args.gpus))
        while live and stopping["sig"] is None:
            for r in sorted(live):
                code = procs[r].poll()
                if code is None:
                    continue
                live.discard(r)
                if code != 0:
                    print("bench: rank %d exited with %d; stopping the other ranks" % (r, code),
                          file=sys.stderr, flush=True)
                    rc = code if code > 0 else 128 - code
                    live.clear()
                    break
            time.sleep(0.1)
        if stopping["sig"] is not None:
            rc = 128 + stopping["sig"]
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for s, h in old.items():
            signal.signal(s, h)
    return rc


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


PMC_PASSES = {  # one rocprofv3 --pmc run each (8 SQ slots; TCC: FETCH_SIZE 3, WRITE_SIZE 2 of 4)
    "valu": ["SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_THREAD_CYCLES_VALU",
             "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
             "SQ_INSTS_VALU_TRANS_F64", "GRBM_GUI_ACTIVE"],
    "fetch": ["FETCH_SIZE"],
    "write": ["WRITE_SIZE"],
}
F64_CLASSES = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
               "SQ_INSTS_VALU_TRANS_F64")


def valu_figures(c):
    """The VALU figures of one launch's SQ counters (rocprofv3's gfx950 counter
    definitions, profiles/r04a_counters_valu.txt; calibrated on saturated
    instruction streams, profiles/r04a_ubench_*):
      SQ_ACTIVE_INST_VALU  quad-cycles of VALU issue, one per instruction (four
                           for a quarter-rate transcendental), summed over SIMDs;
      SQ_ACTIVE_INST_VALU2 the quad-cycles in which TWO VALU instructions issued
                           (gfx950 dual-issues: a saturated stream of 32-bit
                           integer ops issues 1.6, of fp32 FMAs 1.3 instructions
                           per quad-cycle; fp64 / 3-input ops 0.8-0.9);
      SQ_THREAD_CYCLES_VALU the same quad-cycles times the active lanes.
    valu_issue_ratio = ACTIVE / SIMD quad-cycles is rocprofv3's VALUBusy, which
    exceeds 1 under dual issue; valu_busy = (ACTIVE - ACTIVE2) / SIMD
    quad-cycles is the share of quad-cycles in which the VALU issues at all
    (<= 1); valu_lane_fraction = THREAD / (64 ACTIVE) is rocprofv3's
    VALUUtilization, the mean share of a wave's lanes an issued VALU
    instruction works for."""
    simd_quads = c["GRBM_GUI_ACTIVE"] / 8 * 1024 / 4  # GRBM_GUI_ACTIVE is summed over the 8 XCDs
    act = c["SQ_ACTIVE_INST_VALU"]
    out = {"valu_issue_ratio": round(act / simd_quads, 4)}
    if "SQ_ACTIVE_INST_VALU2" in c:
        out["valu_busy"] = round((act - c["SQ_ACTIVE_INST_VALU2"]) / simd_quads, 4)
        out["valu_dual_issue_share"] = round(c["SQ_ACTIVE_INST_VALU2"] / max(1.0, act), 4)
    if "SQ_THREAD_CYCLES_VALU" in c:
        out["valu_lane_fraction"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64 * max(1.0, act)), 4)
    return out


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


def pmc_live(args, config=None):
    """rocprofv3 PMC passes over THIS build and workload, run by bench.py itself
    before it touches the GPU (each pass: a child `bench.py --pmc off` of the
    config, 1 warmup + 2 steps; counters averaged over the plain render
    kernel's launches).  Returns the summary dict or None (no rocprofv3 / a pass
    failed: the caller falls back to the committed profiles/pmc_<config>.json)."""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    tmp = tempfile.mkdtemp(prefix="rtx_pmc_")
    config = config or args.config
    child = [sys.executable, os.path.abspath(__file__), "--config", config, "--steps", "2",
             "--warmup", "1", "--no-cpu-baseline", "--pmc", "off", "--no-other-configs"]
    if config == args.config and args.width:
        child += ["--width", str(args.width)]
    if config == args.config and args.spp:
        child += ["--spp", str(args.spp)]
    res = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for name, ctrs in PMC_PASSES.items():
        d = os.path.join(tmp, name)
        cmd = ["timeout", "-s", "KILL", "240", prof, "--pmc"] + ctrs + [
            "--output-format", "csv", "-d", d, "-o", name, "--"] + child
        print("bench: %s PMC pass %s (%s)" % (config, name, " ".join(ctrs)), file=sys.stderr,
              flush=True)
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
    f64 = sum(res[k] for k in F64_CLASSES)
    return dict(valu_figures(res), **{
        "source": "live: rocprofv3 --pmc passes run by bench.py on this build and workload",
        "hbm_read_bytes_per_launch": int(2 * res["FETCH_SIZE"] * 1024),
        "hbm_write_bytes_per_launch": int(res["WRITE_SIZE"] * 1024),
        "hbm_bytes_per_launch": int(2 * res["FETCH_SIZE"] * 1024 + res["WRITE_SIZE"] * 1024),
        "valu_insts_per_launch": int(res["SQ_INSTS_VALU"]),
        "f64_insts_per_launch": int(f64),
        "f64_flops_per_launch": int(64 * (f64 - res["SQ_INSTS_VALU_FMA_F64"])
                                    + 128 * res["SQ_INSTS_VALU_FMA_F64"]),
        "valu_counters": {k: int(res[k]) for k in PMC_PASSES["valu"]},
        "launches": [res["launches_" + k] for k in PMC_PASSES],
        "config": config,
    })


def load_pmc(args, config, live):
    """The live PMC summary, else the committed profiles/pmc_<config>.json."""
    if live is not None:
        return live
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % config)
    if args.pmc == "off" or not os.path.exists(path):
        return None
    try:
        pmc = json.load(open(path))
    except (OSError, ValueError):
        return None
    pmc["source"] = "committed file profiles/pmc_%s.json (an earlier PMC run)" % config
    return pmc


def roofline(pmc, kernel_ms):
    """Roofline of the render kernel: the fp64 vector roof (the kernel is
    VALU-issue bound and LDS/cache resident).  achieved = fp64
    FLOP per launch (PMC: 64 per ADD/MUL/TRANS, 128 per FMA wave instruction) /
    the HIP-event kernel time; VALU-busy, the fp64 share of VALU instructions
    and the physical HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950
    correction of MI355X_MICROARCH.md) per launch beside it."""
    kernel_s = kernel_ms * 1e-3
    roof = {"bound": "valu", "unit": "TFLOP/s", "peak": F64_PEAK_TFS, "achieved": None,
            "frac": None, "traffic": None, "kernel_ms": round(kernel_ms, 3)}
    if not pmc:
        return roof
    if pmc.get("f64_flops_per_launch"):
        tfs = pmc["f64_flops_per_launch"] / kernel_s / 1e12
        roof["achieved"] = round(tfs, 3)
        roof["frac"] = round(tfs / F64_PEAK_TFS, 4)
    for k in ("valu_busy", "valu_issue_ratio", "valu_dual_issue_share", "valu_lane_fraction"):
        if pmc.get(k) is not None:
            roof[k] = pmc[k]
    if roof["frac"] is not None and pmc.get("valu_lane_fraction") is not None:
        # fp64 FLOP rate counting only the lanes an instruction works for: the
        # issued rate x the mean active-lane share of the VALU instructions
        roof["achieved_active_lanes"] = round(roof["achieved"] * pmc["valu_lane_fraction"], 3)
        roof["frac_active_lanes"] = round(roof["frac"] * pmc["valu_lane_fraction"], 4)
    if pmc.get("valu_insts_per_launch") and pmc.get("f64_insts_per_launch"):
        roof["f64_inst_share"] = round(pmc["f64_insts_per_launch"] / pmc["valu_insts_per_launch"], 4)
        roof["valu_insts_per_launch"] = pmc["valu_insts_per_launch"]
        roof["f64_insts_per_launch"] = pmc["f64_insts_per_launch"]
    if pmc.get("hbm_bytes_per_launch"):
        tb = pmc["hbm_bytes_per_launch"]
        roof["traffic"] = tb
        roof["hbm_read_bytes"] = pmc.get("hbm_read_bytes_per_launch")
        roof["hbm_write_bytes"] = pmc.get("hbm_write_bytes_per_launch")
        roof["hbm_gbs"] = round(tb / kernel_s / 1e9, 2)
        roof["hbm_frac"] = round(tb / kernel_s / 1e9 / HBM_PEAK_GBS, 5)
    roof["pmc_source"] = pmc.get("source")
    return roof


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
    """The reference's OWN multithreaded CPU path, compiled from
    /root/reference/src into oracle/_ref: render_cpu's -p loop (one task per
    pixel, a barrier per row, StaticCamera.cpp:32-100) on the reference's
    ThreadPool (ThreadPool.hpp:6-174), with as many workers as CPUs this process
    may use (the cgroup quota / affinity) -- `value`.  Beside it, as shipped:
    StaticCamera::render -p with its pool of std::thread::hardware_concurrency()
    workers and its PPM writer (`as_shipped_*`); on a box whose quota is far
    below the machine's CPUs its spinning workers oversubscribe the quota.

    Bounded samples: the same scene and depth at 960x540 (the reference pool's
    1024-slot Chase-Lev deque overflows on rows wider than 1023 pixels and
    corrupts the heap -- measured: `malloc(): unaligned fastbin chunk detected`
    at 1920 wide, WorkStealingDeque.hpp:29-43 vs :72-85 -- so the sample keeps
    rows short), at the square sample count grow() reaches from 1 spp for a
    timed run of ~5-10 s; the as-shipped run at 480x270, 1 spp upwards."""
    import ctypes as C
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    host = host_cpu_info()
    hw = host["hardware_concurrency"]
    usable = host.get("cgroup_cpu_quota") or host.get("affinity_cpus") or hw
    usable = max(1, min(hw, int(usable)))
    ref = O.ref_available()

    def cam_at(width, spp):
        return scene.camera_desc(image_width=width, samples_per_pixel=spp,
                                 max_depth=cam_full.max_depth)

    def run_static(width, spp):
        cam = cam_at(width, spp)
        d = scene.desc()
        cwd = os.getcwd()
        tmp = tempfile.mkdtemp(prefix="rtx_cpu_")
        err = os.dup(2)
        try:
            os.chdir(tmp)  # the reference writes output/<file> under the cwd
            with open(os.path.join(tmp, "clog.txt"), "w") as f:
                os.dup2(f.fileno(), 2)  # its "Scanlines remaining" progress (std::clog)
                t = time.perf_counter()
                if ref:
                    O.ref().ref_render_static(C.byref(d), C.byref(cam), 1, int(scene.use_bvh), 1,
                                              b"cpu_baseline.ppm")
                else:  # reference build absent: the oracle restatement, same decomposition
                    O.oracle_render(scene, cam, O.MODE_COUNTER, 1, threads=usable)
                dt = time.perf_counter() - t
        finally:
            os.dup2(err, 2)
            os.close(err)
            os.chdir(cwd)
        return dt

    def hgt(width):
        return max(1, int(width / cam_full.aspect_ratio))

    name = scene_name_of(scene)
    out = {"unit": "Msamples/s", "kind": "reference" if ref else "port"}
    if ref:
        width = 960

        def run_pool(spp):
            t = time.perf_counter()
            O.ref_trace_pool(scene, cam_at(width, spp), usable)
            return time.perf_counter() - t
        spp, dt = grow(run_pool, 10.0)
        out.update({"value": round(width * hgt(width) * spp / dt / 1e6, 4), "cores": usable,
                    "sample": "render_cpu -p loop on the reference ThreadPool with %d workers "
                              "(the CPUs this process may use), %s %dx%d @ %d spp, depth %d, "
                              "%.1f s" % (usable, name, width, hgt(width), spp,
                                          cam_full.max_depth, dt)})
        w2 = 480 if usable < hw else 960
        spp2, dt2 = grow(lambda n: run_static(w2, n), 6.0)
        out.update({"as_shipped_value": round(w2 * hgt(w2) * spp2 / dt2 / 1e6, 4),
                    "as_shipped_workers": hw,
                    "as_shipped_sample": "StaticCamera::render -p (ThreadPool of "
                                         "hardware_concurrency() = %d workers, PPM writer), "
                                         "%s %dx%d @ %d spp, %.1f s" % (
                                             hw, name, w2, hgt(w2), spp2, dt2)})
    else:
        width = 960
        spp, dt = grow(lambda n: run_static(width, n), 10.0)
        out.update({"value": round(width * hgt(width) * spp / dt / 1e6, 4), "cores": usable,
                    "sample": "oracle restatement (reference build absent), %d threads, "
                              "%s %dx%d @ %d spp, %.1f s" % (usable, name, width, hgt(width),
                                                             spp, dt)})
    out.update({k: v for k, v in host.items()})
    return out


def scene_name_of(scene):
    return getattr(scene, "_name", "scene")


def other_configs(args, torch, dev, skip, pmcs):
    """The other single-GPU BASELINE configs at their full size (C3: 486-sphere
    BVH scene at spp 256; C4: Cornell + fog + Perlin at spp 1024; C5: the
    486-sphere scene with motion blur at 3840x2160, spp 4096 -- BASELINE names
    it an 8-GPU config; one GPU renders the whole frame here), timed like the
    headline (device-resident frame buffer, single rank, K steps bracketed by
    device syncs, HIP-event kernel time), so the bench line carries every
    config; C3 and C4 also with their own roofline (live PMC passes when
    available)."""
    from rtx import abi
    from rtx.render import Renderer, camera_frame
    from rtx.scene import load_scene
    res = {}
    plan = {"C3": (1, 4), "C4": (1, 2), "C5": (1, 1)}  # (warmup, steps)
    for c, (warm, steps) in plan.items():
        if c == skip:
            continue
        name, width, spp, depth = CONFIGS[c]
        S = load_scene(os.path.join(SCENES, name + ".json"))
        f = camera_frame(S.camera_desc(image_width=width, samples_per_pixel=spp, max_depth=depth))
        buf = torch.empty((f.image_height, f.image_width, 3), dtype=torch.float64, device=dev)
        with Renderer(S, device=dev.index or 0, tuning=tuning_from_env()) as R:
            def go(seed):
                R.render_device(f, buf.data_ptr(), 0, seed=seed, output=abi.RT_OUT_SUM, accumulate=0)
            for w in range(warm):
                go(999 + w)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            ms = []
            for k in range(steps):
                go(k)
                ms.append(R.last_kernel_ms())
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            finite = bool(torch.isfinite(buf).all().item())
        n = f.image_width * f.image_height * f.sqrt_spp ** 2 * steps
        kms = sum(ms) / len(ms)
        res[c] = {"workload": "%s %s %dx%d spp%d depth%d" % (c, name, f.image_width, f.image_height,
                                                             f.sqrt_spp ** 2, depth),
                  "value": round(n / dt / 1e6, 3), "unit": "Msamples/s", "steps": steps,
                  "warmup": warm, "ms_per_step": round(dt * 1e3 / steps, 3),
                  "kernel_ms": round(kms, 3), "finite": finite}
        if c in pmcs:
            res[c]["roofline"] = roofline(pmcs[c], kms)
    return res


def host_output(torch, R, frame, steps):
    """rt_render, the drop-in for render_gpu's batch loop: the frame kernel plus
    the D2H copy of the scaled radiance into caller host memory, synchronous.
    Pinned (page-locked) and pageable caller buffers."""
    import numpy as np
    n = frame.image_width * frame.image_height * frame.sqrt_spp ** 2
    res = {}
    pinned = torch.empty((frame.image_height, frame.image_width, 3), dtype=torch.float64,
                         pin_memory=True)
    pageable = np.empty((frame.image_height, frame.image_width, 3), dtype=np.float64)
    for kind, ptr in (("pinned", pinned.data_ptr()), ("pageable", pageable.ctypes.data)):
        R.render_into(frame, ptr, seed=77)  # warm (first touch of the pages)
        t0 = time.perf_counter()
        kms = []
        for k in range(steps):
            R.render_into(frame, ptr, seed=k)
            kms.append(R.last_kernel_ms())
        dt = (time.perf_counter() - t0) / steps
        res[kind] = {"value": round(n / dt / 1e6, 3), "unit": "Msamples/s",
                     "ms_per_step": round(dt * 1e3, 3),
                     "kernel_ms": round(sum(kms) / len(kms), 3),
                     "copy_ms": round(dt * 1e3 - sum(kms) / len(kms), 3),
                     "bytes_per_step": frame.image_width * frame.image_height * 24}
    res["note"] = ("rt_render: render + D2H of the %d MB fp64 frame into caller memory, "
                   "host-synchronous per frame" % (frame.image_width * frame.image_height * 24 // 10 ** 6))
    return res


def progressive_rates(torch, dev, width=1920, frames=30):
    """The real-time half (DynamicCamera.cpp:350-564): one
    stratum of every pixel per frame, added into a device accumulator
    (rt_render_device, accumulate) and quantised on the device
    (rt_to_bytes_device), on the null stream.  Per scene at 1080p:
      device_ms  -- frames issued back to back, one sync at the end;
      display_ms -- every frame also copies its 6.2 MB of bytes to pinned host
                    memory and waits for them (what a viewer must do per frame;
                    the reference copies the whole 49.8 MB fp64 accumulator back,
                    DynamicCamera.cpp:524-532);
      pipelined_display_ms -- the same bytes through rtx.progressive's
                    DisplayPipeline: frame k's copy runs on a copy stream while
                    frame k+1 renders, the viewer takes frame k-1's bytes."""
    from rtx.progressive import DisplayPipeline, for_renderer, frame_bytes
    from rtx.render import Renderer, camera_frame
    from rtx.scene import load_scene
    res = {}
    for c in ("C2", "C3", "C4"):
        name, _, spp, depth = CONFIGS[c]
        S = load_scene(os.path.join(SCENES, name + ".json"))
        f = camera_frame(S.camera_desc(image_width=width, samples_per_pixel=spp, max_depth=depth))
        with Renderer(S, device=dev.index or 0) as R:
            pr = for_renderer(R, f, seed=5)
            out = torch.empty(pr.acc.shape, dtype=torch.uint8, device=dev)
            host = torch.empty(pr.acc.shape, dtype=torch.uint8, pin_memory=True)
            for _ in range(2):  # warm
                pr.step(1)
                frame_bytes(pr, out)
            torch.cuda.synchronize(dev)
            pr.reset()
            t0 = time.perf_counter()
            for _ in range(frames):
                pr.step(1)
                frame_bytes(pr, out)
            torch.cuda.synchronize(dev)
            dev_ms = (time.perf_counter() - t0) * 1e3 / frames
            pr.reset()
            t0 = time.perf_counter()
            for _ in range(frames):
                pr.step(1)
                frame_bytes(pr, out)
                host.copy_(out, non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
            disp_ms = (time.perf_counter() - t0) * 1e3 / frames
            pr.reset()
            pipe = DisplayPipeline(pr)
            for _ in range(2):  # warm
                pipe.frame()
                pipe.present()
            pipe.flush()
            pr.reset()
            t0 = time.perf_counter()
            for _ in range(frames):
                pipe.frame()
                pipe.present()
            pipe.flush()
            pipe_ms = (time.perf_counter() - t0) * 1e3 / frames
        res[c] = {"scene": name, "width": f.image_width, "height": f.image_height,
                  "strata_per_frame": 1, "frames_to_converge": f.sqrt_spp ** 2,
                  "device_ms_per_frame": round(dev_ms, 3), "device_fps": round(1e3 / dev_ms, 1),
                  "display_ms_per_frame": round(disp_ms, 3), "display_fps": round(1e3 / disp_ms, 1),
                  "pipelined_display_ms_per_frame": round(pipe_ms, 3),
                  "pipelined_display_fps": round(1e3 / pipe_ms, 1)}
    return res


def rank_diagnostics(torch, dist, dev, rank, ws, launch_work, exchange, wait_exchange, steps=2):
    """N>1: serial diagnostic steps after the timed region.  Each step: barrier,
    this rank's render timed with HIP events on its launch stream, then the
    frame exchange timed on the host from this rank's render completion to the
    exchange's completion (rank 0: the wait for the slowest rank plus the
    transfer).  Returns per-rank kernel ms and exchange ms, gathered on every
    rank (min / mean / max, and the per-rank lists)."""
    cuda = dev.type == "cuda"  # the CPU tests drive the same code with host clocks
    stream = torch.cuda.current_stream(dev) if cuda else None
    kms, xms = [], []
    for k in range(steps):
        dist.barrier()
        if cuda:
            torch.cuda.synchronize(dev)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            launch_work(6000 + k, 0)
            e1.record(stream)
            e1.synchronize()
            kms.append(e0.elapsed_time(e1))
        else:
            t0 = time.perf_counter()
            launch_work(6000 + k, 0)
            kms.append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        wait_exchange(exchange(0))
        if cuda:
            torch.cuda.synchronize(dev)
        xms.append((time.perf_counter() - t0) * 1e3)
    mine = torch.tensor([sum(kms) / len(kms), sum(xms) / len(xms)], dtype=torch.float64)
    if dist.get_backend() == "nccl" and cuda:
        mine = mine.to(dev)
    allv = [torch.zeros_like(mine) for _ in range(ws)]
    dist.all_gather(allv, mine)
    per_k = [round(float(v[0]), 3) for v in allv]
    per_x = [round(float(v[1]), 3) for v in allv]
    return {"kernel_ms_min": min(per_k), "kernel_ms_mean": round(sum(per_k) / ws, 3),
            "kernel_ms_max": max(per_k), "exchange_ms_rank0": per_x[0],
            "exchange_ms_max": max(per_x), "per_rank_kernel_ms": per_k,
            "per_rank_exchange_ms": per_x, "diagnostic_steps": steps,
            "note": "serial steps after the timed region: render (HIP events), then the "
                    "exchange from this rank's render end to its completion (host clock)"}


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
    ap.add_argument("--shard-units", type=int, default=0,
                    help="N>1 tile shards: work units per rank (0: rtx.dist.shard_units)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: every rank renders with the CPU backend (librtx_cpu.so) and "
                         "exchanges over gloo -- the launcher / exchange path without a GPU "
                         "(tests); never the measured line")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # tests: that
    # rank exits 3 once the process group is up (the launcher must stop the others)
    ap.add_argument("--pmc", default="auto", choices=["auto", "file", "off"],
                    help="N=1 roofline counters: auto = rocprofv3 PMC passes of this build "
                         "run before the timed run (fallback: the committed "
                         "profiles/pmc_<config>.json), file = the committed file only")
    args = ap.parse_args()
    cpu = args.device == "cpu"
    if cpu and args.backend != "gloo":
        print("bench: --device cpu exchanges over gloo (--backend gloo)", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus != 1:
        # no launcher: start the ranks here (before anything touches the GPU)
        sys.exit(launch_ranks(args))

    ws, rank, local = dist_env()
    if ws != args.gpus:
        print("bench: --gpus %d but the launcher started WORLD_SIZE %d ranks" % (args.gpus, ws),
              file=sys.stderr)
        sys.exit(2)
    pmc = None
    full_line = (ws == 1 and not cpu and not args.no_other_configs and not args.width
                 and not args.spp)
    pmc_other = {}
    if ws == 1 and args.pmc == "auto" and not cpu:  # before this process initialises the GPU
        pmc = pmc_live(args)
        if pmc and args.pmc_save:
            with open(args.pmc_save, "w") as fh:
                json.dump(dict(pmc, config=args.config), fh, indent=1)
        for c in ("C3", "C4"):  # the other configs with their own live roofline
            if full_line and args.config != c:
                pmc_other[c] = pmc_live(args, c)
    for c in ("C3", "C4"):
        if full_line and args.config != c:
            pmc_other[c] = load_pmc(args, c, pmc_other.get(c))
    import torch
    from rtx import abi
    from rtx.render import Renderer, camera_frame
    from rtx.scene import load_scene

    if args.share_device:
        local = 0
    dev = torch.device("cpu") if cpu else torch.device("cuda", local)
    if not cpu:
        torch.cuda.set_device(dev)

    def sync():
        if not cpu:
            torch.cuda.synchronize(dev)
    use_pg = ws > 1 or args.pg_rehearsal
    seen = 1
    if use_pg:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            print("bench: --gpus %d but the process group has %d ranks" % (
                args.gpus, dist.get_world_size()), file=sys.stderr)
            sys.exit(2)
    from rtx.dist import ShardedRenderer, TileShardedRenderer, max_over_ranks, ranks_seen
    if use_pg:  # the ranks the exchange's collective actually reaches (RCCL for nccl)
        seen = ranks_seen(dev if args.backend == "nccl" else None)
    if rank == args.fail_rank:
        print("bench: rank %d failing on request (--fail-rank)" % rank, file=sys.stderr, flush=True)
        os._exit(3)

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

    if cpu:  # the ranks share this host's CPUs
        from rtx.cpu import CpuRenderer, default_threads
        R = CpuRenderer(scene, threads=max(1, default_threads() // ws))
        info, stream_ptr = None, None
    else:
        R = Renderer(scene, device=local, tuning=tuning_from_env())
        info = R.info()
        # the null stream: ordered with RCCL's waits
        stream_ptr = torch.cuda.current_stream(dev).cuda_stream

    def render_fn(fr, acc, seed, strata):
        # overwrite the partial sums (no memset, no read-modify-write)
        R.render_device(fr, acc.data_ptr(), stream_ptr, seed=seed, samples=strata,
                        output=abi.RT_OUT_SUM, accumulate=0)

    def tile_render_fn(fr, buf, seed, tiles, chunks):
        R.render_device(fr, buf.data_ptr(), stream_ptr, seed=seed, samples=(0, -1),
                        output=abi.RT_OUT_SUM, accumulate=0, tiles=tiles,
                        layout=abi.RT_LAYOUT_TILES, chunks=chunks)

    if tiles_mode:
        shard = TileShardedRenderer(tile_render_fn, frame, rank, ws,
                                    target_units=args.shard_units or None)
        if cpu:
            shard.on_host()
        bufs = [shard.buffer(dev) for _ in range(2)]
        gath = [shard.gather_buffer(dev) if rank == 0 else None for _ in range(2)]
        sums = [shard.sum_buffer(dev) for _ in range(2)]   # per-tile sums (device chunk sum)
        frames = [shard.frame_buffer(dev) if rank == 0 else None for _ in range(2)]
        tsum = [None, None]

        def launch_work(seed, b):
            tsum[b] = shard.render(bufs[b], seed, out=sums[b])
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
                # reorder the gathered tiles on the device (N=1: this rank's own tile sums)
                final["frame"] = shard.frame_sums(gath[b] if use_pg else tsum[b].unsqueeze(0),
                                                  out=frames[b])
            else:
                final["frame"] = bufs[b]
            final["step"] = k

    def exchange(b):
        if not use_pg:
            return None
        if tiles_mode:
            if args.backend == "nccl":
                return shard.gather(tsum[b], gath[b], async_op=True)
            sync()  # gloo: host-staged, no CUDA gather
            host = tsum[b].cpu()
            parts = [torch.empty_like(host) for _ in range(ws)] if rank == 0 else None
            dist.gather(host, gather_list=parts, dst=0)
            if rank == 0:
                gath[b].copy_(torch.stack(parts))
            return None
        if args.backend == "nccl":
            return dist.reduce(bufs[b], dst=0, op=dist.ReduceOp.SUM, async_op=True)
        sync()  # gloo has no CUDA reduce
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
    sync()

    if use_pg:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    host_s = 0.0  # host time spent issuing the steps (the launch side of the pipeline)
    for k in range(args.steps):
        h0 = time.perf_counter()
        step(k, k)
        host_s += time.perf_counter() - h0
        if not use_pg:
            kernel_ms.append(R.last_kernel_ms())  # HIP events around the kernel, launch stream
    drain()
    sync()
    if use_pg:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    check = None
    if args.check and rank == 0:  # the last timed frame on rank 0 vs one device, all strata
        assert final["step"] == args.steps - 1
        last = final["frame"].clone()
        ref = torch.empty_like(last)
        render_fn(frame, ref, args.steps - 1, (0, n_strata))
        sync()
        err = (last - ref).abs().max().item()
        scale = max(1.0, ref.abs().max().item())
        check = {"max_abs_diff": err, "ok": bool(err <= 1e-9 * scale)}

    diag = None
    if use_pg:  # kernel time measured after the timed region (no sync inside it)
        for k in range(min(2, args.steps)):
            launch_work(5000 + k, 0)
            kernel_ms.append(R.last_kernel_ms())
        diag = rank_diagnostics(torch, dist, dev, rank, ws, launch_work, exchange,
                                lambda w: w.wait() if w is not None else None)

    samples_per_step = W * H * n_strata  # whole frame, all ranks together
    value = samples_per_step * args.steps / elapsed / 1e6

    def gpu_roofline(pmc):
        # roofline of the dominant (render) kernel on this rank, one launch
        if tiles_mode:
            st = R.stats(frame, seed=0, tiles=(rank, ws), layout=abi.RT_LAYOUT_TILES,
                         chunks=shard.chunks)
        else:
            st = R.stats(frame, seed=0, samples=(s0, s1 - s0))
        px_launch = shard.tiles_per_rank * max(1, shard.chunks) * 64 if tiles_mode else W * H
        bytes_launch = algorithmic_bytes(st, info, px_launch)
        avg_ms = sum(kernel_ms) / len(kernel_ms)
        achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
        pmc = load_pmc(args, args.config, pmc) if ws == 1 else None
        roof = roofline(pmc, avg_ms)
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
        if st.get("wave_noise_iters"):
            roof["lane_utilisation"]["noise_albedo"] = round(
                st["noise_evals"] / (64 * st["wave_noise_iters"]), 4)
        if st.get("medium_box_tests"):
            # box-boundary media: share of their lanes box_span deferred to the
            # general boundary scan (edge / corner / parallel rays)
            roof["lane_utilisation"]["medium_box_deferred"] = round(
                st["medium_box_deferred"] / st["medium_box_tests"], 6)
        if st.get("model_trace_max"):
            # the node-loop SIMD model (STATS): one walk per lane per trip vs each
            # lane's walks of two consecutive trips back to back (two walks per lane)
            roof["lane_utilisation"]["traversal_model_one_walk"] = round(
                st["node_visits"] / (64 * st["model_trace_max"]), 4)
            roof["lane_utilisation"]["traversal_model_two_walks"] = round(
                st["node_visits"] / (64 * max(1, st["model_trace_pair_max"])), 4)
        roof["note"] = ("fp64 vector roof (VALU-issue bound, scene LDS/cache resident); "
                        "N>1 lines carry no PMC data (traffic null)"
                        if ws == 1 else "N>1: no PMC pass in multi-rank runs (traffic null)")
        return roof

    if cpu:  # the CPU backend's ranks: no kernel, no roof
        roof = {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None,
                "traffic": None, "kernel_ms": round(sum(kernel_ms) / len(kernel_ms), 3),
                "note": "--device cpu: CPU backend ranks (launcher / exchange path), no GPU roof"}
    else:
        roof = gpu_roofline(pmc)

    units_desc = ("library head/tail units, RT_CHUNKS_AUTO" if tiles_mode and shard.library_units
                  else "%d stratum chunks" % shard.chunks if tiles_mode else "")
    out = {
        "metric": BASELINE["metric"],
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": ws,
        "ranks_seen": seen,
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
                   "parallelism": (("1 GPU, tile work units (%s)" % units_desc
                                    if tiles_mode else "1 GPU") if not use_pg else
                                   "tile-shard x%d (tile t on rank t %% %d, %s) + %s gather" % (
                                       ws, ws, units_desc,
                                       "RCCL" if args.backend == "nccl" else "gloo")
                                   if tiles_mode else
                                   "stratum-shard x%d + %s reduce(sum)" % (
                                       ws, "RCCL" if args.backend == "nccl" else "gloo")),
                   "device": "cpu backend (librtx_cpu.so)" if cpu else "gpu",
                   "launcher": os.environ.get("RTX_BENCH_LAUNCHER", "torchrun" if use_pg else None)},
        "roofline": roof,
    }
    if check is not None:
        out["check"] = check
    if diag is not None:
        out["ranks"] = diag
    # rank 0's host time per step in the timed loop: with N>1 the steps are
    # issued without a sync, so the host keeps ahead while this stays below
    # ms_per_step
    out["host_issue_ms_per_step"] = round(host_s * 1e3 / args.steps, 3)
    if rank == 0 and full_line:
        out["other_configs"] = other_configs(args, torch, dev, args.config, pmc_other)
        if not tiles_mode:
            out["host_output"] = host_output(torch, R, frame, max(3, min(args.steps, 10)))
        out["progressive"] = progressive_rates(torch, dev)
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(scene, cam)
    if rank == 0:
        print(json.dumps(out), flush=True)
    R.close()
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
