#!/usr/bin/env python3
"""Per-rank device time of an N-way split, measured on ONE GPU (diagnostic).

For N in 1, 2, 4, 8 renders EVERY rank's share under tile sharding (tile t on
rank t % N; --plan auto, the default: the library's own work units per share,
RT_CHUNKS_AUTO -- bench.py's N>1 default; --plan chunks: uniform stratum
chunks per --units target) and optionally under stratum sharding
(--strata-sharding), each the best of `reps` launches, and adds the library kernels the
N>1 timed region runs besides the render: each rank's chunk sum
(rt_tiles_sum_device) and, on rank 0, the tile -> frame reorder
(rt_tiles_to_frame_device).  Prints the slowest rank's time, the compute-only
speedup t(1) / max(rank) and the gather payload per rank, and prices the RCCL
gather: 1/N of the frame per rank, every rank on its own xGMI link into rank 0
at --link-gbs (default 64 GB/s one way, a conservative share of a link's ~76
GB/s per direction): `gather_ms`.  bench.py double-buffers, so the gather of
frame k overlaps frame k+1's render; what a K-step timed region cannot hide
is the last frame's gather, `speedup_k` = t(1) / (max(rank) + gather / K) for
K = 20 (the driver's step count).  Rank 0's path-trip lane use (STATS: the
share of lane slots of the path loop with a live path; a unit's end drains
it) is reported per N.

    python tools/shard_sim.py [--config C2] [--reps 3] [--n 1 2 4 8] [--units U ...]
(--units: work-unit targets of the chunk choice, rtx.dist.auto_chunks; one
line per N and target)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-ray-tracing-engine_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from rtx import abi  # noqa: E402
from rtx.dist import auto_chunks, device_tiles_sum, device_tiles_to_frame, tile_counts  # noqa: E402
from rtx.render import Renderer, camera_frame  # noqa: E402
from rtx.scene import load_scene  # noqa: E402
from bench import CONFIGS, SCENES  # noqa: E402


def timed(fn, reps):
    """Best of `reps` device times (ms) of fn() on the current stream."""
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1)
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--units", type=int, nargs="+", default=[None])
    ap.add_argument("--link-gbs", type=float, default=64.0)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--rank-order", default="fwd", choices=["fwd", "rev"],
                    help="order the ranks' shares are timed in (rev: a check that the "
                         "per-rank spread is content, not the GPU's clock history)")
    ap.add_argument("--rank-work", action="store_true",
                    help="also report each rank's path segments and wave trips (STATS)")
    ap.add_argument("--plan", default="auto", choices=["chunks", "auto"],
                    help="chunks: every tile in rtx.dist.auto_chunks chunks + the chunk sum "
                         "(--units); auto: strata_chunks = RT_CHUNKS_AUTO, the library's "
                         "head/tail units for the subset, tile sums out")
    ap.add_argument("--tuning", nargs="+", default=[None],
                    help="rt_tuning dicts as JSON (one scene per entry), e.g. "
                         "'{\"sub_head_strata\": 32}'")
    ap.add_argument("--settle", type=int, default=1,
                    help="untimed launches of a share before its timed one (a rank's steady state)")
    ap.add_argument("--strata-sharding", action="store_true",
                    help="also time the stratum-sharded split")
    a = ap.parse_args()
    name, width, spp, depth = CONFIGS[a.config]
    S = load_scene(os.path.join(SCENES, name + ".json"))
    f = camera_frame(S.camera_desc(image_width=width, samples_per_pixel=spp, max_depth=depth))
    strata = f.sqrt_spp ** 2
    frame = torch.empty((f.image_height, f.image_width, 3), dtype=torch.float64, device="cuda")
    for tj in a.tuning:
        tune = json.loads(tj) if tj else None
        with Renderer(S, tuning=tune) as R:
            t1 = timed(lambda: R.render_device(f, frame.data_ptr(), 0, output=abi.RT_OUT_SUM,
                                               accumulate=0), a.reps)
            units = a.units if a.plan == "chunks" else [None]
            for N, U in [(N, U) for N in a.n for U in units]:
                print(json.dumps(dict(case(a, R, f, frame, strata, t1, N, U), tuning=tune)), flush=True)


def case(a, R, f, frame, strata, t1, N, U):
    n, t_r = tile_counts(f, N)
    auto = a.plan == "auto"
    ch = abi.RT_CHUNKS_AUTO if auto else auto_chunks(f, N, U)
    sums = torch.empty((t_r, 64, 3), dtype=torch.float64, device="cuda")
    buf = sums if auto else torch.empty((t_r, ch, 64, 3), dtype=torch.float64, device="cuda")
    gath = torch.zeros((N, t_r, 64, 3), dtype=torch.float64, device="cuda")

    def share(r):
        R.render_device(f, buf.data_ptr(), 0, output=abi.RT_OUT_SUM, accumulate=0,
                        tiles=(r, N), layout=abi.RT_LAYOUT_TILES, chunks=ch)
        if not auto and ch > 1:
            device_tiles_sum(buf, sums)

    # rounds over the ranks, each share launched untimed and then timed: a
    # rank renders its own share launch after launch, so its timed launch
    # follows one of the same shape (tile order from that launch's costs);
    # the best of the rounds per rank (the first share timed after a change
    # of shape otherwise reads slow -- r05m: the same rank fast in reverse order)
    per_rank = [None] * N
    for _ in range(a.reps):
        for r in (range(N) if a.rank_order == "fwd" else range(N - 1, -1, -1)):
            for _ in range(a.settle):
                share(r)
            t = timed(lambda: share(r), 1)  # render + chunk sum
            per_rank[r] = t if per_rank[r] is None else min(per_rank[r], t)
    t_frame = timed(lambda: device_tiles_to_frame(gath, f, frame), a.reps)
    tiles_max = max(per_rank[0] + t_frame, max(per_rank))
    gbytes = t_r * 64 * 3 * 8
    gather = 0.0 if N == 1 else gbytes / (a.link_gbs * 1e9) * 1e3
    st0 = R.stats(f, seed=0, tiles=(0, N), layout=abi.RT_LAYOUT_TILES, chunks=ch)
    out = {
        "config": a.config, "N": N, "t1_ms": round(t1, 3), "plan": a.plan,
        "units_target": U, "tiles_chunks": "library" if auto else ch,
        "tiles_rank_ms": [round(x, 3) for x in per_rank],
        "tiles_chunk_sum_ms": "included per rank",
        "tiles_reorder_ms_rank0": round(t_frame, 3),
        "tiles_ms": round(tiles_max, 3), "tiles_speedup": round(t1 / tiles_max, 2),
        "gather_bytes_per_rank": gbytes, "gather_ms": round(gather, 3),
        "speedup_k": round(t1 / (tiles_max + gather / a.k), 2),
        "rank0_path_trip_lane_use": round(st0["segments"] / max(1, 64 * st0["wave_trips"]), 4),
        "rank_order": a.rank_order, "settle": a.settle}
    if a.rank_work:
        sts = [st0] + [R.stats(f, seed=0, tiles=(r, N), layout=abi.RT_LAYOUT_TILES, chunks=ch)
                       for r in range(1, N)]
        out.update(rank_segments=[x["segments"] for x in sts],
                   rank_wave_trips=[x["wave_trips"] for x in sts])
    if a.strata_sharding:
        st = []
        for r in range(N):
            b, e = r * strata // N, (r + 1) * strata // N
            st.append(timed(lambda: R.render_device(f, frame.data_ptr(), 0, samples=(b, e - b),
                                                    output=abi.RT_OUT_SUM, accumulate=0), a.reps))
        out.update(strata_rank_ms=[round(x, 3) for x in st], strata_ms=round(max(st), 3),
                   strata_speedup=round(t1 / max(st), 2))
    return out


if __name__ == "__main__":
    main()
