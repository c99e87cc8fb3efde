#!/usr/bin/env python3
"""Timeline of one launch's work units (diagnostic; needs the measurement-only
build `make BUILD=build_dbgT EXTRA=-DRT_UNIT_TIMES=1`, loaded with RTX_LIB).

Each unit's start / end on the device's 100 MHz clock gives: the launch span,
the unit durations, and how busy the wave slots are over the span -- the
share of slot-time doing units (1 - idle), and the span's last stretch where
fewer than 90 % / 50 % of the slots still run a unit (the tail).

    RTX_LIB=.../build_dbgT/librtx_hip.so python tools/unit_timeline.py --config C2 --n 8 --plan auto
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-ray-tracing-engine_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from rtx import abi  # noqa: E402
from rtx.dist import auto_chunks, tile_counts  # noqa: E402
from rtx.lib import load  # noqa: E402
from rtx.render import Renderer, camera_frame  # noqa: E402
from rtx.scene import load_scene  # noqa: E402
from bench import CONFIGS, SCENES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--n", type=int, default=8, help="ranks of the tile split (1: the frame launch)")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--plan", default="auto", choices=["auto", "chunks"])
    a = ap.parse_args()
    L = load()
    L.rtk_unit_times.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    name, width, spp, depth = CONFIGS[a.config]
    S = load_scene(os.path.join(SCENES, name + ".json"))
    f = camera_frame(S.camera_desc(image_width=width, samples_per_pixel=spp, max_depth=depth))
    n, t_r = tile_counts(f, a.n)
    with Renderer(S) as R:
        slots = R.info()["waves_per_simd"] * 4 * torch.cuda.get_device_properties(0).multi_processor_count
        if a.n == 1:
            buf = torch.empty((f.image_height, f.image_width, 3), dtype=torch.float64, device="cuda")
            run = lambda: R.render_device(f, buf.data_ptr(), 0, output=abi.RT_OUT_SUM, accumulate=0)  # noqa: E731
        else:
            ch = abi.RT_CHUNKS_AUTO if a.plan == "auto" else auto_chunks(f, a.n)
            shape = (t_r, 64, 3) if a.plan == "auto" else (t_r, ch, 64, 3)
            buf = torch.empty(shape, dtype=torch.float64, device="cuda")
            run = lambda: R.render_device(f, buf.data_ptr(), 0, output=abi.RT_OUT_SUM, accumulate=0,  # noqa: E731
                                          tiles=(a.rank, a.n), layout=abi.RT_LAYOUT_TILES, chunks=ch)
        run()
        torch.cuda.synchronize()
        assert L.rtk_unit_times_clear() == 0
        run()
        torch.cuda.synchronize()
        ms = R.last_kernel_ms()
    cap = 1 << 21
    t = np.zeros(2 * cap, dtype=np.uint64)
    assert L.rtk_unit_times(t.ctypes.data_as(C.POINTER(C.c_ulonglong)), cap) == 0
    t = t.reshape(-1, 2)
    used = np.nonzero(t[:, 1])[0]
    t = t[used].astype(np.int64)
    t0 = t[:, 0].min()
    st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # us
    span = en.max()
    dur = en - st
    # busy slots over time (1 us bins)
    bins = int(np.ceil(span)) + 1
    busy = np.zeros(bins)
    for s_, e_ in zip(st, en):
        busy[int(s_):int(np.ceil(e_))] += 1
    busy = np.minimum(busy, slots)
    peak = busy.max()
    last90 = span - np.nonzero(busy >= 0.9 * peak)[0].max()
    last50 = span - np.nonzero(busy >= 0.5 * peak)[0].max()
    print(json.dumps({
        "config": a.config, "n": a.n, "rank": a.rank, "plan": a.plan if a.n > 1 else "frame",
        "units": int(len(t)), "wave_slots": int(slots), "kernel_ms": round(ms, 4),
        "span_us": round(float(span), 1), "busy_peak": int(peak),
        "slot_time_used": round(float(dur.sum() / (peak * span)), 4),
        "tail_below_90pct_us": round(float(last90), 1), "tail_below_50pct_us": round(float(last50), 1),
        "unit_us_mean": round(float(dur.mean()), 1), "unit_us_p50": round(float(np.median(dur)), 1),
        "unit_us_p99": round(float(np.percentile(dur, 99)), 1), "unit_us_max": round(float(dur.max()), 1),
        "last_start_us": round(float(st.max()), 1)}), flush=True)


if __name__ == "__main__":
    main()
