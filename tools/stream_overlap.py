#!/usr/bin/env python3
"""Do consecutive launches on two HIP streams (a scene each) overlap on the
device?  (diagnostic) 20 launches of one config's share, alternating two
streams, against 20 on one stream: wall ms per launch and the per-launch
event span; an 8-way rank's share (--n 8) has the longest ragged end.

    python tools/stream_overlap.py --config C2 --n 8"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-ray-tracing-engine_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from rtx import abi  # noqa: E402
from rtx.dist import tile_counts  # noqa: E402
from rtx.render import Renderer, camera_frame  # noqa: E402
from rtx.scene import load_scene  # noqa: E402
from bench import CONFIGS, SCENES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--launches", type=int, default=20)
    a = ap.parse_args()
    name, width, spp, depth = CONFIGS[a.config]
    S = load_scene(os.path.join(SCENES, name + ".json"))
    f = camera_frame(S.camera_desc(image_width=width, samples_per_pixel=spp, max_depth=depth))
    _, t_r = tile_counts(f, a.n)
    Rs = [Renderer(S) for _ in range(2)]
    bufs = [torch.empty((t_r, 64, 3), dtype=torch.float64, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]

    def launch(i, two):
        b = i % 2 if two else 0
        Rs[b].render_device(f, bufs[b].data_ptr(), streams[b].cuda_stream, seed=i, output=abi.RT_OUT_SUM,
                            accumulate=0, tiles=(0, a.n), layout=abi.RT_LAYOUT_TILES,
                            chunks=abi.RT_CHUNKS_AUTO)

    for two in (False, True, False, True):
        for i in range(4):
            launch(i, True)  # warm both scenes (tile order)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.launches):
            launch(i, two)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.launches
        print(json.dumps({"config": a.config, "n": a.n, "streams": 2 if two else 1,
                          "wall_ms_per_launch": round(ms, 4),
                          "last_kernel_ms": [round(R.last_kernel_ms(), 4) for R in Rs]}), flush=True)


if __name__ == "__main__":
    main()
