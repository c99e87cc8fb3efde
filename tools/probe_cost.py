#!/usr/bin/env python3
"""Wall time of a launch shape's first launch (the probe that orders its tiles
+ the render) against its later launches, per probe size (rt_tuning
probe_strata): what cost-ordered dispatch costs a one-shot render.
  python tools/probe_cost.py --config C2 --probe 1 4 16"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "real-time-ray-tracing-engine_amd"))
import torch  # noqa: E402  (first: torch and the library share one HIP runtime)
from rtx import abi  # noqa: E402
from rtx.render import Renderer, camera_frame  # noqa: E402
from rtx.scene import load_scene  # noqa: E402

CONFIGS = {"C2": ("three_spheres", 64), "C3": ("bouncing_seed42", 256), "C4": ("cornell_fog", 1024)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--probe", type=int, nargs="+", default=[16])
    ap.add_argument("--repeat", type=int, default=5)
    a = ap.parse_args()
    name, spp = CONFIGS[a.config]
    S = load_scene(os.path.join(os.path.dirname(HERE), "real-time-ray-tracing-engine_amd", "scenes", name + ".json"))
    f = camera_frame(S.camera_desc(image_width=1920, samples_per_pixel=spp, max_depth=8))
    out = torch.empty((f.image_height, f.image_width, 3), dtype=torch.float64, device="cuda")
    for p in [0] + a.probe:  # 0 here: no_tile_order (plan order, no probe)
        tune = {"no_tile_order": 1} if p == 0 else {"probe_strata": p}
        with Renderer(S, tuning=tune) as R:
            ms = []
            for k in range(a.repeat + 1):
                torch.cuda.synchronize()
                t = time.perf_counter()
                R.render_device(f, out.data_ptr(), 0, seed=k, output=abi.RT_OUT_SUM, accumulate=0)
                torch.cuda.synchronize()
                ms.append((time.perf_counter() - t) * 1e3)
        later = sorted(ms[1:])[len(ms[1:]) // 2]
        print("%s probe_strata %s: first launch %.3f ms, later launches (median) %.3f ms, first - later %.3f ms"
              % (a.config, p if p else "none (plan order)", ms[0], later, ms[0] - later), flush=True)


if __name__ == "__main__":
    main()
