#!/usr/bin/env python3
"""rt_multi_render vs rt_render on one GPU.

Virtual shards on device 0 run the multi-GPU code path: shard threads, the
per-shard device chunk sum, the device-to-device copies of the compact tiles
to shard 0's device, the device reorder and the one D2H copy.  Prints per
configuration: rt_render ms per frame (kernel + D2H), rt_multi_render ms per
frame, the exchange ms (rt_multi_gather_ms: slowest shard's render end ->
frame assembled on shard 0's device) and the shard kernel ms.

    python tools/multi_gather.py [--config C2] [--shards 2 4 8] [--frames 5]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-ray-tracing-engine_amd"))

CONFIGS = {"C2": ("three_spheres", 1920, 64), "C3": ("bouncing_seed42", 1920, 256),
           "C4": ("cornell_fog", 1920, 1024)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--shards", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--frames", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    from rtx.render import MultiRenderer, Renderer, camera_frame
    from rtx.scene import load_scene
    name, width, spp = CONFIGS[a.config]
    S = load_scene(os.path.join(ROOT, "real-time-ray-tracing-engine_amd", "scenes", name + ".json"))
    f = camera_frame(S.camera_desc(image_width=width, samples_per_pixel=spp, max_depth=8))
    with Renderer(S, device=0) as R:
        one = R.render(f, seed=1)
        t0 = time.perf_counter()
        for k in range(a.frames):
            R.render(f, seed=k)
        ms1 = (time.perf_counter() - t0) * 1e3 / a.frames
        kms = R.last_kernel_ms()
    print("%s %dx%d spp %d: rt_render %.3f ms/frame (kernel %.3f ms)" % (
        a.config, f.image_width, f.image_height, spp, ms1, kms), flush=True)
    for n in a.shards:
        with MultiRenderer(S, devices=(0,), shards=n) as M:
            got = M.render(f, seed=1)
            same = bool(np.array_equal(got, one))
            g, t = [], time.perf_counter()
            for k in range(a.frames):
                M.render(f, seed=k)
                g.append(M.gather_ms())
            ms = (time.perf_counter() - t) * 1e3 / a.frames
            sh = M.shard_ms()
        print("  %d virtual shards: rt_multi_render %.3f ms/frame, exchange %.3f ms "
              "(min %.3f, max %.3f), shard kernels %.3f-%.3f ms, bit-identical %s" % (
                  n, ms, sum(g) / len(g), min(g), max(g), min(sh), max(sh), same), flush=True)


if __name__ == "__main__":
    main()
