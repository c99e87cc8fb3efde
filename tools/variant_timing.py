#!/usr/bin/env python3
"""Time scene variants on the GPU to attribute kernel cost (diagnostic only).

    python tools/variant_timing.py [--spp 64] [--width 1920]

Each variant is a modified copy of a bench scene; prints Msamples/s, kernel ms
and the kernel instance (feature bits) the library picked."""
import argparse
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-ray-tracing-engine_amd"))
import torch  # noqa: E402,F401  (HIP runtime first)
from rtx import abi  # noqa: E402
from rtx.render import Renderer, camera_frame  # noqa: E402
from rtx.scene import load_scene  # noqa: E402

SC = os.path.join(ROOT, "real-time-ray-tracing-engine_amd", "scenes")


def variants():
    fog = json.load(open(os.path.join(SC, "cornell_fog.json")))
    out = {"fog": fog}
    v = copy.deepcopy(fog)
    v["textures"]["fog"] = {"type": "solid", "color": [0.5, 0.5, 0.5]}
    out["fog_solid_tex"] = v
    v = copy.deepcopy(fog)
    v["world"] = [o for o in v["world"] if o["type"] != "constant_medium"]
    out["no_medium"] = v
    v = copy.deepcopy(out["no_medium"])
    v["lights"] = None
    out["no_medium_no_lights"] = v
    v = copy.deepcopy(fog)
    v["lights"] = None
    out["fog_no_lights"] = v
    out["bouncing"] = json.load(open(os.path.join(SC, "bouncing_seed42.json")))
    out["three_spheres"] = json.load(open(os.path.join(SC, "three_spheres.json")))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    for name, doc in variants().items():
        if a.only and name not in a.only.split(","):
            continue
        S = load_scene(doc)
        cam = S.camera_desc(image_width=a.width, samples_per_pixel=a.spp, max_depth=8)
        f = camera_frame(cam)
        buf = torch.zeros((f.image_height, f.image_width, 3), dtype=torch.float64, device="cuda")
        with Renderer(S) as R:
            st = torch.cuda.current_stream().cuda_stream
            R.render_device(f, buf.data_ptr(), st, seed=1, output=abi.RT_OUT_SUM, accumulate=0)
            torch.cuda.synchronize()
            ms = []
            for k in range(3):
                R.render_device(f, buf.data_ptr(), st, seed=2 + k, output=abi.RT_OUT_SUM, accumulate=0)
                torch.cuda.synchronize()
                ms.append(R.last_kernel_ms())
            stats = R.stats(f, seed=2)
            info = R.info()
        n = f.image_width * f.image_height * f.sqrt_spp ** 2
        best = min(ms)
        print(json.dumps({"variant": name, "features": info["features"],
                          "Msamples_s": round(n / best / 1e3, 1), "kernel_ms": round(best, 3),
                          "seg_per_sample": round(stats["segments"] / stats["samples"], 3),
                          "nodes_per_seg": round(stats["node_visits"] / stats["segments"], 2),
                          "quads_per_seg": round(stats["quad_tests"] / stats["segments"], 2),
                          "spheres_per_seg": round(stats["sphere_tests"] / stats["segments"], 2),
                          "media_per_seg": round(stats["other_tests"] / stats["segments"], 2),
                          "lights_per_seg": round(stats["light_tests"] / stats["segments"], 2)}),
              flush=True)


if __name__ == "__main__":
    main()
