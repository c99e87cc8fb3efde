#!/usr/bin/env python3
"""World-BVH build: host binned SAH vs device LBVH (rt_bvh_build.hip) vs device
binned SAH (rt_bvh_sah.hip), each walked as a binary or a 4-wide BVH.

For N random spheres: rt_scene_create time (compile + upload + build) with each
builder, the tree depth, and the render rate through each tree (1920x1080,
spp 4, depth 8).
  python tools/bvh_build_bench.py [--n 100000 500000] [--arity 2 4] [--builders device_sah]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-ray-tracing-engine_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from rtx import abi  # noqa: E402
from rtx.render import Renderer, camera_frame  # noqa: E402
from rtx.scene import SceneDescription  # noqa: E402


def scene(n, seed=1):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-100, 100, size=(n, 3))
    r = rng.uniform(0.05, 0.6, size=n)
    S = SceneDescription()
    t = S.add_texture(abi.RT_TEX_SOLID, color=(0.6, 0.5, 0.4))
    mats = [S.add_material(abi.RT_MAT_LAMBERTIAN, texture=t),
            S.add_material(abi.RT_MAT_METAL, albedo=(0.8, 0.7, 0.6), fuzz=0.1),
            S.add_material(abi.RT_MAT_DIELECTRIC, refraction_index=1.5)]
    ids = [S.add_object(abi.RT_OBJ_SPHERE, material=mats[k % 3], a=tuple(c[k]), s=float(r[k]))
           for k in range(n)]
    S.world = S.add_list(ids)
    S.camera = {"aspect_ratio": 16 / 9, "vfov": 50.0, "lookfrom": [0, 40, 230], "lookat": [0, 0, 0],
                "background": [0.7, 0.8, 1.0]}
    return S


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[100000, 500000])
    ap.add_argument("--arity", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--builders", nargs="+", default=["host_sah", "device_lbvh", "device_sah"])
    a = ap.parse_args()
    by_name = {"host_sah": abi.RT_BVH_HOST, "device_lbvh": abi.RT_BVH_DEVICE,
               "device_sah": abi.RT_BVH_DEVICE_SAH}
    for n in a.n:
        S = scene(n)
        cam = S.camera_desc(image_width=1920, samples_per_pixel=4, max_depth=8)
        f = camera_frame(cam)
        buf = torch.zeros((f.image_height, f.image_width, 3), dtype=torch.float64, device="cuda")
        for b, ar in [(by_name[x], ar) for x in a.builders for ar in a.arity]:
            S.bvh_builder = b
            S.bvh_arity = ar
            S.desc()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            R = Renderer(S)
            t_create = time.perf_counter() - t0
            info = R.info()
            R.render_device(f, buf.data_ptr(), 0, seed=1, output=abi.RT_OUT_SUM, accumulate=0)
            torch.cuda.synchronize()
            ms = []
            for k in range(3):
                R.render_device(f, buf.data_ptr(), 0, seed=2 + k, output=abi.RT_OUT_SUM, accumulate=0)
                torch.cuda.synchronize()
                ms.append(R.last_kernel_ms())
            cost = R.bvh_cost()
            R.close()
            name = {abi.RT_BVH_HOST: "host_sah", abi.RT_BVH_DEVICE: "device_lbvh",
                    abi.RT_BVH_DEVICE_SAH: "device_sah"}[b]
            print(json.dumps({"n": n, "builder": name, "built_by": info["bvh_builder"],
                              "arity": info["bvh_arity"], "lds_nodes": info["lds_nodes"],
                              "create_s": round(t_create, 4), "bvh_depth": info["bvh_depth"],
                              "nodes": info["n_nodes"], "sah_cost": round(cost, 2),
                              "render_Msamples_s": round(f.image_width * f.image_height * 4 / min(ms) / 1e3, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
