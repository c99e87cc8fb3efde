"""Host-side mirror of the reference's StaticCamera for the HIP path.

    StaticCamera(config, out).render(world, lights)   (StaticCamera.cpp:25-30)
 -> Renderer(scene).render(camera) / render_ppm(...)

Camera setup, scene upload, the render launch and the PPM writer are the
reference's steps; the per-pixel work runs in the HIP kernel behind the C ABI.
"""
import ctypes as C

import numpy as np

from . import abi
from .lib import check, load
from .ppm import write_ppm


def camera_frame(cam):
    """Camera::initialize (Camera.cpp:31-73) via rt_camera_setup."""
    f = abi.Frame()
    check(load().rt_camera_setup(C.byref(cam), C.byref(f)))
    return f


class Renderer:
    """Owns one device-side scene (rt_scene) on one GPU.  `tuning`: None (the
    default plan), an abi.Tuning or a dict of its fields (rt_scene_create_tuned)."""

    def __init__(self, scene, device=0, tuning=None):
        self.lib = load()
        self.scene_desc = scene
        self._desc = scene.desc()
        self._tuning = abi.tuning(tuning)
        h = C.c_void_p()
        t = C.byref(self._tuning) if self._tuning is not None else None
        check(self.lib.rt_scene_create_tuned(C.byref(self._desc), int(device), t, C.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            self.lib.rt_scene_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        i = abi.SceneInfo()
        check(self.lib.rt_scene_info_get(self.handle, C.byref(i)))
        return {k: getattr(i, k) for k, _ in abi.SceneInfo._fields_}

    @staticmethod
    def params(seed=0, rows=(0, 0), samples=(0, -1), output=abi.RT_OUT_SCALED, accumulate=0,
               tiles=(0, 1), layout=abi.RT_LAYOUT_FRAME, chunks=1):
        p = abi.RenderParams()
        p.row_begin, p.row_end = int(rows[0]), int(rows[1])
        p.sample_begin, p.sample_count = int(samples[0]), int(samples[1])
        p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        p.output = int(output)
        p.accumulate = int(accumulate)
        p.tile_first, p.tile_stride = int(tiles[0]), int(tiles[1])
        p.layout = int(layout)
        p.strata_chunks = int(chunks)
        return p

    @staticmethod
    def local_tiles(frame, rows=(0, 0), tiles=(0, 1)):
        """Number of 8x8 tiles a launch with this tile subset renders."""
        r0, r1 = rows
        if r0 == 0 and r1 == 0:
            r1 = frame.image_height
        n = ((frame.image_width + 7) // 8) * ((r1 - r0 + 7) // 8)
        first, stride = tiles[0], max(1, tiles[1])
        return max(0, (n - first + stride - 1) // stride)

    def render(self, frame, seed=0, rows=(0, 0), samples=(0, -1), output=abi.RT_OUT_SCALED,
               tiles=(0, 1), layout=abi.RT_LAYOUT_FRAME, chunks=1):
        """Synchronous render -> float64 array [rows, W, 3] (frame layout),
        [tiles, 64, 3] (tile layout) or [tiles, chunks, 64, 3] (chunks > 1), on
        the host."""
        r0, r1 = rows
        if r0 == 0 and r1 == 0:  # the ABI's "whole image"
            r1 = frame.image_height
        if layout == abi.RT_LAYOUT_TILES:
            n = self.local_tiles(frame, rows, tiles)
            shape = (n, 64, 3) if chunks <= 1 else (n, chunks, 64, 3)
            out = np.zeros(shape, dtype=np.float64)
        else:
            out = np.empty((max(0, r1 - r0), frame.image_width, 3), dtype=np.float64)
        p = self.params(seed, (r0, r1), samples, output, 0, tiles, layout, chunks)
        check(self.lib.rt_render(self.handle, C.byref(frame), C.byref(p),
                                 out.ctypes.data_as(C.POINTER(C.c_double))))
        return out

    def render_into(self, frame, host_ptr, seed=0, rows=(0, 0), samples=(0, -1),
                    output=abi.RT_OUT_SCALED):
        """rt_render into caller host memory at `host_ptr` (e.g. a pinned torch
        tensor's data_ptr(), or a numpy buffer's address): kernel + D2H copy,
        synchronous -- the reference's render_gpu batch loop."""
        p = self.params(seed, rows, samples, output, 0)
        check(self.lib.rt_render(self.handle, C.byref(frame), C.byref(p),
                                 C.cast(C.c_void_p(host_ptr), C.POINTER(C.c_double))))

    def render_device(self, frame, dev_ptr, stream_ptr=None, seed=0, rows=(0, 0), samples=(0, -1),
                      output=abi.RT_OUT_SUM, accumulate=1, tiles=(0, 1), layout=abi.RT_LAYOUT_FRAME,
                      chunks=1):
        """Asynchronous render into a device buffer (e.g. a torch.cuda tensor's
        data_ptr()) on `stream_ptr` (0/None = the HIP null stream)."""
        p = self.params(seed, rows, samples, output, accumulate, tiles, layout, chunks)
        check(self.lib.rt_render_device(self.handle, C.byref(frame), C.byref(p),
                                        C.c_void_p(dev_ptr), C.c_void_p(stream_ptr or 0)))

    def stats(self, frame, seed=0, rows=(0, 0), samples=(0, -1), tiles=(0, 1),
              layout=abi.RT_LAYOUT_FRAME, chunks=1):
        s = abi.PathStats()
        p = self.params(seed, rows, samples, tiles=tiles, layout=layout, chunks=chunks)
        check(self.lib.rt_render_stats(self.handle, C.byref(frame), C.byref(p), C.byref(s)))
        return {k: getattr(s, k) for k, _ in abi.PathStats._fields_}

    def bvh_cost(self):
        """SAH cost of the world BVH relative to the root box (rt_scene_bvh_cost)."""
        c = C.c_double()
        check(self.lib.rt_scene_bvh_cost(self.handle, C.byref(c)))
        return c.value

    def last_kernel_ms(self):
        ms = C.c_double()
        check(self.lib.rt_last_kernel_ms(self.handle, C.byref(ms)))
        return ms.value


class MultiRenderer:
    """rt_multi_*: one device scene per shard (shard k on devices[k % len]),
    one host thread per shard, 8x8 tiles dealt round-robin; the multi-device
    form of StaticCamera::render_gpu (StaticCamera.cpp:136-313)."""

    def __init__(self, scene, devices=(0,), shards=None, tuning=None):
        self.lib = load()
        self._desc = scene.desc()
        self._tuning = abi.tuning(tuning)
        devs = (C.c_int32 * len(devices))(*devices)
        self.n_shards = int(shards or len(devices))
        h = C.c_void_p()
        t = C.byref(self._tuning) if self._tuning is not None else None
        check(self.lib.rt_multi_create_tuned(C.byref(self._desc), devs, len(devices),
                                             self.n_shards, t, C.byref(h)))
        self.handle = h

    def close(self):
        if self.handle:
            self.lib.rt_multi_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def render(self, frame, seed=0, rows=(0, 0), samples=(0, -1), output=abi.RT_OUT_SCALED,
               chunks=0):
        r0, r1 = rows
        if r0 == 0 and r1 == 0:
            r1 = frame.image_height
        out = np.empty((max(0, r1 - r0), frame.image_width, 3), dtype=np.float64)
        p = Renderer.params(seed, (r0, r1), samples, output, 0, (0, 1), abi.RT_LAYOUT_FRAME, chunks)
        check(self.lib.rt_multi_render(self.handle, C.byref(frame), C.byref(p),
                                       out.ctypes.data_as(C.POINTER(C.c_double))))
        return out

    def shard_ms(self):
        ms = (C.c_double * self.n_shards)()
        check(self.lib.rt_multi_shard_ms(self.handle, ms))
        return list(ms)

    def gather_ms(self):
        """Host ms of the last render's device exchange (slowest shard's render
        end -> frame assembled on shard 0's device; D2H excluded)."""
        ms = C.c_double()
        check(self.lib.rt_multi_gather_ms(self.handle, C.byref(ms)))
        return ms.value


def render_ppm(scene, path, device=0, seed=0, **cam_overrides):
    """StaticCamera::render on the HIP path: camera setup, render, PPM."""
    cam = scene.camera_desc(**cam_overrides)
    frame = camera_frame(cam)
    with Renderer(scene, device) as R:
        img = R.render(frame, seed=seed)
    write_ppm(path, img)
    return img
