"""ctypes mirror of include/rt_api.h (the C ABI of the HIP hot path).

Field order and types must match the header exactly; tests/test_abi.py checks
sizes against the compiled library's own view (rt_abi_sizes) when available.
"""
import ctypes as C

RT_ABI_VERSION = 5  # include/rt_api.h; rtx/lib.py refuses a library of another version

RT_OK = 0
RT_ERR_INVALID = -1
RT_ERR_DEVICE = -2
RT_ERR_OOM = -3
RT_ERR_UNSUPPORTED = -4

RT_TEX_SOLID, RT_TEX_CHECKER, RT_TEX_NOISE = 0, 1, 2
RT_MAT_LAMBERTIAN, RT_MAT_METAL, RT_MAT_DIELECTRIC, RT_MAT_DIFFUSE_LIGHT, RT_MAT_ISOTROPIC = range(5)
RT_OBJ_SPHERE, RT_OBJ_QUAD, RT_OBJ_LIST, RT_OBJ_ROTATE_Y, RT_OBJ_TRANSLATE, RT_OBJ_MEDIUM = range(6)
RT_STORED_FORM = 2  # rt_object_desc.moving: sphere displacement / rotate_y (sin, cos) as stored
RT_OUT_SCALED, RT_OUT_SUM = 0, 1
RT_PERLIN_POINTS = 256


class Vec3(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double)]

    @staticmethod
    def of(v):
        return Vec3(float(v[0]), float(v[1]), float(v[2]))

    def tolist(self):
        return [self.x, self.y, self.z]


class TextureDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("even", C.c_int32), ("odd", C.c_int32),
                ("perlin", C.c_int32), ("scale", C.c_double), ("color", Vec3)]


class PerlinDesc(C.Structure):
    _fields_ = [("rand_vec", Vec3 * RT_PERLIN_POINTS),
                ("perm_x", C.c_int32 * RT_PERLIN_POINTS),
                ("perm_y", C.c_int32 * RT_PERLIN_POINTS),
                ("perm_z", C.c_int32 * RT_PERLIN_POINTS)]


class MaterialDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("texture", C.c_int32), ("albedo", Vec3),
                ("fuzz", C.c_double), ("refraction_index", C.c_double)]


class ObjectDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_int32), ("child", C.c_int32),
                ("count", C.c_int32), ("a", Vec3), ("b", Vec3), ("c", Vec3),
                ("s", C.c_double), ("moving", C.c_int32), ("phase", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [("textures", C.POINTER(TextureDesc)), ("n_textures", C.c_int32),
                ("n_perlin", C.c_int32), ("perlin", C.POINTER(PerlinDesc)),
                ("materials", C.POINTER(MaterialDesc)), ("n_materials", C.c_int32),
                ("n_objects", C.c_int32), ("objects", C.POINTER(ObjectDesc)),
                ("children", C.POINTER(C.c_int32)), ("n_children", C.c_int32),
                ("world", C.c_int32), ("lights", C.c_int32), ("use_bvh", C.c_int32),
                ("bvh_builder", C.c_int32), ("bvh_arity", C.c_int32)]


RT_BVH_AUTO, RT_BVH_HOST, RT_BVH_DEVICE, RT_BVH_DEVICE_SAH = 0, 1, 2, 3
# kernel instance bits (rt_scene_info.features)
RT_FEAT_MEDIA, RT_FEAT_XFORM, RT_FEAT_LIGHTS, RT_FEAT_NOISE, RT_FEAT_FLAT, RT_FEAT_BVH4 = 1, 2, 4, 8, 16, 32


class CameraDesc(C.Structure):
    _fields_ = [("image_width", C.c_int32), ("samples_per_pixel", C.c_int32),
                ("max_depth", C.c_int32), ("_pad0", C.c_int32),
                ("aspect_ratio", C.c_double), ("vfov", C.c_double),
                ("defocus_angle", C.c_double), ("focus_dist", C.c_double),
                ("lookfrom", Vec3), ("lookat", Vec3), ("vup", Vec3), ("background", Vec3)]


class Frame(C.Structure):
    _fields_ = [("image_width", C.c_int32), ("image_height", C.c_int32),
                ("sqrt_spp", C.c_int32), ("max_depth", C.c_int32),
                ("center", Vec3), ("pixel00_loc", Vec3), ("pixel_delta_u", Vec3),
                ("pixel_delta_v", Vec3), ("u", Vec3), ("v", Vec3), ("w", Vec3),
                ("defocus_disk_u", Vec3), ("defocus_disk_v", Vec3),
                ("defocus_angle", C.c_double), ("pixel_samples_scale", C.c_double),
                ("background", Vec3)]


class RenderParams(C.Structure):
    _fields_ = [("row_begin", C.c_int32), ("row_end", C.c_int32),
                ("sample_begin", C.c_int32), ("sample_count", C.c_int32),
                ("seed", C.c_uint64), ("output", C.c_int32), ("accumulate", C.c_int32),
                ("tile_first", C.c_int32), ("tile_stride", C.c_int32),
                ("layout", C.c_int32), ("strata_chunks", C.c_int32)]


RT_LAYOUT_FRAME, RT_LAYOUT_TILES = 0, 1
RT_CHUNKS_AUTO = -1  # strata_chunks: the library's units for a tile subset, per-tile sums out


class PathStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "samples", "segments", "node_visits", "sphere_tests", "quad_tests",
        "other_tests", "light_tests", "shade_events",
        "wave_trips", "wave_node_iters", "wave_leaf_iters", "wave_shade_iters",
        "cyc_loop", "cyc_regen", "cyc_trace", "cyc_media", "cyc_shade", "cyc_lights",
        "model_trace_max", "model_trace_pair_max", "noise_evals", "wave_noise_iters",
        "medium_box_tests", "medium_box_deferred")]


class SceneInfo(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("n_leaf_refs", C.c_int32),
                ("n_spheres", C.c_int32), ("n_quads", C.c_int32),
                ("n_objects", C.c_int32), ("n_light_leaves", C.c_int32),
                ("bvh_depth", C.c_int32), ("node_bytes", C.c_int32),
                ("sphere_bytes", C.c_int32), ("quad_bytes", C.c_int32),
                ("device_bytes", C.c_int64), ("features", C.c_int32), ("lds_nodes", C.c_int32),
                ("bvh_builder", C.c_int32), ("bvh_arity", C.c_int32),
                ("stack_depth", C.c_int32), ("lds_fixed_bytes", C.c_int32),
                ("lds_block_budget", C.c_int32), ("waves_per_simd", C.c_int32),
                ("lds_nodes_persistent", C.c_int32), ("lds_prims_persistent", C.c_int32),
                ("persistent_block_waves", C.c_int32), ("lds_perlin", C.c_int32),
                ("lds_node_bytes", C.c_int32)]


class Tuning(C.Structure):
    """rt_tuning: a scene's work-unit plan, LDS staging and BVH-builder
    overrides, passed at creation (zero-filled = the default plan)."""
    _fields_ = [("chunk_target", C.c_int32), ("head_strata", C.c_int32),
                ("tail_split", C.c_int32), ("no_uniform_tail", C.c_int32),
                ("no_persistent", C.c_int32), ("grid_cap", C.c_int32),
                ("tail_tiles", C.c_double),
                ("lds_nodes", C.c_int32), ("lds_nodes_pc", C.c_int32),
                ("no_lds_prims", C.c_int32), ("no_lds_perlin", C.c_int32),
                ("lds_cap", C.c_int32), ("pc_waves", C.c_int32),
                ("sah_stack_budget", C.c_int32), ("lbvh_max_depth", C.c_int32),
                ("sah_leaf_max", C.c_int32), ("sah_leaf_split", C.c_int32),
                ("sah_trav_x4", C.c_int32), ("sah_bins", C.c_int32),
                ("extra_features", C.c_int32),
                ("sub_head_strata", C.c_int32), ("sub_tail_split", C.c_int32),
                ("sub_tail_permille", C.c_int32), ("no_tile_order", C.c_int32),
                ("probe_strata", C.c_int32), ("reserved", C.c_int32 * 2)]


def tuning(t=None):
    """A Tuning from None (the default), a Tuning, or a dict of its fields."""
    if t is None or isinstance(t, Tuning):
        return t
    out = Tuning()
    for k, v in dict(t).items():
        if k not in dict(Tuning._fields_):
            raise KeyError("unknown rt_tuning field %r" % k)
        setattr(out, k, v)
    return out


# Every symbol include/rt_api.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "rt_abi_version", "rt_last_error", "rt_device_count", "rt_camera_setup",
    "rt_scene_create", "rt_scene_info_get", "rt_scene_destroy", "rt_render",
    "rt_render_device", "rt_render_stats", "rt_last_kernel_ms", "rt_to_bytes_device",
    "rt_multi_create", "rt_multi_render", "rt_multi_shard_ms", "rt_multi_destroy",
    "rt_scene_bvh_cost", "rt_tiles_sum_device", "rt_tiles_to_frame_device", "rt_multi_gather_ms",
    "rt_scene_create_tuned", "rt_multi_create_tuned",
)
