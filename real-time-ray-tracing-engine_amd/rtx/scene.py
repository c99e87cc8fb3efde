"""JSON scene files -> the flat rt_scene_desc / rt_camera_desc of include/rt_api.h.

The reference hard-codes its scenes in C++ (src/main.cpp:21-131) and only claims
JSON input (README.md:18); this module defines that surface.  Every JSON object
type maps one to one onto a reference class:

  sphere           Sphere(center, r, mat) / Sphere(c0, c1, r, mat)   Sphere.cpp:8-23
  quad             Plane(Q, u, v, mat)                                Plane.cpp:6-21
  box              make_box(a, b, mat) -> list of 6 quads             PlaneUtility.hpp:11-39
  list             HittableList                                       HittableList.cpp
  rotate_y         RotateY(object, angle_degrees)                     RotateY.cpp:5-35
  translate        Translate(object, offset)                          Translate.cpp:7-10
  constant_medium  ConstantMedium(boundary, density, texture|albedo)  ConstantMedium.cpp:7-21

Materials: lambertian (albedo | texture), metal (albedo, fuzz), dielectric
(refraction_index), diffuse_light (emit | texture), isotropic (albedo | texture).
Textures: solid (color), checker (scale, even, odd), noise (scale, perlin).
"""
import copy
import ctypes as C
import json
import math

from . import abi


class SceneError(ValueError):
    pass


def _v3(x, what="vector"):
    if not isinstance(x, (list, tuple)) or len(x) != 3:
        raise SceneError("%s must be a 3-element list, got %r" % (what, x))
    return [float(x[0]), float(x[1]), float(x[2])]


DEFAULT_CAMERA = {
    # CameraConfig.hpp:12-35 defaults
    "image_width": 600, "samples_per_pixel": 10, "max_depth": 10,
    "aspect_ratio": 1.0, "vfov": 90.0, "defocus_angle": 0.0, "focus_dist": 10.0,
    "lookfrom": [0.0, 0.0, 0.0], "lookat": [0.0, 0.0, -1.0], "vup": [0.0, 1.0, 0.0],
    "background": [0.0, 0.0, 0.0],
}


def camera_desc(cam):
    c = dict(DEFAULT_CAMERA)
    c.update(cam or {})
    d = abi.CameraDesc()
    d.image_width = int(c["image_width"])
    d.samples_per_pixel = int(c["samples_per_pixel"])
    d.max_depth = int(c["max_depth"])
    d.aspect_ratio = float(c["aspect_ratio"])
    d.vfov = float(c["vfov"])
    d.defocus_angle = float(c["defocus_angle"])
    d.focus_dist = float(c["focus_dist"])
    d.lookfrom = abi.Vec3.of(_v3(c["lookfrom"], "lookfrom"))
    d.lookat = abi.Vec3.of(_v3(c["lookat"], "lookat"))
    d.vup = abi.Vec3.of(_v3(c["vup"], "vup"))
    d.background = abi.Vec3.of(_v3(c["background"], "background"))
    if d.image_width < 1 or d.samples_per_pixel < 1 or d.max_depth < 0:
        raise SceneError("camera: image_width/samples_per_pixel must be >= 1")
    return d


def make_box_quads(a, b):
    """make_box (PlaneUtility.hpp:11-39): the 6 sides as (Q, u, v)."""
    mn = [min(a[0], b[0]), min(a[1], b[1]), min(a[2], b[2])]
    mx = [max(a[0], b[0]), max(a[1], b[1]), max(a[2], b[2])]
    dx = [mx[0] - mn[0], 0.0, 0.0]
    dy = [0.0, mx[1] - mn[1], 0.0]
    dz = [0.0, 0.0, mx[2] - mn[2]]
    neg = lambda v: [-v[0], -v[1], -v[2]]
    return [
        ([mn[0], mn[1], mx[2]], dx, dy),       # front
        ([mx[0], mn[1], mx[2]], neg(dz), dy),  # right
        ([mx[0], mn[1], mn[2]], neg(dx), dy),  # back
        ([mn[0], mn[1], mn[2]], dz, dy),       # left
        ([mn[0], mx[1], mx[2]], dx, neg(dz)),  # top
        ([mn[0], mn[1], mn[2]], dx, dz),       # bottom
    ]


class SceneDescription:
    """Owns the ctypes arrays behind one rt_scene_desc."""

    def __init__(self):
        self.textures = []
        self.perlin = []
        self.materials = []
        self.objects = []
        self.children = []
        self.world = -1
        self.lights = -1
        self.use_bvh = 0
        self.bvh_builder = abi.RT_BVH_AUTO
        self.bvh_arity = 0  # 0 auto, 2 or 4
        self.camera = None
        self._named_tex = {}
        self._named_mat = {}
        self._named_perlin = {}
        self._keep = None

    # ---- builders
    def add_texture(self, kind, color=(0, 0, 0), scale=0.0, even=-1, odd=-1, perlin=-1):
        t = abi.TextureDesc()
        t.kind, t.even, t.odd, t.perlin, t.scale = kind, even, odd, perlin, float(scale)
        t.color = abi.Vec3.of(color)
        self.textures.append(t)
        return len(self.textures) - 1

    def add_material(self, kind, texture=-1, albedo=(0, 0, 0), fuzz=0.0, refraction_index=1.0):
        m = abi.MaterialDesc()
        m.kind, m.texture = kind, texture
        m.albedo = abi.Vec3.of(albedo)
        m.fuzz, m.refraction_index = float(fuzz), float(refraction_index)
        self.materials.append(m)
        return len(self.materials) - 1

    def add_object(self, kind, material=-1, child=-1, count=0, a=(0, 0, 0), b=(0, 0, 0),
                   c=(0, 0, 0), s=0.0, moving=0, phase=-1):
        o = abi.ObjectDesc()
        o.kind, o.material, o.child, o.count = kind, material, child, count
        o.a, o.b, o.c = abi.Vec3.of(a), abi.Vec3.of(b), abi.Vec3.of(c)
        o.s, o.moving, o.phase = float(s), int(moving), phase
        self.objects.append(o)
        return len(self.objects) - 1

    def add_list(self, child_ids):
        first = len(self.children)
        self.children.extend(child_ids)
        return self.add_object(abi.RT_OBJ_LIST, child=first, count=len(child_ids))

    # ---- ctypes view
    def desc(self):
        T = (abi.TextureDesc * max(1, len(self.textures)))(*self.textures)
        P = (abi.PerlinDesc * max(1, len(self.perlin)))(*self.perlin)
        M = (abi.MaterialDesc * max(1, len(self.materials)))(*self.materials)
        O = (abi.ObjectDesc * max(1, len(self.objects)))(*self.objects)
        K = (C.c_int32 * max(1, len(self.children)))(*self.children)
        self._keep = (T, P, M, O, K)
        d = abi.SceneDesc()
        d.textures, d.n_textures = T, len(self.textures)
        d.perlin, d.n_perlin = P, len(self.perlin)
        d.materials, d.n_materials = M, len(self.materials)
        d.objects, d.n_objects = O, len(self.objects)
        d.children, d.n_children = K, len(self.children)
        d.world, d.lights, d.use_bvh = self.world, self.lights, int(self.use_bvh)
        d.bvh_builder = int(self.bvh_builder)
        d.bvh_arity = int(self.bvh_arity)
        return d

    def camera_desc(self, **overrides):
        cam = dict(self.camera or {})
        cam.update(overrides)
        return camera_desc(cam)


def _perlin_from_json(p):
    d = abi.PerlinDesc()
    rv = p["rand_vec"]
    if len(rv) != 256:
        raise SceneError("perlin.rand_vec needs 256 vectors")
    for k in range(256):
        d.rand_vec[k] = abi.Vec3.of(_v3(rv[k], "perlin.rand_vec"))
    for name in ("perm_x", "perm_y", "perm_z"):
        arr = p[name]
        if len(arr) != 256 or sorted(arr) != list(range(256)):
            raise SceneError("perlin.%s must be a permutation of 0..255" % name)
        getattr(d, name)[:] = [int(x) for x in arr]
    return d


def load_scene(src):
    """Parse a scene (path, JSON text or dict) into a SceneDescription."""
    if isinstance(src, dict):
        doc = copy.deepcopy(src)
    elif isinstance(src, str) and src.lstrip().startswith("{"):
        doc = json.loads(src)
    else:
        with open(src) as f:
            doc = json.load(f)
    S = SceneDescription()
    S.camera = doc.get("camera", {})
    S.use_bvh = 1 if doc.get("use_bvh", False) else 0

    for name, p in (doc.get("perlin") or {}).items():
        S.perlin.append(_perlin_from_json(p))
        S._named_perlin[name] = len(S.perlin) - 1

    tex_specs = doc.get("textures") or {}

    def tex(ref):
        if isinstance(ref, list):  # inline colour
            return S.add_texture(abi.RT_TEX_SOLID, color=_v3(ref, "color"))
        if isinstance(ref, dict):
            return tex_from_spec(ref)
        if ref not in S._named_tex:
            if ref not in tex_specs:
                raise SceneError("unknown texture %r" % ref)
            S._named_tex[ref] = None  # cycle guard
            S._named_tex[ref] = tex_from_spec(tex_specs[ref])
        if S._named_tex[ref] is None:
            raise SceneError("texture cycle at %r" % ref)
        return S._named_tex[ref]

    def tex_from_spec(t):
        ty = t.get("type")
        if ty == "solid":
            return S.add_texture(abi.RT_TEX_SOLID, color=_v3(t["color"], "color"))
        if ty == "checker":
            even, odd = tex(t["even"]), tex(t["odd"])
            return S.add_texture(abi.RT_TEX_CHECKER, scale=float(t["scale"]), even=even, odd=odd)
        if ty == "noise":
            pn = t["perlin"]
            if pn not in S._named_perlin:
                raise SceneError("unknown perlin table %r" % pn)
            return S.add_texture(abi.RT_TEX_NOISE, scale=float(t["scale"]), perlin=S._named_perlin[pn])
        raise SceneError("unknown texture type %r" % ty)

    mat_specs = doc.get("materials") or {}

    def mat(ref):
        if ref is None:
            return -1
        if isinstance(ref, dict):
            return mat_from_spec(ref)
        if ref not in S._named_mat:
            if ref not in mat_specs:
                raise SceneError("unknown material %r" % ref)
            S._named_mat[ref] = mat_from_spec(mat_specs[ref])
        return S._named_mat[ref]

    def tex_or_color(m, color_key):
        if "texture" in m:
            return tex(m["texture"])
        return S.add_texture(abi.RT_TEX_SOLID, color=_v3(m[color_key], color_key))

    def mat_from_spec(m):
        ty = m.get("type")
        if ty == "lambertian":
            return S.add_material(abi.RT_MAT_LAMBERTIAN, texture=tex_or_color(m, "albedo"))
        if ty == "metal":
            return S.add_material(abi.RT_MAT_METAL, albedo=_v3(m["albedo"], "albedo"),
                                  fuzz=float(m.get("fuzz", 0.0)))
        if ty == "dielectric":
            return S.add_material(abi.RT_MAT_DIELECTRIC,
                                  refraction_index=float(m["refraction_index"]))
        if ty == "diffuse_light":
            return S.add_material(abi.RT_MAT_DIFFUSE_LIGHT, texture=tex_or_color(m, "emit"))
        if ty == "isotropic":
            return S.add_material(abi.RT_MAT_ISOTROPIC, texture=tex_or_color(m, "albedo"))
        raise SceneError("unknown material type %r" % ty)

    def obj(o, need_material=True):
        ty = o.get("type")
        mref = o.get("material")
        if ty == "sphere":
            if need_material and mref is None:
                raise SceneError("world sphere without material")
            m = mat(mref)
            if "displacement" in o:  # stored form: Sphere's m_center direction (c1 - c0)
                return S.add_object(abi.RT_OBJ_SPHERE, material=m, a=_v3(o["center"]),
                                    b=_v3(o["displacement"]), s=float(o["radius"]),
                                    moving=abi.RT_STORED_FORM)
            if "center2" in o:
                return S.add_object(abi.RT_OBJ_SPHERE, material=m, a=_v3(o["center"]),
                                    b=_v3(o["center2"]), s=float(o["radius"]), moving=1)
            return S.add_object(abi.RT_OBJ_SPHERE, material=m, a=_v3(o["center"]),
                                s=float(o["radius"]))
        if ty == "quad":
            if need_material and mref is None:
                raise SceneError("world quad without material")
            return S.add_object(abi.RT_OBJ_QUAD, material=mat(mref), a=_v3(o["Q"]),
                                b=_v3(o["u"]), c=_v3(o["v"]))
        if ty == "box":
            if need_material and mref is None:
                raise SceneError("world box without material")
            m = mat(mref)
            ids = [S.add_object(abi.RT_OBJ_QUAD, material=m, a=q, b=u, c=v)
                   for (q, u, v) in make_box_quads(_v3(o["a"]), _v3(o["b"]))]
            return S.add_list(ids)
        if ty == "list":
            ids = [obj(k, need_material) for k in o["objects"]]
            return S.add_list(ids)
        if ty == "rotate_y":
            ch = obj(o["object"], need_material)
            if "sin_cos" in o:  # stored form: RotateY's (sin, cos)
                sc = o["sin_cos"]
                if len(sc) != 2:
                    raise SceneError("rotate_y.sin_cos must be [sin, cos]")
                return S.add_object(abi.RT_OBJ_ROTATE_Y, child=ch,
                                    a=[float(sc[0]), float(sc[1]), 0.0],
                                    moving=abi.RT_STORED_FORM)
            return S.add_object(abi.RT_OBJ_ROTATE_Y, child=ch, s=float(o["angle"]))
        if ty == "translate":
            ch = obj(o["object"], need_material)
            return S.add_object(abi.RT_OBJ_TRANSLATE, child=ch, a=_v3(o["offset"]))
        if ty == "constant_medium":
            ch = obj(o["boundary"], False)
            if "phase" in o:
                ph = mat(o["phase"])
            else:
                ph = S.add_material(abi.RT_MAT_ISOTROPIC, texture=tex_or_color(o, "albedo"))
            dens = float(o["density"])
            if not dens > 0:
                raise SceneError("constant_medium density must be > 0")
            return S.add_object(abi.RT_OBJ_MEDIUM, child=ch, s=dens, phase=ph)
        raise SceneError("unknown object type %r" % ty)

    world_ids = [obj(o) for o in doc.get("world", [])]
    S.world = S.add_list(world_ids)
    if "lights" in doc and doc["lights"] is not None:
        light_ids = [obj(o, need_material=False) for o in doc["lights"]]
        S.lights = S.add_list(light_ids)
    return S


def dump_scene(S):
    """SceneDescription -> JSON document (dict) that load_scene reads back into
    the same tables: every texture/material/Perlin table is named by its index
    and referenced by name, objects keep their nesting (so the lazy loader
    re-creates every table entry and object in the same order), boxes come back
    as their 6-quad lists, and the stored forms (sphere displacement, rotate_y
    sin/cos) are written as such, so no double changes."""
    v = lambda x: [x.x, x.y, x.z]  # noqa: E731
    doc = {}
    if S.camera:
        doc["camera"] = copy.deepcopy(S.camera)
    doc["use_bvh"] = bool(S.use_bvh)
    if S.perlin:
        doc["perlin"] = {"p%d" % i: {"rand_vec": [v(p.rand_vec[k]) for k in range(256)],
                                     "perm_x": list(p.perm_x), "perm_y": list(p.perm_y),
                                     "perm_z": list(p.perm_z)}
                         for i, p in enumerate(S.perlin)}
    tex = {}
    for i, t in enumerate(S.textures):
        if t.kind == abi.RT_TEX_SOLID:
            tex["t%d" % i] = {"type": "solid", "color": v(t.color)}
        elif t.kind == abi.RT_TEX_CHECKER:
            tex["t%d" % i] = {"type": "checker", "scale": t.scale,
                              "even": "t%d" % t.even, "odd": "t%d" % t.odd}
        else:
            tex["t%d" % i] = {"type": "noise", "scale": t.scale, "perlin": "p%d" % t.perlin}
    if tex:
        doc["textures"] = tex
    mats = {}
    for i, m in enumerate(S.materials):
        if m.kind == abi.RT_MAT_LAMBERTIAN:
            mats["m%d" % i] = {"type": "lambertian", "texture": "t%d" % m.texture}
        elif m.kind == abi.RT_MAT_METAL:
            mats["m%d" % i] = {"type": "metal", "albedo": v(m.albedo), "fuzz": m.fuzz}
        elif m.kind == abi.RT_MAT_DIELECTRIC:
            mats["m%d" % i] = {"type": "dielectric", "refraction_index": m.refraction_index}
        elif m.kind == abi.RT_MAT_DIFFUSE_LIGHT:
            mats["m%d" % i] = {"type": "diffuse_light", "texture": "t%d" % m.texture}
        else:
            mats["m%d" % i] = {"type": "isotropic", "texture": "t%d" % m.texture}
    if mats:
        doc["materials"] = mats

    def obj(i):
        o = S.objects[i]
        mref = ("m%d" % o.material) if o.material >= 0 else None
        if o.kind == abi.RT_OBJ_SPHERE:
            d = {"type": "sphere", "center": v(o.a), "radius": o.s}
            if o.moving == abi.RT_STORED_FORM:
                d["displacement"] = v(o.b)
            elif o.moving:
                d["center2"] = v(o.b)
        elif o.kind == abi.RT_OBJ_QUAD:
            d = {"type": "quad", "Q": v(o.a), "u": v(o.b), "v": v(o.c)}
        elif o.kind == abi.RT_OBJ_LIST:
            return {"type": "list",
                    "objects": [obj(S.children[o.child + k]) for k in range(o.count)]}
        elif o.kind == abi.RT_OBJ_ROTATE_Y:
            d = {"type": "rotate_y", "object": obj(o.child)}
            if o.moving == abi.RT_STORED_FORM:
                d["sin_cos"] = [o.a.x, o.a.y]
            else:
                d["angle"] = o.s
            return d
        elif o.kind == abi.RT_OBJ_TRANSLATE:
            return {"type": "translate", "offset": v(o.a), "object": obj(o.child)}
        else:
            return {"type": "constant_medium", "boundary": obj(o.child), "density": o.s,
                    "phase": "m%d" % o.phase}
        if mref is not None:
            d["material"] = mref
        return d

    w = S.objects[S.world]
    doc["world"] = [obj(S.children[w.child + k]) for k in range(w.count)]
    if S.lights >= 0:
        li = S.objects[S.lights]
        doc["lights"] = [obj(S.children[li.child + k]) for k in range(li.count)]
    return doc


def dump_float(x):
    """%.17g round-trip float formatting for scene files."""
    return float(repr(float(x)))


def frame_height(width, aspect):
    """Camera::initialize image height rule (Camera.cpp:32-33)."""
    h = int(width / aspect)
    return max(1, h)


def perlin_reference_tables(rng_draw_double, rng_draw_int):
    """Build Perlin tables the way PerlinNoise() does (PerlinNoise.hpp:19-26,
    150-170) from caller-supplied draw functions (unused by the runtime; kept
    for scene tooling)."""
    rv = []
    for _ in range(256):
        z = rng_draw_double(-1, 1)
        y = rng_draw_double(-1, 1)
        x = rng_draw_double(-1, 1)
        l = math.sqrt(x * x + y * y + z * z)
        rv.append([x / l, y / l, z / l] if l > 1e-8 else [1.0, 0.0, 0.0])
    perms = []
    for _ in range(3):
        p = list(range(256))
        for i in range(255, 0, -1):
            t = rng_draw_int(0, i)
            p[i], p[t] = p[t], p[i]
        perms.append(p)
    return {"rand_vec": rv, "perm_x": perms[0], "perm_y": perms[1], "perm_z": perms[2]}
