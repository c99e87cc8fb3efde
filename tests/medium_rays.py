"""Deterministic test rays for the box-boundary medium queries (rt_path.h
box_span vs boundary_span vs the reference's ConstantMedium boundary queries).

The rays come from a splitmix64 counter stream computed here with numpy
integer arithmetic, so the same rays are regenerated on any machine and numpy
version: the golden file (tests/golden/ref_medium_box.npz, made by
tests/golden/make_medium_kats.py from oracle/_ref) stores only the
reference's outputs.

The boundary is cornell_fog's medium: make_box((0,0,0), (165,330,165)) under
RotateY(15) and Translate(265, 0, 295) (scenes/cornell_fog.json; the
reference's main.cpp builds the same).  Eight families of rays, k mod 8:
  0 random origins towards the box's world bounds
  1 towards points on the 12 box edges, perturbed by 10^-14 .. 1
  2 towards the 8 corners, perturbed likewise
  3 world directions with d_y = 0, +-1e-8, +-5e-9, +-2e-8 (parallel or
    nearly parallel to the top / bottom faces; Plane::hit's 1e-8 test)
  4 origins inside the box
  5 origins on a face plane (up to the rounding of the transform)
  6 tiny / huge direction scales and far origins
  7 grazing rays nearly inside a face plane
"""
import numpy as np

BOX_LO = np.array([0.0, 0.0, 0.0])
BOX_HI = np.array([165.0, 330.0, 165.0])
OFFSET = np.array([265.0, 0.0, 295.0])
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix(idx):
    z = (idx.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniforms(seed, n, m):
    """n x m uniforms in [0, 1), 53-bit, from stream `seed`."""
    idx = (np.arange(n * m, dtype=np.uint64) + np.uint64(seed) * np.uint64(1 << 40))
    with np.errstate(over="ignore"):
        z = _splitmix(idx)
    return ((z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53).reshape(n, m)


def _rot(deg):
    # RotateY (RotateY.cpp:7-9): sin, cos of the angle in radians
    r = np.deg2rad(deg)
    return np.sin(r), np.cos(r)


def to_world(p):
    """Local box-frame points -> world (RotateY(15) then Translate)."""
    s, c = _rot(15.0)
    x = c * p[..., 0] + s * p[..., 2]
    z = -s * p[..., 0] + c * p[..., 2]
    return np.stack([x, p[..., 1], z], -1) + OFFSET


def dir_to_world(d):
    s, c = _rot(15.0)
    return np.stack([c * d[..., 0] + s * d[..., 2], d[..., 1], -s * d[..., 0] + c * d[..., 2]], -1)


def make_rays(n, seed=5):
    U = uniforms(seed, n, 16)
    fam = np.arange(n) % 8
    org = -100.0 + 750.0 * U[:, 0:3]
    tgt = np.empty((n, 3))
    ext = BOX_HI - BOX_LO
    wlo = to_world(np.array([[0, 0, 0], [165, 0, 165], [0, 0, 165], [165, 0, 0]], float)).min(0)
    whi = to_world(np.array([[0, 330, 0], [165, 330, 165], [0, 330, 165], [165, 330, 0]], float)).max(0)
    tgt[:] = wlo + (whi - wlo) * U[:, 3:6]
    eps = 10.0 ** (-14.0 * U[:, 6]) * np.where(U[:, 7] < 0.5, -1.0, 1.0)
    # 1: edges -- two coordinates at a box bound, the third along the edge
    local = BOX_LO + ext * U[:, 8:11]
    axis = (U[:, 11] * 3).astype(int)
    b1 = U[:, 12] < 0.5
    b2 = U[:, 13] < 0.5
    edge = local.copy()
    for a in range(3):
        m = axis == a
        o1, o2 = (a + 1) % 3, (a + 2) % 3
        edge[m, o1] = np.where(b1[m], BOX_HI[o1], BOX_LO[o1]) + eps[m]
        edge[m, o2] = np.where(b2[m], BOX_HI[o2], BOX_LO[o2]) - eps[m]
    sel = fam == 1
    tgt[sel] = to_world(edge[sel])
    # 2: corners
    corner = np.where(U[:, 8:11] < 0.5, BOX_LO, BOX_HI) + eps[:, None] * np.sign(U[:, 11:14] - 0.5)
    sel = fam == 2
    tgt[sel] = to_world(corner[sel])
    d = tgt - org
    # 3: world d_y exactly 0 or near Plane::hit's 1e-8 threshold
    sel = fam == 3
    dy = np.array([0.0, 1e-8, -1e-8, 5e-9, -5e-9, 2e-8, -2e-8, 0.0])[(U[:, 14] * 8).astype(int)]
    d[sel, 1] = dy[sel]
    org[sel, 1] = 330.0 * U[sel, 15]
    # 4: origins inside the box, random directions
    sel = fam == 4
    org[sel] = to_world(BOX_LO + ext * U[sel, 8:11])
    d[sel] = U[sel, 3:6] - 0.5
    # 5: origins on a face plane (local), random directions
    sel = fam == 5
    p = BOX_LO + ext * U[:, 8:11]
    for a in range(3):
        m = sel & (axis == a)
        p[m, a] = np.where(b1[m], BOX_HI[a], BOX_LO[a])
    org[sel] = to_world(p[sel])
    d[sel] = U[sel, 3:6] - 0.5
    # 6: direction scales 1e-4 .. 1e4, some origins 1e5 away
    sel = fam == 6
    d[sel] *= (10.0 ** (8.0 * U[sel, 14] - 4.0))[:, None]
    far = sel & (U[:, 15] < 0.3)
    org[far] = tgt[far] - 1e5 * (d[far] / np.linalg.norm(d[far], axis=1)[:, None])
    # 7: grazing -- origin within eps of a face plane, direction nearly inside it
    sel = fam == 7
    p = BOX_LO - 0.5 * ext + 2.0 * ext * U[:, 8:11]
    dl = U[:, 3:6] - 0.5
    for a in range(3):
        m = sel & (axis == a)
        p[m, a] = np.where(b1[m], BOX_HI[a], BOX_LO[a]) + eps[m]
        dl[m, a] = eps[m] * (U[m, 15] - 0.5)
    org[sel] = to_world(p[sel])
    d[sel] = dir_to_world(dl[sel])
    tm = U[:, 15]
    return np.ascontiguousarray(np.concatenate([org, d, tm[:, None]], 1), dtype=np.float64)
