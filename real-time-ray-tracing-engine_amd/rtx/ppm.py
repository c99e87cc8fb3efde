"""PPM "P3" output with the reference's quantisation (utils/ColorUtility.hpp:11-36).

byte = (unsigned char)(256 * clamp(x > 0 ? sqrt(x) : 0, 0.000, 0.999)), so NaN
maps to 0; the file is "P3\\nW H\\n255\\n" then "r g b\\n" per pixel, rows top to
bottom (StaticCamera.cpp:57, 93-99).
"""
import numpy as np


def to_bytes(rgb):
    x = np.asarray(rgb, dtype=np.float64)
    with np.errstate(invalid="ignore"):
        g = np.where(x > 0, np.sqrt(np.where(x > 0, x, 0.0)), 0.0)
        g = np.where(g < 0.0, 0.0, g)
        g = np.where(g > 0.999, 0.999, g)
    return (256.0 * g).astype(np.uint8)


def ppm_bytes(rgb):
    """rgb: float array [H, W, 3] of scaled radiance -> the P3 file contents."""
    b = to_bytes(rgb)
    h, w = b.shape[0], b.shape[1]
    flat = b.reshape(-1, 3)
    lines = ["%d %d %d\n" % (int(r), int(g), int(bb)) for r, g, bb in flat]
    return ("P3\n%d %d\n255\n" % (w, h) + "".join(lines)).encode()


def write_ppm(path, rgb):
    data = ppm_bytes(rgb)
    with open(path, "wb") as f:
        f.write(data)
    return len(data)
