"""numpy restatement of csrc/so100_render.hip's rasterisation rules (TEST INFRASTRUCTURE ONLY).

Checks the HIP rasteriser against the same rules evaluated in float64 on the oracle's body frames:
pixel centres (x + 0.5, y + 0.5) inside a triangle by its three edge functions (edges included),
perspective-correct depth, nearest depth wins and equal depths take the smaller packed RGB, flat
two-sided Lambert shading from the headlight and the directional lights, black background.

This pins the kernel to its own specification; it is not MuJoCo's renderer (parity with MuJoCo's
OpenGL images is unpinned).
"""
import numpy as np


def pack_rgb(rgb):
    c = np.clip(np.asarray(rgb, np.float64), 0.0, 1.0)
    q = np.floor(c * 255.0 + 0.5).astype(np.uint32)
    return q[..., 0] | (q[..., 1] << 8) | (q[..., 2] << 16)


def shade(cam, p, rgb8):
    """Shaded RGB8 of triangles p [T,3,3] (world) with base colours rgb8 [T] (uint32 packed)."""
    n = np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0])
    ln = np.linalg.norm(n, axis=1, keepdims=True)
    n = np.where(ln > 0, n / np.where(ln > 0, ln, 1.0), 0.0)
    v = cam["pos"][None, :] - p[:, 0]
    n = np.where((np.sum(n * v, axis=1) < 0)[:, None], -n, n)
    zc = cam["mat"][:, 2]
    lum = cam["head_ambient"] + cam["head_diffuse"] * np.maximum(0.0, n @ zc)
    for d, c in zip(cam["light_dir"], cam["light_diffuse"]):
        lum = lum + c * np.maximum(0.0, -(n @ d))
    base = np.stack([(rgb8 >> (8 * k)) & 0xFF for k in range(3)], axis=1).astype(np.float64) / 255.0
    val = np.clip(base * lum[:, None], 0.0, 1.0)
    q = np.floor(val * 255.0 + 0.5).astype(np.uint32)
    return q[:, 0] | (q[:, 1] << 8) | (q[:, 2] << 16)


def tracking_frame(pos, target):
    """MuJoCo's targetbody camera frame (mj_camlight): z = pos - target, x = (0,0,1) x z, y = z x x."""
    z = np.asarray(pos, float) - np.asarray(target, float)
    n = np.linalg.norm(z)
    z = z / n if n > 1e-15 else np.array([1.0, 0, 0])
    x = np.cross([0.0, 0.0, 1.0], z)
    n = np.linalg.norm(x)
    x = x / n if n > 1e-15 else np.array([1.0, 0, 0])
    return np.stack([x, np.cross(z, x), z], axis=1)


def render(scene_tri, scene_body, scene_rgb, frames, cam, width, height, target=None):
    """frames: [NBODY] of (R [3,3], p [3]) world frames; target: the tracked point (ee_site) of a
    tracking camera; returns uint8 [H, W, 3]."""
    if cam.get("track"):
        cam = dict(cam, mat=tracking_frame(cam["pos"], target))
    R = np.stack([f[0] for f in frames])[scene_body]                   # [T,3,3]
    P = np.stack([f[1] for f in frames])[scene_body]                   # [T,3]
    w = np.einsum("tij,tvj->tvi", R, scene_tri.astype(np.float64)) + P[:, None, :]
    d = w - cam["pos"]
    c = d @ cam["mat"]                                                  # camera coordinates
    depth = -c[..., 2]
    th = np.tan(0.5 * np.radians(cam["fovy"]))
    aspect = width / height
    ok = np.all(depth > cam["znear"], axis=1)
    iz = 1.0 / np.where(depth > 0, depth, 1.0)
    sx = (c[..., 0] * iz / (th * aspect) * 0.5 + 0.5) * width
    sy = (0.5 - c[..., 1] * iz / th * 0.5) * height
    col = shade(cam, w, pack_rgb(scene_rgb))
    key = np.full((height, width), np.iinfo(np.uint64).max, np.uint64)
    for t in np.nonzero(ok)[0]:
        x, y, z = sx[t], sy[t], iz[t]
        area = (x[1] - x[0]) * (y[2] - y[0]) - (x[2] - x[0]) * (y[1] - y[0])
        if not abs(area) > 1e-12:
            continue
        bx0, bx1 = max(0, int(np.floor(x.min() - 0.5))), min(width - 1, int(np.ceil(x.max() - 0.5)))
        by0, by1 = max(0, int(np.floor(y.min() - 0.5))), min(height - 1, int(np.ceil(y.max() - 0.5)))
        if bx0 > bx1 or by0 > by1:
            continue
        px, py = np.meshgrid(np.arange(bx0, bx1 + 1) + 0.5, np.arange(by0, by1 + 1) + 0.5)
        w0 = (x[2] - x[1]) * (py - y[1]) - (y[2] - y[1]) * (px - x[1])
        w1 = (x[0] - x[2]) * (py - y[2]) - (y[0] - y[2]) * (px - x[2])
        w2 = (x[1] - x[0]) * (py - y[0]) - (y[1] - y[0]) * (px - x[0])
        sg = 1.0 if area > 0 else -1.0
        inside = (w0 * sg >= 0) & (w1 * sg >= 0) & (w2 * sg >= 0)
        izp = (w0 * z[0] + w1 * z[1] + w2 * z[2]) / area
        inside &= izp > 0
        dep = (1.0 / np.where(inside, izp, 1.0)).astype(np.float32)
        k = (dep.view(np.uint32).astype(np.uint64) << np.uint64(32)) | np.uint64(col[t])
        sub = key[by0:by1 + 1, bx0:bx1 + 1]
        np.copyto(sub, np.minimum(sub, k), where=inside)
    rgb = np.where(key == np.iinfo(np.uint64).max, np.uint64(0), key & np.uint64(0xFFFFFF)).astype(np.uint32)
    return np.stack([(rgb >> (8 * k)) & 0xFF for k in range(3)], axis=-1).astype(np.uint8)


def camera_dict(cam_struct):
    """so100_camera ctypes struct -> numpy dict for render()."""
    return {"pos": np.array(cam_struct.pos[:], np.float64),
            "mat": np.array(cam_struct.mat[:], np.float64).reshape(3, 3), "track": int(cam_struct.track),
            "fovy": float(cam_struct.fovy), "znear": float(cam_struct.znear),
            "head_ambient": float(cam_struct.head_ambient), "head_diffuse": float(cam_struct.head_diffuse),
            "light_dir": [np.array(cam_struct.light_dir[i][:], np.float64) for i in range(cam_struct.nlight)],
            "light_diffuse": [float(cam_struct.light_diffuse[i]) for i in range(cam_struct.nlight)]}
