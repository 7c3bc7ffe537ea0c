#!/usr/bin/env python3
"""Build-owned render-mesh compiler: reference MJCF/STL (read as DATA) -> gym_so100/assets/so100_render.npz.

The reference's default observation (``obs_type="so100_pixels_agent_pos"``, gym_so100/__init__.py:4-32)
renders the ``top`` camera (gym_so100/env.py:84-94, scene_so100.xml:30).  The batched rasteriser
(csrc/so100_render.hip) draws the geoms MuJoCo shows by default -- geom groups 0-2: the class="visual"
meshes of the arm (so_arm100.xml:52-56,69-70,77-78,85-86,93-94,101-102,109-110,135), the table
(scene_so100.xml:20, group 1), the bin boxes and the cube (so100_transfer_cube.xml:10,18-22) -- and not
the collision geoms (group 3: the hulls and the finger pads).  This script writes their triangles in
their body frames with the geom colours (material / rgba; MuJoCo's default geom rgba 0.5 0.5 0.5 1):

* arm meshes: the STL decimated by vertex clustering on a grid (cell chosen per mesh so that at most
  MAX_TRIS triangles survive) -- at the top camera's 64x48 a pixel is ~2.7 cm on the table, the meshes
  lose nothing visible at that size; larger renders show facets;
* boxes (table, bin walls/floor, cube): their 12 triangles.

Bodies: 0 world (table, bin), 1 Base (static, its own frame), 2..7 arm links, 8 the cube -- the numbering
of include/so100_model.h.  Runs in the build container only; the .npz is committed.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import compile_model as cm  # noqa: E402

OUT = os.path.join(os.path.dirname(__file__), "..", "gym_so100", "assets", "so100_render.npz")
MAX_TRIS = 320
DEFAULT_RGBA = (0.5, 0.5, 0.5)


def cluster(v, f, cell):
    """Vertex clustering: snap vertices to grid cells (representative = cell mean), drop collapsed and
    duplicate triangles."""
    key = np.floor(v / cell).astype(np.int64)
    _, inv = np.unique(key, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    rep = np.zeros((inv.max() + 1, 3))
    np.add.at(rep, inv, v)
    rep /= np.bincount(inv)[:, None]
    g = inv[f]
    ok = (g[:, 0] != g[:, 1]) & (g[:, 1] != g[:, 2]) & (g[:, 0] != g[:, 2])
    g = g[ok]
    _, uniq = np.unique(np.sort(g, axis=1), axis=0, return_index=True)
    g = g[np.sort(uniq)]
    return rep[g]


def decimate(tri):
    v = tri.reshape(-1, 3)
    vu, inv = np.unique(v, axis=0, return_inverse=True)
    f = inv.reshape(-1, 3)
    if len(f) <= MAX_TRIS:
        return tri
    lo, hi = 1e-4, float(np.ptp(vu, axis=0).max())
    for _ in range(40):
        mid = np.sqrt(lo * hi)
        if len(cluster(vu, f, mid)) > MAX_TRIS:
            lo = mid
        else:
            hi = mid
    return cluster(vu, f, hi)


def box_tris(center, half):
    c, h = np.asarray(center, float), np.asarray(half, float)
    corners = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]) * h + c
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    out = []
    for a, b, cc, d in quads:
        out += [corners[[a, b, cc]], corners[[a, cc, d]]]
    return np.array(out)


# scene_so100.xml:7-30: headlight, the three directional lights and the cameras (mode="targetbody" on the
# static table body at (0, .6, 0); front_close tracks vx300s_left/camera_focus, the ee_site body, so its
# frame is computed per env in the kernel)
HEADLIGHT = dict(ambient=0.4, diffuse=0.4)            # ambient from :9; diffuse MuJoCo's default 0.4
LIGHTS = [((1, 1, -1), 0.3), ((-1, 1, -1), 0.3), ((0, -1, -1), 0.3)]
CAMERAS = {"top": (0, 0.6, 0.8), "angle": (0, 0, 0.6), "left_pillar": (-0.5, 0.2, 0.6),
           "right_pillar": (0.5, 0.2, 0.6)}
CAMERA_TARGET = (0.0, 0.6, 0.0)
FRONT_CLOSE = (0.0, 0.2, 0.4)
FOVY = 78.0


def normalize(v):
    n = np.linalg.norm(v)
    return v / n if n > 1e-15 else np.array([1.0, 0.0, 0.0])   # mju_normalize3's fallback


def targetbody_frame(pos, target):
    """MuJoCo's mjCAMLIGHT_TARGETBODY camera frame (engine_core_smooth.c mj_camlight): z = pos - target,
    x = up(0,0,1) x z, y = z x x; rows of the returned matrix are world coordinates, columns camera axes."""
    z = normalize(np.asarray(pos, float) - np.asarray(target, float))
    x = normalize(np.cross([0.0, 0.0, 1.0], z))
    y = np.cross(z, x)
    return np.stack([x, y, z], axis=1)


def main():
    opt, bodies, actuators, excludes = cm.parse()
    names = ["world"] + cm.ARM_BODIES + ["box"]
    bid = {n: i for i, n in enumerate(names)}
    arm = os.path.join(cm.ASSETS, "trs_so_arm100")
    mats = {"white": (1.0, 1.0, 1.0), "black": (0.1, 0.1, 0.1)}
    tris, body, rgb = [], [], []
    for bname in cm.ARM_BODIES:
        for g in bodies[bname]["geoms"]:
            if g.get("type") != "mesh" or g.get("group", "0") not in ("0", "1", "2"):
                continue
            assert not g.get("pos") and not g.get("quat") and not g.get("euler"), "visual mesh with an offset"
            t = decimate(cm.load_stl(os.path.join(arm, g["mesh"] + ".stl")).reshape(-1, 3, 3))
            tris.append(t)
            body += [bid[bname]] * len(t)
            rgb += [mats[g.get("material", "white")]] * len(t)
    # table (mesh tabletop.stl, an exact box: compile_model), bin boxes, cube
    m = cm.compile_model()
    for g in m["geoms"]:
        if "pad" in g["name"]:
            continue                                   # finger pads: class "collision", group 3 (hidden)
        if g["name"] == "table":
            col = (0.2, 0.2, 0.2)                      # scene_so100.xml:20 rgba
        elif g["name"] == "red_box":
            col = (1.0, 0.0, 0.0)                      # so100_transfer_cube.xml:10-11 rgba
        else:
            col = DEFAULT_RGBA
        t = box_tris(g["pos"], g["size"])
        tris.append(t)
        body += [g["body"]] * len(t)
        rgb += [col] * len(t)
    tris = np.concatenate(tris).astype(np.float32)
    cams = {}
    for name, pos in CAMERAS.items():
        cams["cam_" + name + "_pos"] = np.asarray(pos, np.float32)
        cams["cam_" + name + "_mat"] = targetbody_frame(pos, CAMERA_TARGET).astype(np.float32)
    cams["cam_front_close_pos"] = np.asarray(FRONT_CLOSE, np.float32)
    cams["cam_front_close_mat"] = np.eye(3, dtype=np.float32)          # unused: tracked per env
    np.savez_compressed(OUT, tri=tris, body=np.array(body, np.int32), rgb=np.array(rgb, np.float32),
                        fovy=np.float32(FOVY), head=np.array([HEADLIGHT["ambient"], HEADLIGHT["diffuse"]], np.float32),
                        light_dir=np.array([normalize(np.asarray(d, float)) for d, _ in LIGHTS], np.float32),
                        light_diffuse=np.array([c for _, c in LIGHTS], np.float32), **cams)
    print("wrote", os.path.abspath(OUT), "triangles", len(tris), "per body", np.bincount(body))


if __name__ == "__main__":
    main()
