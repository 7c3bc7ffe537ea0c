#!/usr/bin/env python3
"""Build-owned model compiler: reference MJCF/STL (read as DATA) -> derived so100 model table.

This runs only in the build container (where /root/reference exists) and writes
``gym_so100/assets/so100_model.json``, which is committed; the GPU box never reads the
reference.  It restates what MuJoCo's compiler does for the parts of
``gym_so100/assets/so100_transfer_cube.xml`` that the hot path needs
(reference: gym_so100/env.py:111-112 loads that file):

* body tree + frames      (trs_so_arm100/so_arm100.xml:67-153, so100_transfer_cube.xml:7-24)
* explicit inertials      (so_arm100.xml:73-75,81-83,89-91,97-99,105-107,130-132; cube :9)
* hinge axes/ranges, frictionloss/armature classes (so_arm100.xml:30-51)
* position actuators kp=50, dampratio=1 -> kv, forcerange, inheritrange (so_arm100.xml:33,156-163)
* collision boxes: finger pads (so_arm100.xml:60-62,113-120,139-146), cube (transfer_cube.xml:10-11),
  bin walls/floor (transfer_cube.xml:18-22), table = 8-vertex box hull of tabletop.stl
  (scene_so100.xml:3,20) emitted as an exact box
* arm/jaw collision hulls: qhull convex hulls (scipy) of the class="collision" meshes on the moving arm
  bodies; hull-hull self-collision pairs of non-adjacent links (MuJoCo's parent-child filter);
  bodies (so_arm100.xml:79,87,95,103,111-112,136-138), vertices in the body frame, mesh volume
  centroid (the mesh geom's frame origin), for the hull-vs-table contacts and the box-vs-hull pairs of
  the convex collider (cube and bin boxes vs every hull); pair parameters mixed like
  the box pairs
* contact-pair parameter mixing (MuJoCo mj_contactParam semantics, restated): condim=max,
  friction=elementwise max, solref/solimp = solmix-weighted mean (solmix defaults 1 -> mean)
* setConst quantities at qpos0 (MuJoCo mj_setConst, restated): dof_M0 (diag of M incl. armature),
  dof_invweight0, body_invweight0 (mean diagonal of J M^-1 J^T at the body COM), meaninertia,
  actuator kv = dampratio * 2 * sqrt(kp * dof_M0).

MuJoCo itself is not available here; these restatements are [3P-unverified] against MuJoCo 3.3.3
(parity unpinned) and are pinned by the analytic tests in tests/test_oracle_physics.py.
"""
import json
import math
import os
import struct
import sys
import xml.etree.ElementTree as ET

import numpy as np

REF = os.environ.get("SO100_REFERENCE", "/root/reference")
ASSETS = os.path.join(REF, "gym_so100", "assets")
OUT = os.path.join(os.path.dirname(__file__), "..", "gym_so100", "assets", "so100_model.json")


# ----------------------------------------------------------------------------- math helpers
def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                     w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def quat_normalize(q):
    q = np.asarray(q, dtype=np.float64)
    return q / np.linalg.norm(q)


def quat2mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def axis_angle_quat(axis, ang):
    axis = np.asarray(axis, dtype=np.float64)
    s = math.sin(ang / 2)
    return np.array([math.cos(ang / 2), axis[0] * s, axis[1] * s, axis[2] * s])


def euler_xyz_intrinsic(e):
    # MuJoCo compiler default eulerseq="xyz" (lower case = rotating axes)
    q = np.array([1.0, 0, 0, 0])
    for ax, ang in zip(np.eye(3), e):
        q = quat_mul(q, axis_angle_quat(ax, ang))
    return q


def vec(s, n=None):
    v = [float(x) for x in s.split()]
    if n is not None:
        assert len(v) == n, (s, n)
    return np.array(v)


# ----------------------------------------------------------------------------- MJCF walker
class Defaults:
    """MuJoCo default-class tree (restated: nested <default class=...> inherit from parents)."""

    def __init__(self):
        self.classes = {"main": {}}
        self.parent = {"main": None}

    def load(self, elem, parent="main"):
        for d in elem.findall("default"):
            name = d.get("class", "main")
            self.parent[name] = None if name == "main" else parent
            attrs = {}
            for child in d:
                if child.tag != "default":
                    attrs[child.tag] = dict(child.attrib)
            self.classes[name] = attrs
            self.load(d, name)

    def resolve(self, cls, tag):
        chain = []
        c = cls
        while c is not None:
            chain.append(c)
            c = self.parent.get(c)
        out = {}
        for c in reversed(chain):
            out.update(self.classes.get(c, {}).get(tag, {}))
        return out


def load_stl(path):
    b = open(path, "rb").read()
    if b[:5] == b"solid" and b"facet" in b[:300]:
        v = []
        for line in b.decode().splitlines():
            line = line.strip()
            if line.startswith("vertex"):
                v.append([float(x) for x in line.split()[1:]])
        return np.array(v)
    n = struct.unpack("<I", b[80:84])[0]
    a = np.frombuffer(b[84:84 + 50 * n], dtype=np.dtype([("n", "<3f4"), ("v", "<9f4"), ("a", "<u2")]))
    return a["v"].reshape(-1, 3).astype(np.float64)


def parse():
    main = ET.parse(os.path.join(ASSETS, "so100_transfer_cube.xml")).getroot()
    scene = ET.parse(os.path.join(ASSETS, "scene_so100.xml")).getroot()
    arm = ET.parse(os.path.join(ASSETS, "trs_so_arm100", "so_arm100.xml")).getroot()
    opt = arm.find("option").attrib
    defaults = Defaults()
    defaults.load(arm)

    bodies = {}   # name -> dict(parent, pos, quat, inertial, joints, geoms, sites)

    def frame(e):
        pos = vec(e.get("pos", "0 0 0"), 3)
        if e.get("quat"):
            q = quat_normalize(vec(e.get("quat"), 4))
        elif e.get("euler"):
            q = euler_xyz_intrinsic(vec(e.get("euler"), 3))
        else:
            q = np.array([1.0, 0, 0, 0])
        return pos, q

    def walk(elem, parent, childclass):
        for b in elem.findall("body"):
            name = b.get("name")
            cc = b.get("childclass", childclass)
            pos, q = frame(b)
            rec = dict(parent=parent, pos=pos, quat=q, inertial=None, joints=[], geoms=[], sites=[])
            inert = b.find("inertial")
            if inert is not None:
                ipos, iq = frame(inert)
                rec["inertial"] = dict(pos=ipos, quat=iq, mass=float(inert.get("mass")),
                                       diag=vec(inert.get("diaginertia"), 3))
            for j in b.findall("joint"):
                cls = j.get("class", cc)
                attrs = defaults.resolve(cls, "joint") if cls else {}
                attrs.update(j.attrib)
                rec["joints"].append(attrs)
            for g in b.findall("geom"):
                cls = g.get("class", cc)
                attrs = defaults.resolve(cls, "geom") if cls else {}
                attrs.update(g.attrib)
                rec["geoms"].append(attrs)
            for s in b.findall("site"):
                rec["sites"].append(dict(s.attrib))
            bodies[name] = rec
            walk(b, name, cc)

    walk(scene.find("worldbody"), "world", None)
    walk(arm.find("worldbody"), "world", None)
    walk(main.find("worldbody"), "world", None)

    actuators = []
    for a in arm.find("actuator").findall("position"):
        attrs = defaults.resolve(a.get("class"), "position")
        attrs.update(a.attrib)
        actuators.append(attrs)
    excludes = [(e.get("body1"), e.get("body2")) for e in arm.find("contact").findall("exclude")]
    return opt, bodies, actuators, excludes


# ----------------------------------------------------------------------------- compile
ARM_BODIES = ["Base", "Rotation_Pitch", "Upper_Arm", "Lower_Arm", "Wrist_Pitch_Roll", "Fixed_Jaw",
              "Moving_Jaw"]
# MuJoCo defaults (mjModel option / geom / joint defaults) [3P-unverified restatement]
MJ_TIMESTEP = 0.002
MJ_GRAVITY = [0.0, 0.0, -9.81]
MJ_ITERATIONS = 100
MJ_TOLERANCE = 1e-8
MJ_SOLREF = [0.02, 1.0]
MJ_SOLIMP = [0.9, 0.95, 0.001, 0.5, 2.0]
MJ_FRICTION = [1.0, 0.005, 0.0001]
MJ_CONDIM = 3
MOCAP_BODY = 9          # the EE variant's mocap body (include/so100_model.h SO100_MOCAP_BODY): no dofs, not in the body arrays


def compile_model():
    opt, bodies, actuators, excludes = parse()

    # ---- kinematic bodies (compact numbering) ----
    names = ["world"] + ARM_BODIES + ["box"]
    bid = {n: i for i, n in enumerate(names)}
    nbody = len(names)
    body_parent = [-1] + [bid[bodies[n]["parent"]] for n in names[1:]]
    body_pos = [[0, 0, 0]] + [bodies[n]["pos"].tolist() for n in names[1:]]
    body_quat = [[1, 0, 0, 0]] + [bodies[n]["quat"].tolist() for n in names[1:]]
    body_ipos, body_iquat, body_mass, body_inertia = [[0, 0, 0]], [[1, 0, 0, 0]], [0.0], [[0, 0, 0]]
    for n in names[1:]:
        ine = bodies[n]["inertial"]
        if ine is None:    # Base: static body; its inertia never enters the dynamics
            body_ipos.append([0, 0, 0]); body_iquat.append([1, 0, 0, 0])
            body_mass.append(0.0); body_inertia.append([0, 0, 0])
        else:
            body_ipos.append(ine["pos"].tolist()); body_iquat.append(ine["quat"].tolist())
            body_mass.append(ine["mass"]); body_inertia.append(ine["diag"].tolist())

    # ---- joints: 6 hinges (arm) + 1 free (cube) ----
    hinge_names, jnt_body, jnt_axis, jnt_range = [], [], [], []
    dof_armature, dof_frictionloss = [], []
    for n in ARM_BODIES:
        for j in bodies[n]["joints"]:
            hinge_names.append(j["name"])
            jnt_body.append(bid[n])
            ax = vec(j["axis"], 3)
            jnt_axis.append((ax / np.linalg.norm(ax)).tolist())
            jnt_range.append(vec(j["range"], 2).tolist())
            dof_armature.append(float(j.get("armature", 0)))
            dof_frictionloss.append(float(j.get("frictionloss", 0)))
    assert len(hinge_names) == 6, hinge_names
    free = bodies["box"]["joints"][0]
    assert free["type"] == "free"
    dof_armature += [0.0] * 6
    dof_frictionloss += [float(free.get("frictionloss", 0))] * 6

    # ---- forward kinematics at qpos0 (numpy restatement of mj_kinematics) ----
    def fk(qarm, box_pos, box_quat):
        xpos = [np.zeros(3)] * nbody
        xquat = [np.array([1.0, 0, 0, 0])] * nbody
        xanchor, xaxis = [None] * 6, [None] * 6
        for b in range(1, nbody):
            p = body_parent[b]
            if names[b] == "box":
                xpos[b] = np.array(box_pos, dtype=float); xquat[b] = quat_normalize(box_quat)
                continue
            R = quat2mat(xquat[p])
            pos = xpos[p] + R @ np.array(body_pos[b])
            q = quat_mul(xquat[p], np.array(body_quat[b]))
            if b in jnt_body:
                j = jnt_body.index(b)
                xanchor[j] = pos.copy()
                xaxis[j] = quat2mat(q) @ np.array(jnt_axis[j])
                q = quat_mul(q, axis_angle_quat(jnt_axis[j], qarm[j]))
            xpos[b] = pos; xquat[b] = quat_normalize(q)
        return xpos, xquat, xanchor, xaxis

    box_pos0 = bodies["box"]["pos"]
    xpos, xquat, xanchor, xaxis = fk(np.zeros(6), box_pos0, [1, 0, 0, 0])

    # ---- mass matrix at qpos0 by the Jacobian method (independent of the CRBA in oracle/ and csrc/)
    nv = 12
    M = np.zeros((nv, nv))
    jac_com = {}
    for b in range(1, nbody):
        if body_mass[b] == 0:
            continue
        R = quat2mat(xquat[b])
        c = xpos[b] + R @ np.array(body_ipos[b])
        Ri = R @ quat2mat(body_iquat[b])
        Iw = Ri @ np.diag(body_inertia[b]) @ Ri.T
        Jv = np.zeros((3, nv)); Jw = np.zeros((3, nv))
        if names[b] == "box":
            Jv[:, 6:9] = np.eye(3)
            Jw[:, 9:12] = R                 # free-joint angular dofs are body-frame axes
            Jv[:, 9:12] = np.array([np.cross(R[:, k], c - xpos[b]) for k in range(3)]).T
        else:
            a = b
            while a > 0:
                if a in jnt_body:
                    j = jnt_body.index(a)
                    Jw[:, j] = xaxis[j]
                    Jv[:, j] = np.cross(xaxis[j], c - xanchor[j])
                a = body_parent[a]
        M += body_mass[b] * Jv.T @ Jv + Jw.T @ Iw @ Jw
        jac_com[b] = np.vstack([Jv, Jw])
    M += np.diag(dof_armature)
    Minv = np.linalg.inv(M)
    dof_M0 = np.diag(M).tolist()
    dof_invweight0 = []
    for k in range(6):
        dof_invweight0.append(Minv[k, k])
    tr = float(np.mean(np.diag(Minv)[6:9])); rot = float(np.mean(np.diag(Minv)[9:12]))
    dof_invweight0 += [tr] * 3 + [rot] * 3
    body_invweight0 = [[0.0, 0.0]]
    for b in range(1, nbody):
        if b not in jac_com or names[b] == "Base":
            body_invweight0.append([0.0, 0.0]); continue
        J = jac_com[b]
        A = J @ Minv @ J.T
        body_invweight0.append([float(np.trace(A[:3, :3]) / 3), float(np.trace(A[3:, 3:]) / 3)])
    meaninertia = float(np.trace(M) / nv)

    # ---- actuators ----
    act_kp, act_kv, act_forcerange, act_ctrlrange = [], [], [], []
    for a in actuators:
        j = hinge_names.index(a["joint"])
        kp = float(a["kp"])
        dr = float(a.get("dampratio", 0))
        act_kp.append(kp)
        act_kv.append(dr * 2.0 * math.sqrt(kp * dof_M0[j]))
        act_forcerange.append(vec(a["forcerange"], 2).tolist())
        assert a.get("inheritrange") in ("1", "1.0")
        act_ctrlrange.append(jnt_range[j])

    # ---- collision geoms in scope: table (box hull), 8 pads, cube, 5 bin boxes ----
    geoms = []

    def add_geom(name, body, pos, quat, size, g):
        geoms.append(dict(name=name, body=body, pos=list(map(float, pos)), quat=list(map(float, quat)),
                          size=list(map(float, size)),
                          condim=int(g.get("condim", MJ_CONDIM)),
                          friction=(vec(g["friction"]).tolist() if "friction" in g else MJ_FRICTION),
                          solref=(vec(g["solref"]).tolist() if "solref" in g else MJ_SOLREF),
                          solimp=((vec(g["solimp"]).tolist() + MJ_SOLIMP[3:])[:5] if "solimp" in g
                                  else MJ_SOLIMP)))

    # table: tabletop.stl (scale 0.001) has exactly 8 hull vertices = an axis-aligned box
    tb = bodies["table"]; tg = tb["geoms"][0]
    v = load_stl(os.path.join(ASSETS, "tabletop.stl")) * 0.001
    lo, hi = v.min(0), v.max(0)
    add_geom("table", 0, tb["pos"] + (lo + hi) / 2, [1, 0, 0, 0], (hi - lo) / 2, tg)
    for side, bname in (("fixed", "Fixed_Jaw"), ("moving", "Moving_Jaw")):
        pads = [g for g in bodies[bname]["geoms"] if g.get("name", "").startswith(side + "_jaw_pad_")]
        assert len(pads) == 4
        for g in pads:
            add_geom(g["name"], bid[bname], vec(g["pos"], 3), [1, 0, 0, 0], vec(g["size"], 3), g)
    cg = bodies["box"]["geoms"][0]
    add_geom(cg["name"], bid["box"], vec(cg.get("pos", "0 0 0"), 3), [1, 0, 0, 0], vec(cg["size"], 3), cg)
    binb = bodies["bin"]
    for g in binb["geoms"]:
        add_geom(g["name"], 0, binb["pos"] + vec(g["pos"], 3), [1, 0, 0, 0], vec(g["size"], 3), g)
    # geom 15: the EE variant's mocap marker box (so_arm100_ee.xml:155: a group-0 box with the default contype /
    # conaffinity, so MuJoCo collides it).  Its body is the mocap body (MOCAP_BODY, no dofs: its pose is the env's
    # mocap input); it exists in both variants' tables, its pairs are collided only in the EE variant.
    ee_root = ET.parse(os.path.join(ASSETS, "trs_so_arm100", "so_arm100_ee.xml")).getroot()
    mocap_b = [b for b in ee_root.find("worldbody").findall("body") if b.get("mocap") == "true"][0]
    mg = mocap_b.find("geom")
    assert mg.get("type") == "box" and not mg.get("pos") and not mg.get("quat") and not mg.get("contype")
    add_geom("mocap_target_box", MOCAP_BODY, [0, 0, 0], [1, 0, 0, 0], vec(mg.get("size"), 3), dict(mg.attrib))
    gid = {g["name"]: i for i, g in enumerate(geoms)}
    assert len(geoms) == 16

    # ---- arm/jaw collision hulls (convex hulls of the class="collision" meshes of the moving bodies) ----
    from scipy.spatial import ConvexHull
    hulls = []
    for bname in ARM_BODIES[1:] + ARM_BODIES[:1]:      # the 9 link hulls, then the static Base's (hull 9)
        for g in bodies[bname]["geoms"]:
            if g.get("type") != "mesh" or g.get("group") != "3" or g.get("contype", "1") == "0":
                continue
            v = load_stl(os.path.join(ASSETS, "trs_so_arm100", g["mesh"] + ".stl"))
            pos = vec(g.get("pos", "0 0 0"), 3)
            assert not g.get("quat") and not g.get("euler"), "collision mesh with a rotated frame"
            hv = v[ConvexHull(v).vertices] + pos
            lo, hi = hv.min(0), hv.max(0)
            c = (lo + hi) / 2
            # volume centroid of the (closed) mesh: MuJoCo re-centres a mesh geom on its inertial frame,
            # so geom_xpos -- the centre mjc_Convex's MPR starts its portal from -- is this point
            tri = v.reshape(-1, 3, 3)
            vol6 = np.einsum("ij,ij->i", tri[:, 0], np.cross(tri[:, 1], tri[:, 2]))
            assert vol6.sum() > 0, g["mesh"]
            centroid = (vol6[:, None] * tri.sum(1)).sum(0) / (4 * vol6.sum()) + pos
            hulls.append(dict(name=g["mesh"], body=bid[bname], verts=hv.tolist(), center=c.tolist(),
                              centroid=centroid.tolist(),
                              half=((hi - lo) / 2).tolist(),
                              condim=int(g.get("condim", MJ_CONDIM)),
                              friction=(vec(g["friction"]).tolist() if "friction" in g else MJ_FRICTION),
                              solref=(vec(g["solref"]).tolist() if "solref" in g else MJ_SOLREF),
                              solimp=((vec(g["solimp"]).tolist() + MJ_SOLIMP[3:])[:5] if "solimp" in g
                                      else MJ_SOLIMP)))
    tbl = geoms[gid["table"]]
    table_plane = dict(top=tbl["pos"][2] + tbl["size"][2],
                       lo=[tbl["pos"][0] - tbl["size"][0], tbl["pos"][1] - tbl["size"][1]],
                       hi=[tbl["pos"][0] + tbl["size"][0], tbl["pos"][1] + tbl["size"][1]])

    # ---- contact pairs (geom1, geom2 in MuJoCo's orientation: type order box<mesh, then id) ----
    pair_names = ([(f"fixed_jaw_pad_{i}", "red_box") for i in range(1, 5)]
                  + [(f"moving_jaw_pad_{i}", "red_box") for i in range(1, 5)]
                  + [("red_box", "table")]
                  + [("red_box", n) for n in ("bin_wall", "bin_wall2", "bin_wall3", "bin_wall4", "bin_floor")])
    pairs = []

    def mixed(g1, g2):
        mix = 0.5   # solmix defaults 1 and 1
        return dict(condim=max(g1["condim"], g2["condim"]),
                    friction=[max(a, b) for a, b in zip(g1["friction"], g2["friction"])],
                    solref=[mix * a + (1 - mix) * b for a, b in zip(g1["solref"], g2["solref"])],
                    solimp=[mix * a + (1 - mix) * b for a, b in zip(g1["solimp"], g2["solimp"])],
                    margin=0.0, gap=0.0)

    for n1, n2 in pair_names:
        g1, g2 = geoms[gid[n1]], geoms[gid[n2]]
        pairs.append(dict(g1=gid[n1], g2=gid[n2], body1=g1["body"], body2=g2["body"], name1=n1, name2=n2,
                          **mixed(g1, g2)))
    # (table, hull k): geom1 = the table (world geom, lower id), normal from the table to the hull
    for k, h in enumerate(hulls[:9]):
        pairs.append(dict(g1=gid["table"], g2=-1 - k, body1=0, body2=h["body"], name1="table", name2=h["name"],
                          hull=k, **mixed(tbl, h)))
    # (box, hull k) through the general convex collider (MPR): geom1 = the box (MuJoCo orders a pair by
    # geom type, box < mesh), normal from the box to the hull.  Pairs 23..31: the cube against every
    # arm/jaw hull; pairs 32..76: bin box j (walls, floor) against hull k at 32 + 9 j + k (the static
    # Base hull against the static bin boxes is a static-static pair, filtered).
    boxes = ["red_box"] + ["bin_wall", "bin_wall2", "bin_wall3", "bin_wall4", "bin_floor"]
    for n1 in boxes:
        g1 = geoms[gid[n1]]
        for k, h in enumerate(hulls[:9]):
            pairs.append(dict(g1=gid[n1], g2=-1 - k, body1=g1["body"], body2=h["body"], name1=n1,
                              name2=h["name"], hull=k, **mixed(g1, h)))
    # Pairs 77..97: hull-hull self-collision of the arm, through the same collider.  MuJoCo filters only
    # parent-child body pairs and the explicit exclude (Base / Rotation_Pitch, so_arm100.xml:165-167);
    # geom1 = the hull on the body nearer the root, normal from it to the other.
    parent = {bid[n]: bid[bodies[n]["parent"]] if bodies[n]["parent"] in bid else 0 for n in ARM_BODIES}
    excl = {frozenset((bid[a], bid[b])) for a, b in excludes}
    for k1, h1 in enumerate(hulls[:9]):
        for k2, h2 in enumerate(hulls[:9]):
            b1, b2 = h1["body"], h2["body"]
            if not b1 < b2 or parent[b2] == b1 or frozenset((b1, b2)) in excl:
                continue
            pairs.append(dict(g1=-1 - k1, g2=-1 - k2, body1=b1, body2=b2, name1=h1["name"], name2=h2["name"],
                              hull=k2, hull1=k1, **mixed(h1, h2)))

    # Pairs 98..106: the static Base's hull (hull 9).  The Base has no joint, so MuJoCo's parent filter
    # (which skips world-welded bodies) does not apply; the model's exclude removes Rotation_Pitch, and the
    # static-static rule the table and the bin.  (red_box, Base): box < mesh, geom1 = the cube; (Base, hull
    # k): the Base's geom has the lower id, geom1 = the Base hull.
    assert len(hulls) == 10 and hulls[9]["body"] == bid["Base"]
    pairs.append(dict(g1=gid["red_box"], g2=-1 - 9, body1=geoms[gid["red_box"]]["body"], body2=bid["Base"],
                      name1="red_box", name2=hulls[9]["name"], hull=9, **mixed(geoms[gid["red_box"]], hulls[9])))
    for k, h in enumerate(hulls[:9]):
        if frozenset((bid["Base"], h["body"])) in excl:
            continue
        pairs.append(dict(g1=-1 - 9, g2=-1 - k, body1=bid["Base"], body2=h["body"], name1=hulls[9]["name"],
                          name2=h["name"], hull=k, hull1=9, **mixed(hulls[9], h)))
    assert len(pairs) == 107
    # Pairs 107..142: the finger pads (boxes on the jaws) against the arm's own link hulls, through MPR:
    # the Base (hull 9), Rotation_Pitch, Upper_Arm, Lower_Arm (hulls 0..2) and Wrist_Pitch_Roll (hull 3),
    # less the fixed-jaw pads vs Wrist_Pitch_Roll (their parent body: MuJoCo's parent filter).  geom1 = the
    # pad (box < mesh), normal from the pad to the hull.
    pads = [f"{side}_jaw_pad_{i}" for side in ("fixed", "moving") for i in range(1, 5)]
    for n1 in pads:
        g1 = geoms[gid[n1]]
        for k in (9, 0, 1, 2, 3):
            h = hulls[k]
            if parent[g1["body"]] == h["body"]:
                continue
            pairs.append(dict(g1=gid[n1], g2=-1 - k, body1=g1["body"], body2=h["body"], name1=n1,
                              name2=h["name"], hull=k, **mixed(g1, h)))
    assert len(pairs) == 143
    # Pairs 143..151 (EE variant only): the mocap marker box against the 9 link hulls, through the convex
    # collider (MuJoCo's static-static filter removes the marker against the table, the bin and the Base: a mocap
    # body is welded to the world; geom1 = the box, box < mesh)
    mk = geoms[gid["mocap_target_box"]]
    for k, h in enumerate(hulls[:9]):
        pairs.append(dict(g1=gid["mocap_target_box"], g2=-1 - k, body1=MOCAP_BODY, body2=h["body"],
                          name1="mocap_target_box", name2=h["name"], hull=k, ee_only=True, **mixed(mk, h)))
    assert len(pairs) == 152
    # Pairs 152..159: the 8 finger pads against the table; 160..199: against the 5 bin boxes (160 + 5 i + j).
    # geom1 = the pad: the table is a mesh (box < mesh) and the bin boxes come after the arm in the model
    # (so100_transfer_cube.xml includes the arm before the bin), so the normal points from the pad to the
    # table / bin box.  Pad-table contacts follow the hull-table rule (one per pair); pad-bin pairs are
    # box-box like the cube's.
    pad_pairs = ([(n1, "table") for n1 in pads]
                 + [(n1, n2) for n1 in pads for n2 in ("bin_wall", "bin_wall2", "bin_wall3", "bin_wall4", "bin_floor")])
    for n1, n2 in pad_pairs:
        g1, g2 = geoms[gid[n1]], geoms[gid[n2]]
        pairs.append(dict(g1=gid[n1], g2=gid[n2], body1=g1["body"], body2=g2["body"], name1=n1, name2=n2,
                          **mixed(g1, g2)))
    assert len(pairs) == 200
    # Pairs 200..208 (EE variant only): the cube and the 8 finger pads against the mocap marker box, box-box (the
    # marker has the highest geom id: geom1 = the cube / pad, normal towards the marker)
    for n1 in ["red_box"] + pads:
        g1 = geoms[gid[n1]]
        pairs.append(dict(g1=gid[n1], g2=gid["mocap_target_box"], body1=g1["body"], body2=MOCAP_BODY, name1=n1,
                          name2="mocap_target_box", ee_only=True, **mixed(g1, mk)))
    assert len(pairs) == 209

    # ---- EE / mocap variant (so100_transfer_cube_ee.xml: the same scene with trs_so_arm100/so_arm100_ee.xml,
    # whose only differences are the mocap body at :155 and the weld equality at :171-173) ----
    ee = ET.parse(os.path.join(ASSETS, "trs_so_arm100", "so_arm100_ee.xml")).getroot()
    weld = ee.find("equality").find("weld")
    assert weld.get("site1") == "mocap_target_site" and weld.get("site2") == "ee_site"
    mocap = [b for b in ee.find("worldbody").findall("body") if b.get("mocap") == "true"][0]
    msite = [x for x in mocap.findall("site") if x.get("name") == "mocap_target_site"][0]
    assert vec(msite.get("pos", "0 0 0"), 3).tolist() == [0, 0, 0] and not msite.get("quat")
    cf = bodies["vx300s_left/camera_focus"]
    assert bodies["vx300s_left/camera_focus"]["parent"] == "Fixed_Jaw" and np.allclose(cf["quat"], [1, 0, 0, 0])
    ee_local = cf["pos"] + vec([x for x in cf["sites"] if x["name"] == "ee_site"][0].get("pos", "0 0 0"), 3)
    # body_invweight0 of the ee_site body (massless, COM at its origin; welded to Fixed_Jaw) at qpos0
    fj = bid["Fixed_Jaw"]
    c = xpos[fj] + quat2mat(xquat[fj]) @ ee_local
    Jv = np.zeros((3, nv)); Jw = np.zeros((3, nv))
    a = fj
    while a > 0:
        if a in jnt_body:
            j = jnt_body.index(a)
            Jw[:, j] = xaxis[j]
            Jv[:, j] = np.cross(xaxis[j], c - xanchor[j])
        a = body_parent[a]
    Aw = np.vstack([Jv, Jw]) @ Minv @ np.vstack([Jv, Jw]).T
    solimp = vec(weld.get("solimp"), 3).tolist() + [0.5, 2.0]          # MuJoCo defaults for mid, power
    weld_info = dict(body2=fj, pos2=ee_local.tolist(), quat2=[1.0, 0.0, 0.0, 0.0],
                     solref=vec(weld.get("solref"), 2).tolist(), solimp=solimp,
                     torquescale=float(weld.get("torquescale", 1)),
                     invweight0=[float(np.trace(Aw[:3, :3]) / 3), float(np.trace(Aw[3:, 3:]) / 3)],
                     mocap_pos=vec(mocap.get("pos"), 3).tolist(), mocap_quat=[1.0, 0.0, 0.0, 0.0],
                     mocap_box=dict(size=vec(mocap.find("geom").get("size"), 3).tolist()))

    # ---- sites ----
    cube_site = vec(bodies["box"]["sites"][0]["pos"], 3)
    cf = bodies["vx300s_left/camera_focus"]
    ee_site = cf["pos"] + vec([s for s in cf["sites"] if s["name"] == "ee_site"][0].get("pos", "0 0 0"), 3)
    bin_center = binb["pos"] + vec([s for s in binb["sites"] if s["name"] == "bin_center"][0]["pos"], 3)

    model = dict(
        source="derived from /root/reference/gym_so100/assets/so100_transfer_cube.xml by tools/compile_model.py",
        nbody=nbody, body_names=names, body_parent=body_parent, body_pos=body_pos, body_quat=body_quat,
        body_ipos=body_ipos, body_iquat=body_iquat, body_mass=body_mass, body_inertia=body_inertia,
        body_invweight0=body_invweight0,
        jnt_names=hinge_names + ["red_box_joint"], jnt_body=jnt_body, jnt_axis=jnt_axis, jnt_range=jnt_range,
        jnt_solref=MJ_SOLREF, jnt_solimp=MJ_SOLIMP,
        dof_armature=dof_armature, dof_frictionloss=dof_frictionloss, dof_invweight0=dof_invweight0,
        dof_M0=dof_M0, dof_solref=MJ_SOLREF, dof_solimp=MJ_SOLIMP,
        act_kp=act_kp, act_kv=act_kv, act_forcerange=act_forcerange, act_ctrlrange=act_ctrlrange,
        geoms=geoms, pairs=pairs, hulls=hulls, table_plane=table_plane,
        site_cube=dict(body=bid["box"], pos=cube_site.tolist()),
        site_ee=dict(body=bid["Fixed_Jaw"], pos=ee_site.tolist()),
        site_bin_center=bin_center.tolist(),
        opt=dict(timestep=MJ_TIMESTEP, gravity=MJ_GRAVITY, impratio=float(opt.get("impratio", 1)),
                 cone=opt.get("cone", "pyramidal"), iterations=MJ_ITERATIONS, tolerance=MJ_TOLERANCE,
                 meaninertia=meaninertia),
        qpos0_box=box_pos0.tolist(),
        M0=M.tolist(),
        weld=weld_info,
    )
    return model


if __name__ == "__main__":
    m = compile_model()
    out = sys.argv[1] if len(sys.argv) > 1 else OUT
    with open(out, "w") as f:
        json.dump(m, f, indent=1)
    print("wrote", os.path.abspath(out))
    print("dof_M0", np.round(m["dof_M0"], 6))
    print("kv", np.round(m["act_kv"], 4))
    print("meaninertia", m["opt"]["meaninertia"])
