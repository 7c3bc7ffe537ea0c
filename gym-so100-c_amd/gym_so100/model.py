"""Derived SO-ARM100 model table -> ``so100_model`` C struct (include/so100_model.h).

The table (assets/so100_model.json) is produced by tools/compile_model.py from the reference MJCF
(/root/reference/gym_so100/assets/so100_transfer_cube.xml, loaded by the reference at
gym_so100/env.py:111-112).  Task constants below mirror the reference's Python module constants and
cite them; they are data, not compute.
"""
import ctypes
import json
import os

import numpy as np

from . import constants as C

ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "so100_model.json")

NBODY, NHINGE, NQ, NV, NU, NGEOM = 9, 6, 13, 12, 6, 16
MOCAP_GEOM, MOCAP_BODY = 15, 9                  # the EE variant's mocap marker box and its (mocap) body
NPAIR_BOX, NHULL, HULL_NVERT, NBINBOX = 14, 9, 2560, 5
PAIR_MPR0 = NPAIR_BOX + NHULL                  # (box, hull) pairs of the MPR convex collider start here
PAIR_SELF0 = PAIR_MPR0 + (1 + NBINBOX) * NHULL  # 77: hull-hull self-collision pairs
NHULL_ALL, HULL_BASE = NHULL + 1, NHULL          # hull arrays hold the static Base's hull at index 9
NPAIR_SELF = 21
PAIR_BASE0 = PAIR_SELF0 + NPAIR_SELF             # 98: (cube, Base hull), 99..106 (Base hull, hull k = 1..8)
PAIR_PADLINK0 = PAIR_BASE0 + 9                   # 107: (pad, link hull) pairs 107..142 through MPR
NPAIR_PADLINK = 36
PAIR_MOCAPHULL0 = PAIR_PADLINK0 + NPAIR_PADLINK  # 143: (mocap marker, link hull k) 143..151, EE only, convex
PAIR_PAD0 = PAIR_MOCAPHULL0 + NHULL              # 152: (pad i, table) pairs 152..159
PAIR_PADBIN0 = PAIR_PAD0 + 8                     # 160: (pad i, bin box j) at 160 + 5 i + j, box-box
NPAIR_PAD = 8 * (1 + NBINBOX)                    # 48
PAIR_MOCAPBOX0 = PAIR_PAD0 + NPAIR_PAD           # 200: (cube | pad i, mocap marker) 200..208, EE only, box-box
NPAIR = PAIR_MOCAPBOX0 + 9                       # 209
NPAIR_BITS = PAIR_MPR0                         # contact_bits covers pairs 0..22
MAXCON, CONDIM, NOBS = 16, 4, 15      # MAXCON: contacts an env holds on chip (include/so100_model.h)
NCON_MAX = 62 * 8 + 209 - 62           # SO100_NCON_MAX: the whole contact list (every pair at its maximum)
NEFC_MAX = NV + NHINGE + NCON_MAX * CONDIM

_d = ctypes.c_double
_i = ctypes.c_int


def _arr(t, *dims):
    for n in reversed(dims):
        t = t * n
    return t


class SO100Model(ctypes.Structure):
    """Mirror of ``so100_model`` (include/so100_model.h) — field order must match exactly."""
    _fields_ = [
        ("timestep", _d), ("nsubstep", _i), ("iterations", _i), ("solver", _i), ("tolerance", _d),
        ("impratio", _d),
        ("gravity", _arr(_d, 3)), ("meaninertia", _d),
        ("body_parent", _arr(_i, NBODY)), ("body_pos", _arr(_d, NBODY, 3)), ("body_quat", _arr(_d, NBODY, 4)),
        ("body_ipos", _arr(_d, NBODY, 3)), ("body_iquat", _arr(_d, NBODY, 4)), ("body_mass", _arr(_d, NBODY)),
        ("body_inertia", _arr(_d, NBODY, 3)), ("body_invweight0", _arr(_d, NBODY, 2)),
        ("jnt_body", _arr(_i, NHINGE)), ("jnt_axis", _arr(_d, NHINGE, 3)), ("jnt_range", _arr(_d, NHINGE, 2)),
        ("jnt_solref", _arr(_d, 2)), ("jnt_solimp", _arr(_d, 5)),
        ("dof_armature", _arr(_d, NV)), ("dof_frictionloss", _arr(_d, NV)), ("dof_invweight0", _arr(_d, NV)),
        ("dof_solref", _arr(_d, 2)), ("dof_solimp", _arr(_d, 5)),
        ("act_kp", _arr(_d, NU)), ("act_kv", _arr(_d, NU)), ("act_forcerange", _arr(_d, NU, 2)),
        ("act_ctrlrange", _arr(_d, NU, 2)),
        ("geom_body", _arr(_i, NGEOM)), ("geom_pos", _arr(_d, NGEOM, 3)), ("geom_quat", _arr(_d, NGEOM, 4)),
        ("geom_size", _arr(_d, NGEOM, 3)),
        ("pair_geom1", _arr(_i, NPAIR)), ("pair_geom2", _arr(_i, NPAIR)),
        ("pair_body1", _arr(_i, NPAIR)), ("pair_body2", _arr(_i, NPAIR)), ("pair_condim", _arr(_i, NPAIR)),
        ("pair_friction", _arr(_d, NPAIR, 3)), ("pair_solref", _arr(_d, NPAIR, 2)),
        ("pair_solimp", _arr(_d, NPAIR, 5)), ("pair_margin", _arr(_d, NPAIR)),
        ("hull_body", _arr(_i, NHULL_ALL)), ("hull_start", _arr(_i, NHULL_ALL)), ("hull_count", _arr(_i, NHULL_ALL)),
        ("hull_center", _arr(_d, NHULL_ALL, 3)), ("hull_half", _arr(_d, NHULL_ALL, 3)),
        ("hull_centroid", _arr(_d, NHULL_ALL, 3)),
        ("hull_vert", _arr(_d, HULL_NVERT, 3)),
        ("table_top", _d), ("table_lo", _arr(_d, 2)), ("table_hi", _arr(_d, 2)),
        ("site_cube_body", _i), ("site_cube_pos", _arr(_d, 3)), ("site_ee_body", _i), ("site_ee_pos", _arr(_d, 3)),
        ("bin_center", _arr(_d, 3)),
        ("start_qpos", _arr(_d, NU)), ("action_lo", _arr(_d, NU)), ("action_hi", _arr(_d, NU)),
        ("spawn_lo", _arr(_d, 3)), ("spawn_hi", _arr(_d, 3)),
        ("bin_hw", _d), ("bin_h", _d), ("cube_half", _d), ("goal_threshold", _d), ("max_reward", _d),
        ("goal_bin_lo", _arr(_d, 3)), ("goal_bin_hi", _arr(_d, 3)),
        ("ee", ctypes.c_int), ("weld_pos2", _arr(_d, 3)), ("weld_quat2", _arr(_d, 4)), ("weld_solref", _arr(_d, 2)),
        ("weld_solimp", _arr(_d, 5)), ("weld_torquescale", _d), ("weld_invweight0", _arr(_d, 2)),
        ("mocap_pos0", _arr(_d, 3)), ("mocap_quat0", _arr(_d, 4)),
        ("convex", _i),
    ]


def _set(m, name, values):
    f = getattr(m, name)
    flat = np.asarray(values).reshape(-1)
    if not hasattr(f, "_length_"):
        setattr(m, name, type(f)(flat[0]) if not isinstance(f, float) else float(flat[0]))
        return

    def rec(arr, vals):
        if hasattr(arr[0], "_length_"):
            step = len(vals) // len(arr)
            for k in range(len(arr)):
                rec(arr[k], vals[k * step:(k + 1) * step])
        else:
            for k in range(len(arr)):
                arr[k] = vals[k].item() if hasattr(vals[k], "item") else vals[k]
    rec(f, flat)


def load_model_dict(path=ASSET):
    with open(path) as f:
        return json.load(f)


VARIANTS = ("joint", "ee")
SOLVERS = {"pgs": 0, "newton": 1}      # SO100_SOLVER_* (include/so100_model.h)
CONVEX = {"mpr": 0, "epa": 1}          # SO100_CONVEX_* (include/so100_model.h)


def build_model(path=ASSET, iterations=None, nsubstep=None, solver="newton", variant="joint", convex="epa"):
    """Return an ``SO100Model`` ctypes struct filled from the derived model table.

    solver: "newton" (default: MuJoCo's default solver, which the reference's model uses --
    so_arm100.xml:4 sets no solver) or "pgs" (north_star's projected Gauss-Seidel).
    convex: the collider of the mesh pairs: "epa" (default: GJK + EPA, MuJoCo 3.3.3's default native
    convex collider, the minimum penetration) or "mpr" (libccd's MPR, MuJoCo behind mjDSBL_NATIVECCD).
    variant: "joint" (so100_transfer_cube.xml, the registered envs) or "ee" (so100_transfer_cube_ee.xml:
    a weld equality pulls ee_site to a per-env mocap pose, so_arm100_ee.xml:155,171-173)."""
    if variant not in VARIANTS:
        raise ValueError(f"variant {variant!r}: one of {VARIANTS}")
    d = load_model_dict(path)
    m = SO100Model()
    o = d["opt"]
    m.timestep = o["timestep"]
    m.nsubstep = int(round(C.DT / o["timestep"])) if nsubstep is None else int(nsubstep)   # env.py:120-127
    m.iterations = int(o["iterations"] if iterations is None else iterations)
    m.solver = SOLVERS[solver]
    if convex not in CONVEX:
        raise ValueError(f"convex {convex!r}: one of {tuple(CONVEX)}")
    m.convex = CONVEX[convex]
    m.tolerance = o["tolerance"]
    m.impratio = o["impratio"]
    _set(m, "gravity", o["gravity"])
    m.meaninertia = o["meaninertia"]
    for k in ("body_parent",):
        _set(m, k, np.asarray(d[k], dtype=np.int64))
    for k in ("body_pos", "body_quat", "body_ipos", "body_iquat", "body_mass", "body_inertia", "body_invweight0",
              "jnt_axis", "jnt_range", "jnt_solref", "jnt_solimp", "dof_armature", "dof_frictionloss",
              "dof_invweight0", "dof_solref", "dof_solimp", "act_kp", "act_kv", "act_forcerange", "act_ctrlrange"):
        _set(m, k, np.asarray(d[k], dtype=np.float64))
    _set(m, "jnt_body", np.asarray(d["jnt_body"], dtype=np.int64))
    g = d["geoms"]
    _set(m, "geom_body", np.asarray([x["body"] for x in g], dtype=np.int64))
    _set(m, "geom_pos", np.asarray([x["pos"] for x in g]))
    _set(m, "geom_quat", np.asarray([x["quat"] for x in g]))
    _set(m, "geom_size", np.asarray([x["size"] for x in g]))
    p = d["pairs"]
    _set(m, "pair_geom1", np.asarray([x["g1"] for x in p], dtype=np.int64))
    _set(m, "pair_geom2", np.asarray([x["g2"] for x in p], dtype=np.int64))
    _set(m, "pair_condim", np.asarray([x["condim"] for x in p], dtype=np.int64))
    _set(m, "pair_friction", np.asarray([x["friction"] for x in p]))
    _set(m, "pair_solref", np.asarray([x["solref"] for x in p]))
    _set(m, "pair_solimp", np.asarray([x["solimp"] for x in p]))
    _set(m, "pair_margin", np.asarray([x["margin"] - x["gap"] for x in p]))
    _set(m, "pair_body1", np.asarray([x["body1"] for x in p], dtype=np.int64))
    _set(m, "pair_body2", np.asarray([x["body2"] for x in p], dtype=np.int64))
    h = d["hulls"]
    assert len(h) == NHULL_ALL and len(p) == NPAIR
    counts = [len(x["verts"]) for x in h]
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    verts = np.zeros((HULL_NVERT, 3))
    allv = np.concatenate([np.asarray(x["verts"]) for x in h])
    assert len(allv) <= HULL_NVERT
    verts[:len(allv)] = allv
    _set(m, "hull_body", np.asarray([x["body"] for x in h], dtype=np.int64))
    _set(m, "hull_start", starts)
    _set(m, "hull_count", np.asarray(counts, dtype=np.int64))
    _set(m, "hull_center", np.asarray([x["center"] for x in h]))
    _set(m, "hull_half", np.asarray([x["half"] for x in h]))
    _set(m, "hull_centroid", np.asarray([x["centroid"] for x in h]))
    _set(m, "hull_vert", verts)
    tp = d["table_plane"]
    m.table_top = tp["top"]
    _set(m, "table_lo", tp["lo"])
    _set(m, "table_hi", tp["hi"])
    m.site_cube_body = d["site_cube"]["body"]
    _set(m, "site_cube_pos", d["site_cube"]["pos"])
    m.site_ee_body = d["site_ee"]["body"]
    _set(m, "site_ee_pos", d["site_ee"]["pos"])
    _set(m, "bin_center", d["site_bin_center"])
    # task constants (reference cited in constants.py)
    _set(m, "start_qpos", C.SO100_START_ARM_POSE)
    _set(m, "action_lo", [r[0] for r in C.SO100_ACTION_RANGES])
    _set(m, "action_hi", [r[1] for r in C.SO100_ACTION_RANGES])
    _set(m, "spawn_lo", [r[0] for r in C.SO100_BOX_SPAWN_RANGES])
    _set(m, "spawn_hi", [r[1] for r in C.SO100_BOX_SPAWN_RANGES])
    m.bin_hw = C.BIN_HALF_WIDTH
    m.bin_h = C.BIN_INNER_HEIGHT
    m.cube_half = C.CUBE_HALF
    m.goal_threshold = C.GOAL_DISTANCE_THRESHOLD
    m.max_reward = C.MAX_REWARD
    # SO100GoalEnv.bin_goal_space (env.py:245-249): float32 bin_min/max (constants.py:29-30) +- 0.005
    lo = [float(np.float32(C.bin_min[0]) + np.float32(0.005)), float(np.float32(C.bin_min[1]) + np.float32(0.005)), 0.01]
    hi = [float(np.float32(C.bin_max[0]) - np.float32(0.005)), float(np.float32(C.bin_max[1]) - np.float32(0.005)), 0.05]
    _set(m, "goal_bin_lo", lo)
    _set(m, "goal_bin_hi", hi)
    w = d["weld"]
    m.ee = 1 if variant == "ee" else 0
    _set(m, "weld_pos2", w["pos2"])
    _set(m, "weld_quat2", w["quat2"])
    _set(m, "weld_solref", w["solref"])
    _set(m, "weld_solimp", w["solimp"])
    m.weld_torquescale = w["torquescale"]
    _set(m, "weld_invweight0", w["invweight0"])
    _set(m, "mocap_pos0", w["mocap_pos"])
    _set(m, "mocap_quat0", w["mocap_quat"])
    return m


def pair_names(path=ASSET):
    d = load_model_dict(path)
    return [(p["name1"], p["name2"]) for p in d["pairs"]]
