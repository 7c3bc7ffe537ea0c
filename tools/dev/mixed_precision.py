"""Which stage's fp32 arithmetic carries the error on the contact-rich classes? (CPU only.)

The fp32 restatement of the oracle misses north_star's 1e-4 on the table-edge and EE classes by as much as the GPU
does, while the fp64 oracle's response to a 1-ulp perturbation of the state stays near 3e-6: the amplifier is fp32
ARITHMETIC somewhere in the substep, not fp32 state.  This tool runs the oracle's substep stage by stage
(so100o_stage: kinematics, CRB + weld fold + factor, collision, constraint rows, velocity, smooth acceleration,
solve, Euler), each stage in fp64 (liboracle64) or fp32 (liboracle32), converting the whole so100o_data between the
two builds' layouts at each change of precision, and measures each mix's qvel error against the all-fp64 step on
the classes' states.

    python tools/dev/mixed_precision.py [--cls table_edge|ee|both] [--states 48] [--steps 3]

Rows: "all fp32" (the fp32 restatement), "fp32 but S in fp64" for each stage S (how much of the error S carries),
"fp64 but S in fp32" (whether S alone reproduces it)."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
from oracle.oracle import Oracle, NQ, NV  # noqa: E402
from gym_so100.model import build_model  # noqa: E402

STAGES = ["kin", "crb", "coll", "constr", "vel", "smooth", "solve", "euler"]


class Converter:
    """copies an so100o_data between the fp64 and the fp32 builds' layouts, field by field (reals converted,
    ints copied; the contact array element by element)"""

    def __init__(self, o64, o32):
        self.o64, self.o32 = o64, o32
        self.fields = []
        for (name, t64), (_, t32) in zip(o64.Data._fields_, o32.Data._fields_):
            f64, f32 = getattr(o64.Data, name), getattr(o32.Data, name)
            if name == "con":
                self.fields.append((name, f64.offset, f32.offset, "con", None))
                continue
            base = t64
            while hasattr(base, "_length_"):
                base = base._type_
            kind = "real" if base in (ctypes.c_double,) else "int"
            self.fields.append((name, f64.offset, f32.offset, kind, f64.size))
        c64, c32 = o64.Contact, o32.Contact
        self.csz64, self.csz32 = ctypes.sizeof(c64), ctypes.sizeof(c32)
        self.cpair64, self.cpair32 = c64.pair.offset, c32.pair.offset
        self.ncon_off64 = o64.Data.ncon.offset

    @staticmethod
    def _bytes(d):
        return np.frombuffer((ctypes.c_char * ctypes.sizeof(d)).from_address(ctypes.addressof(d)), np.uint8)

    def convert(self, src, dst, to32):
        b_src, b_dst = self._bytes(src), self._bytes(dst)
        for name, o64, o32, kind, size in self.fields:
            so, do = (o64, o32) if to32 else (o32, o64)
            if kind == "con":
                n = src.ncon
                ss, ds = (self.csz64, self.csz32) if to32 else (self.csz32, self.csz64)
                sp, dp = (self.cpair64, self.cpair32) if to32 else (self.cpair32, self.cpair64)
                st, dt = (np.float64, np.float32) if to32 else (np.float32, np.float64)
                sr = np.lib.stride_tricks.as_strided
                for c in range(n):
                    sv = b_src[so + c * ss: so + c * ss + 13 * np.dtype(st).itemsize].view(st)
                    b_dst[do + c * ds: do + c * ds + 13 * np.dtype(dt).itemsize].view(dt)[:] = sv
                    b_dst[do + c * ds + dp: do + c * ds + dp + 4] = b_src[so + c * ss + sp: so + c * ss + sp + 4]
                del sr
            elif kind == "int":
                b_dst[do: do + size] = b_src[so: so + size]
            else:
                n = size // 8
                if to32:
                    b_dst[o32: o32 + 4 * n].view(np.float32)[:] = b_src[o64: o64 + 8 * n].view(np.float64)
                else:
                    b_dst[o64: o64 + 8 * n].view(np.float64)[:] = b_src[o32: o32 + 4 * n].view(np.float32)


def mixed_step(model, o64, o32, conv, d64, d32, ctrl, prec, nsub):
    """one env step's substeps with stage k in fp32 where prec[k] == 32; starts from d64's state, ends in d64"""
    for k in range(NU):
        d64.ctrl[k] = float(ctrl[k])
    cur = 64
    for _ in range(nsub):
        for k, p in enumerate(prec):
            if p != cur:
                if p == 32:
                    conv.convert(d64, d32, True)
                else:
                    conv.convert(d32, d64, False)
                cur = p
            (o32 if p == 32 else o64).lib.so100o_stage(Oracle._p(model), Oracle._p(d32 if p == 32 else d64), k)
    if cur == 32:
        conv.convert(d32, d64, False)


NU = 6


def rel(a, o):
    return (np.abs(a - o) / (1 + np.abs(o))).max()


def states_for(cls, model, o64, nstates, seed):
    """the GPU tests' state generators (tests/test_gpu_parity.py): table-edge = _arm_contact_parity(seed 31, a table
    contact with a non-vertical normal), ee = the EE variant's rollout states"""
    from gym_so100.model import NPAIR_BOX, NHULL, PAIR_PAD0, PAIR_PADBIN0
    rng = np.random.default_rng(seed)
    lo_j = np.array([r[0] for r in model.jnt_range]); hi_j = np.array([r[1] for r in model.jnt_range])
    lo, hi = np.array(model.action_lo[:]), np.array(model.action_hi[:])
    d = o64.new_data()
    table = lambda p: NPAIR_BOX <= p < NPAIR_BOX + NHULL or PAIR_PAD0 <= p < PAIR_PADBIN0
    out = []
    while len(out) < nstates:
        arm = rng.uniform(lo_j, hi_j)
        o64.reset(model, d, np.array([0.4, 0.95, 0.6, 1, 0, 0, 0]))
        for k in range(6):
            d.qpos[k] = arm[k]
        o64.call("so100o_fwd_position", model, d)
        if cls == "table_edge":
            ok = any(table(d.con[i].pair) and abs(d.con[i].frame[2]) < 0.99 for i in range(d.ncon))
        elif cls == "base":            # test_base_contact_parity's class: a link against the static Base's hull
            from gym_so100.model import PAIR_BASE0, PAIR_PADLINK0
            ok = any(PAIR_BASE0 <= d.con[i].pair < PAIR_PADLINK0 for i in range(d.ncon)) and not d.ncon_dropped
        else:
            ok = True
        if ok:
            q = np.array(d.qpos[:], np.float64)
            out.append((q, np.clip((arm - lo) / (hi - lo) * 2 - 1, -1, 1)))
    return out


def ee_episodes(model, o64, n=32):
    """tests/test_gpu_parity.py::test_ee_weld_parity's workload: spawns RandomState(77 + i), mocap targets within 4 cm
    and 0.4 rad of the start end-effector frame, 30 random-action steps"""
    from scipy.spatial.transform import Rotation
    d = o64.new_data()
    rng = np.random.default_rng(5)
    out = []
    for i in range(n):
        o64.reset(model, d, o64.spawn_pose(77 + i))
        o64.call("so100o_fwd_position", model, d)
        R = np.array(d.xmat[6][:]).reshape(3, 3)
        rot = Rotation.from_rotvec(rng.uniform(-0.4, 0.4, 3)) * Rotation.from_matrix(R)
        mocap = np.zeros(7)
        mocap[:3] = np.array(d.site_ee[:]) + rng.uniform(-0.04, 0.04, 3)
        mocap[3:] = rot.as_quat()[[3, 0, 1, 2]]
        out.append((np.array(d.qpos[:]), mocap))
    return out


def set_mocap(d, mocap):
    if mocap is None:
        return
    for k in range(3):
        d.mocap_pos[k] = float(mocap[k])
    for k in range(4):
        d.mocap_quat[k] = float(mocap[3 + k])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cls", default="table_edge", choices=["table_edge", "ee", "base"])
    ap.add_argument("--states", type=int, default=48)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--lib32", default=None, help="another fp32 build of the oracle (experiments)")
    ap.add_argument("--rows", default="", help="comma-separated mix names to print (default all)")
    args = ap.parse_args()
    o64, o32 = Oracle(64), Oracle(32, path=args.lib32)
    for o in (o64, o32):
        o.lib.so100o_stage.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    conv = Converter(o64, o32)
    variant = "ee" if args.cls == "ee" else "joint"
    model = build_model(solver="newton", variant=variant)
    nsub = model.nsubstep
    if args.cls == "ee":
        act_rng = np.random.default_rng(77)
        eps = ee_episodes(model, o64, args.states)
        acts = [act_rng.uniform(-1, 1, (len(eps), 6)) if t % 20 < 10 else np.clip(act_rng.normal(0, 0.3, (len(eps), 6)), -1, 1)
                for t in range(args.steps)]
        episodes = [(q, mocap, [acts[t][i] for t in range(args.steps)]) for i, (q, mocap) in enumerate(eps)]
    else:
        seed = {"table_edge": 31, "base": 19}[args.cls]
        rng = np.random.default_rng(seed)
        episodes = [(q, None, [np.clip(target + rng.normal(0, 0.02, 6), -1, 1) for _ in range(args.steps)])
                    for q, target in states_for(args.cls, model, o64, args.states, seed)]
    mixes = [("all fp64", [64] * 8), ("all fp32", [32] * 8)]
    for k, s in enumerate(STAGES):
        mixes.append((f"fp32, {s} in fp64", [64 if j == k else 32 for j in range(8)]))
    for k, s in enumerate(STAGES):
        mixes.append((f"fp64, {s} in fp32", [32 if j == k else 64 for j in range(8)]))
    errs = {name: [] for name, _ in mixes}
    d64, dref, d32 = o64.new_data(), o64.new_data(), o32.new_data()
    for i, (q0, mocap, actions) in enumerate(episodes):
        q, v, w = q0.copy(), np.zeros(NV), np.zeros(NV)
        for act in actions:
            act = np.asarray(act, np.float32)
            # fp32 state, as the GPU's teacher-forced states are
            q, v, w = q.astype(np.float32).astype(np.float64), v.astype(np.float32).astype(np.float64), \
                w.astype(np.float32).astype(np.float64)
            ctrl = o64.unnormalize(model, act)
            o64.set_state(dref, q, v, w)
            set_mocap(dref, mocap)
            mixed_step(model, o64, o32, conv, dref, d32, ctrl, [64] * 8, nsub)
            vref = np.array(dref.qvel[:])
            for name, prec in mixes[1:]:
                o64.set_state(d64, q, v, w)
                set_mocap(d64, mocap)
                mixed_step(model, o64, o32, conv, d64, d32, ctrl, prec, nsub)
                errs[name].append(rel(np.array(d64.qvel[:]), vref))
            errs["all fp64"].append(0.0)
            q, v, w = np.array(dref.qpos[:]), vref, np.array(dref.qacc_warmstart[:])
        print(f"episode {i + 1}/{len(episodes)}", file=sys.stderr, flush=True)
    print(f"{args.cls}: {len(episodes)} states x {len(episodes[0][2])} teacher-forced env steps (Newton, {nsub} substeps); "
          f"qvel rel. error vs all-fp64: median / p90 / p99 / max, share within 1e-4")
    for name, _ in mixes[1:]:
        if args.rows and name not in args.rows.split(","):
            continue
        e = np.array(errs[name])
        print(f"  {name:28s} {np.median(e):.2e} / {np.quantile(e, .9):.2e} / {np.quantile(e, .99):.2e} / "
              f"{e.max():.2e}  {np.mean(e < 1e-4):.3f}")


if __name__ == "__main__":
    main()
