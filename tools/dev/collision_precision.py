"""Contact-by-contact fp32 error of the collision stage, by pair class (CPU only; follows tools/dev/mixed_precision.py,
which found the collision stage to carry the table-edge class's fp32 error).

On each state the fp64 oracle runs kinematics .. CRB; the data is rounded to fp32 and collision runs in both builds
on the same (fp32-representable) frames.  Contacts are matched by pair (and order within a pair); per class the depth
error (m), the normal's angle error (rad) and the position error (m).

    python tools/dev/collision_precision.py [--cls table_edge] [--states 200]"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mixed_precision import Converter, states_for, ROOT  # noqa: E402,F401
from oracle.oracle import Oracle  # noqa: E402
from gym_so100.model import build_model, NPAIR_BOX, NHULL, PAIR_MPR0, PAIR_PAD0, PAIR_PADBIN0  # noqa: E402


def cls_of(p, table_fast):
    if p == 8:
        return "cube-table (SAT)"
    if NPAIR_BOX <= p < NPAIR_BOX + NHULL:
        return "hull-table top-face rule" if table_fast else "hull-table GJK+EPA"
    if PAIR_PAD0 <= p < PAIR_PADBIN0:
        return "pad-table (SAT)"
    if p < NPAIR_BOX or p >= PAIR_PADBIN0:
        return "box-box"
    return "convex (GJK+EPA)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cls", default="table_edge")
    ap.add_argument("--states", type=int, default=200)
    args = ap.parse_args()
    o64, o32 = Oracle(64), Oracle(32)
    for o in (o64, o32):
        o.lib.so100o_stage.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    conv = Converter(o64, o32)
    model = build_model(solver="newton")
    sts = states_for(args.cls, model, o64, args.states, 31)
    d64, d32, dq = o64.new_data(), o32.new_data(), o64.new_data()
    res = {}
    for q, _ in sts:
        q = q.astype(np.float32).astype(np.float64)
        o64.set_state(d64, q, np.zeros(12), np.zeros(12))
        for k in (0, 1):
            o64.lib.so100o_stage(Oracle._p(model), Oracle._p(d64), k)
        conv.convert(d64, d32, True)
        conv.convert(d32, dq, False)         # the same fp32-rounded frames in fp64
        o64.lib.so100o_stage(Oracle._p(model), Oracle._p(dq), 2)
        o32.lib.so100o_stage(Oracle._p(model), Oracle._p(d32), 2)
        c64 = [(dq.con[i].pair, np.array(dq.con[i].pos[:]), np.array(dq.con[i].frame[:3]), dq.con[i].dist)
               for i in range(dq.ncon)]
        c32 = [(d32.con[i].pair, np.array(d32.con[i].pos[:], np.float64), np.array(d32.con[i].frame[:3], np.float64),
                float(d32.con[i].dist)) for i in range(d32.ncon)]
        p64, p32 = [c[0] for c in c64], [c[0] for c in c32]
        if p64 != p32:
            res.setdefault("list differs", []).append((0, 0, 0))
            continue
        for a, b in zip(c64, c32):
            # the top-face rule's contacts have a vertical normal at the lowest vertex
            fast = abs(a[2][2]) > 0.999999 and NPAIR_BOX <= a[0] < NPAIR_BOX + NHULL
            ang = np.arccos(np.clip(np.dot(a[2], b[2]) / np.linalg.norm(a[2]) / np.linalg.norm(b[2]), -1, 1))
            res.setdefault(cls_of(a[0], fast), []).append((abs(a[3] - b[3]), ang, np.linalg.norm(a[1] - b[1])))
    print(f"{len(sts)} {args.cls} states: fp32 collision vs fp64 on the same fp32 frames; per class median / p90 / max")
    for k, v in sorted(res.items()):
        v = np.array(v)
        q = lambda x: f"{np.median(x):.1e} / {np.quantile(x, .9):.1e} / {x.max():.1e}"
        print(f"  {k:26s} n={len(v):5d}  depth {q(v[:, 0])} m  normal {q(v[:, 1])} rad  pos {q(v[:, 2])} m")


if __name__ == "__main__":
    main()
