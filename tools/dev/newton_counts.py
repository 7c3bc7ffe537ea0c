"""Newton work per substep in the fp32 oracle (so100o_newton_counts: gradient evaluations, Hessian + Cholesky
factorizations, line searches) on the bench workload (64 spawns x 30 random-action steps) and EE episodes, for the tree's
oracle ("cur") and oracle variants built to oracle/build/liboracle32_<name>.so (e.g. -DNEWTON_QUADSTOP=0).
usage: python tools/dev/newton_counts.py cur [name ...]"""
import sys, numpy as np, ctypes
import os
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "gym-so100-c_amd")); sys.path.insert(0, os.path.join(R, "tools", "dev"))
from oracle.oracle import Oracle
from gym_so100.model import build_model
from mixed_precision import ee_episodes, set_mocap
libs = {k: (None if k == "cur" else os.path.join(R, "oracle", "build", f"liboracle32_{k}.so")) for k in sys.argv[1:]}
for cls in ("bench", "ee"):
    model = build_model(variant="ee" if cls == "ee" else "joint")
    for name, path in libs.items():
        o = Oracle(32, path=path); o64 = Oracle(64)
        d = o.new_data(); its = []
        c = (ctypes.c_long * 3).in_dll(o.lib, "so100o_newton_counts"); c[0] = c[1] = c[2] = 0
        rng = np.random.default_rng(0)
        eps = ee_episodes(model, o64, 16) if cls == "ee" else [(None, None)] * 64
        for i, (q0, mocap) in enumerate(eps):
            if cls == "ee":
                o.set_state(d, q0, np.zeros(12), np.zeros(12)); set_mocap(d, mocap)
            else:
                o.reset(model, d, o.spawn_pose(1000 + i))
            for t in range(30):
                c = o.unnormalize(model, rng.uniform(-1, 1, 6).astype(np.float32))
                for k in range(6): d.ctrl[k] = float(c[k])
                for s in range(10):
                    o.call("so100o_substep", model, d); its.append(d.solver_iter)
        c = (ctypes.c_long * 3).in_dll(o.lib, "so100o_newton_counts")
        n = len(its)
        print(cls, name, f"per substep: gradients {c[0]/n:.2f}, Hessian+Cholesky {c[1]/n:.2f}, line searches {c[2]/n:.2f}")
