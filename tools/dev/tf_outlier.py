"""Teacher-forced outlier probe (GPU dev tool): rebuild the state set of a parity test, find the env step whose
GPU qvel is furthest from the fp64 oracle, and walk that step one substep at a time (nsubstep = 1 envs) on
the GPU's product and debug kernels and in both oracles: per substep the qvel error, the contact lists with
their distances, and the contact forces.

    python tools/dev/tf_outlier.py mpr pgs epa [out.npz]
    python tools/dev/tf_outlier.py heavy pgs epa
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
from oracle.oracle import Oracle  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def mpr_states(o64, model):
    from gym_so100.model import PAIR_MPR0, PAIR_PAD0
    rng = np.random.default_rng(21)
    d = o64.new_data()
    states = []
    for e in range(128):
        o64.reset(model, d, o64.spawn_pose(2000 + e))
        for _ in range(200):
            o64.env_step(model, d, 0, rng.uniform(-1, 1, 6).astype(np.float32))
            mp = [d.con[i].pair for i in range(d.ncon) if PAIR_MPR0 <= d.con[i].pair < PAIR_PAD0]
            if mp and not d.ncon_dropped:
                states.append(o64.get_state(d)[:3])
                break
        if len(states) >= 48:
            break
    return states, rng, lambda rng, n: rng.uniform(-1, 1, (n, 6)), 3


def heavy_states(o64, model):
    """test_heavy_contact_parity's states: the cube pressed into a bin corner (floor + two walls)"""
    n = 32
    rng = np.random.default_rng(7)
    d = o64.new_data()
    o64.reset(model, d, o64.spawn_pose(5))
    q_start = o64.get_state(d)[0]
    pen = rng.uniform(2e-4, 1e-3, (n, 3))
    ang = rng.uniform(-0.01, 0.01, n)
    states = []
    for i in range(n):
        q = q_start.copy()
        q[6] = -0.145 - 0.02 + pen[i, 0]
        q[7] = 0.755 - 0.02 + pen[i, 1]
        q[8] = 0.001 + 0.02 - pen[i, 2]
        q[9:13] = [np.cos(ang[i] / 2), 0, 0, np.sin(ang[i] / 2)]
        v = np.zeros(12)
        v[6:9] = rng.normal(0, 0.02, 3)
        states.append((np.float32(q).astype(np.float64), np.float32(v).astype(np.float64), np.zeros(12)))
    return states, rng, lambda rng, n: rng.uniform(-0.2, 0.2, (n, 6)), 3


def main():
    which, solver, convex = sys.argv[1], sys.argv[2], sys.argv[3]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "gpurun_out", f"tf_outlier_{which}_{solver}_{convex}.npz")
    from gym_so100.model import build_model
    o64, o32 = Oracle(64), Oracle(32)
    model = build_model(solver=solver, convex=convex)
    states, rng, act, steps = {"mpr": mpr_states, "heavy": heavy_states}[which](o64, model)
    n = len(states)
    env = T._new_env(n, solver, convex=convex)
    env.reset(seed=3)
    T._set_states(env, states)
    r = T._tf_run(env, model, o64, o32, steps, lambda step: act(rng, n)).arrays()
    env.close()
    print(r.summary(f"{which} {solver} {convex}"))
    key = r.qa if os.environ.get("BY_QACC") else r.qv
    order = np.argsort(-key)[:4]
    print("worst env-steps (qv, fqv, pqv, qa, fqa, pqa):", [(int(k), float(r.qv[k]), float(r.fqv[k]), float(r.pqv[k]),
                                  float(r.qa[k]), float(r.fqa[k]), float(r.pqa[k])) for k in order])
    k = int(order[0])
    q0, v0, w0, a = r.states[k][:4]
    np.savez(out, q0=q0, v0=v0, w0=w0, act=a, qv=r.qv, fqv=r.fqv, pqv=r.pqv)
    # substep walk: a 1-substep env (an env step = one mj_step + the final mj_step1) stepped 10 times
    m1 = build_model(solver=solver, convex=convex, nsubstep=1)
    e1 = T._new_env(1, solver, convex=convex, nsubstep=1)
    e1.reset(seed=3)
    e1.set_state(q0[None].astype(np.float32), v0[None].astype(np.float32), w0[None].astype(np.float32))
    ds = {b: o.new_data() for b, o in ((64, o64), (32, o32))}
    for b, o in ((64, o64), (32, o32)):
        o.set_state(ds[b], q0, v0, w0)
    for s in range(10):
        _, _, _, dbg, _ = T._step_all_builds(e1, a[None])
        gv = e1.qvel.cpu().numpy()[0]
        gp, gf, _, gqa = T._gpu_solve(dbg[0])
        gd = dbg[0][16:16 + len(gp)]
        line = [f"substep {s}: GPU pairs {gp.tolist()} dist {np.round(gd * 1e3, 4).tolist()} mm fN {np.round(gf[:, 0], 5).tolist()}"]
        ov = None
        for b, o in ((64, o64), (32, o32)):
            o.env_step(m1, ds[b], 0, a)
            p, f, _, qa, _ = o.last_solve(ds[b])
            # distances of the last solve's contacts: the data's contacts were replaced by the final stage;
            # the final stage recomputes the same substep's positions only for the NEXT substep, so report f
            v = o.get_state(ds[b])[1]
            if b == 64:
                ov = v
            line.append(f"  o{b} pairs {p.tolist()} fN {np.round(f[:, 0], 5).tolist()} qvel rel vs o64 {T._rel(v, ov):.2e}")
        line.append(f"  GPU qvel rel vs o64 {T._rel(gv, ov):.2e}  qacc rel {T._rel(gqa, o64.last_solve(ds[64])[3]):.2e}")
        print("\n".join(line))
        # teacher-force the next substep from the GPU state in the oracles (isolates the substep that diverges)
        gq, gw = e1.qpos.cpu().numpy()[0].astype(np.float64), e1.qacc_warmstart.cpu().numpy()[0].astype(np.float64)
        for b, o in ((64, o64), (32, o32)):
            o.set_state(ds[b], gq, gv.astype(np.float64), gw)
    e1.close()


if __name__ == "__main__":
    main()
