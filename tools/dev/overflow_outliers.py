"""The largest GPU errors of test_overflow_contact_parity's states (contact lists longer than 16), with the fp32
restatement's error, the ensemble of 1-ulp perturbations and the contact lists of each (GPU box; test-side tool).

    python tools/dev/overflow_outliers.py [newton|pgs] [nsubstep, 0 = the model's 10] [states.npz] [overflow|base|self|padlink]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "gym-so100-c_amd"), ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import test_gpu_parity as T  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from gym_so100.model import NPAIR, build_model  # noqa: E402


def main():
    solver = sys.argv[1] if len(sys.argv) > 1 else "newton"
    nsub = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    nsub = nsub or None
    case = sys.argv[4] if len(sys.argv) > 4 else "overflow"
    from gym_so100.model import PAIR_SELF0, PAIR_BASE0, PAIR_PADLINK0, PAIR_MOCAPHULL0
    cases = {"overflow": (0, NPAIR, 29, lambda d: d.ncon > 16), "base": (PAIR_BASE0, PAIR_PADLINK0, 19, None),
             "self": (PAIR_SELF0, PAIR_BASE0, 17, None), "padlink": (PAIR_PADLINK0, PAIR_MOCAPHULL0, 23, None)}
    p0, p1, seed, select = cases[case]
    o64, o32 = Oracle(64), Oracle(32)
    orig = T._ensemble_bars
    T._ensemble_bars = lambda r, name="qv": np.zeros(len(r.qv), bool)     # report, do not assert
    keep = {}
    orig_tf = T._tf_run

    def tf(*a, **k):
        r = orig_tf(*a, **k)
        keep["r"] = r
        return r
    T._tf_run = tf
    try:
        T._arm_contact_parity(solver, o64, o32, p0, p1, case, seed, nsubstep=nsub, select=select)
    except AssertionError as e:
        print("assertion:", e)
    T._ensemble_bars = orig
    r = keep["r"].arrays() if not isinstance(keep["r"].qv, np.ndarray) else keep["r"]
    model = build_model(solver=solver, nsubstep=nsub)
    order = np.argsort(-r.qv)[:8]
    d = o64.new_data()
    for i in order:
        q0, v0, w0, act = r.states[i][:4]
        o64.set_state(d, q0, v0, w0)
        o64.env_step(model, d, 0, act)
        p64, f64, _, qa64, _ = o64.last_solve(d)
        gp = r.pairs[i]
        print(f"step {i}: GPU qvel err {r.qv[i]:.3e} qacc {r.qa[i]:.3e} | fp32 oracle {r.fqv[i]:.3e} (FMA {r.mqv[i]:.3e}) | ensemble "
              f"{np.array2string(np.asarray(r.eqv[i]), precision=2)} | ncon GPU {len(gp)} oracle {len(p64)} same {r.same[i]}")
        if len(gp) != len(p64) or not np.array_equal(gp, p64):
            print("   pairs GPU ", list(gp))
            print("   pairs fp64", list(p64))
    for i in order[:3]:
        detail(r, int(i), solver, nsub)
    # the outlier states, for a CPU replay of their collision (tools/dev/epa_replay.py)
    if len(sys.argv) > 3:
        np.savez(sys.argv[3], **{f"s{int(i)}": np.concatenate([np.ravel(x) for x in r.states[int(i)][:4]]) for i in order})



def detail(r, idx, solver, nsub):
    """one state again, alone, with the debug record: per contact (pair, dist, forces) GPU vs the fp64 oracle"""
    import torch
    from gym_so100 import SO100VecEnv
    from gym_so100.model import build_model
    o64 = Oracle(64)
    model = build_model(solver=solver, nsubstep=nsub)
    q0, v0, w0, act = r.states[idx][:4]
    env = SO100VecEnv(1, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver=solver, nsubstep=nsub)
    env.reset(seed=3)
    env.set_state(q0[None].astype(np.float32), v0[None].astype(np.float32), w0[None].astype(np.float32))
    env.step(torch.as_tensor(act[None], dtype=torch.float32).cuda())
    torch.cuda.synchronize()
    dbg = env.debug.cpu().numpy()[0]
    gp, gf, _, gqa = T._gpu_solve(dbg)
    from gym_so100._native import SO100_DBG_OVF
    nc = int(dbg[0])
    gd = np.concatenate([dbg[16:16 + min(nc, 16)], dbg[SO100_DBG_OVF:SO100_DBG_OVF + 6 * max(nc - 16, 0)].reshape(-1, 6)[:, 0]])
    d = o64.new_data()
    o64.set_state(d, q0, v0, w0)
    o64.env_step(model, d, 0, act)
    p64, f64, _, qa64, _ = o64.last_solve(d)
    # the solve's contact list in the oracle (nsub = 1: the position stage of the step's one substep), fp64 and fp32
    o32 = Oracle(32)
    cons = []
    for o in (o64, o32):
        d2 = o.new_data()
        o.set_state(d2, q0, v0, w0)
        o.call("so100o_fwd_position", model, d2)
        cons.append([(d2.con[i].pair, d2.con[i].dist, np.array(d2.con[i].pos[:]), np.array(d2.con[i].frame[:3]))
                     for i in range(d2.ncon)])
    d32 = o32.new_data()
    o32.set_state(d32, q0, v0, w0)
    o32.env_step(model, d32, 0, act)
    p32, f32, _, qa32, _ = o32.last_solve(d32)
    print(f"--- state {idx}: GPU ncon {nc}, oracle {len(p64)}; qacc GPU {np.array2string(gqa, precision=4)}\n"
          f"    fp64 qacc {np.array2string(qa64, precision=4)}\n    fp32 qacc {np.array2string(qa32, precision=4)}")
    for c in range(max(nc, len(p64))):
        g = f"pair {gp[c]:3d} dist {gd[c]: .4e} f {np.array2string(gf[c], precision=4)}" if c < nc else "-"
        o = (f"pair {p64[c]:3d} dist {cons[0][c][1]: .4e} (fp32 {cons[1][c][1]: .4e}) f {np.array2string(f64[c], precision=4)}"
             f" (fp32 {np.array2string(f32[c], precision=4)}) n {np.array2string(cons[0][c][3], precision=4)}"
             if c < len(p64) and c < len(cons[1]) else "-")
        print(f"  c{c:2d} GPU {g} | fp64 {o}")
    env.close()


if __name__ == "__main__":
    main()
