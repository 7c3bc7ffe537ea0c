"""One dumped state (tools/dev/overflow_outliers.py states.npz) stepped substep by substep on the GPU (a model with
nsubstep = 1, the action held) beside the fp64 / fp32 / fp32-FMA oracle: per substep the qacc difference and each
contact's pair, depth and forces, to find where the GPU leaves the restatement (GPU box; test-side tool).

    python tools/dev/substep_trace.py states.npz s98 [newton|pgs] [nsub]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "gym-so100-c_amd"), ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import test_gpu_parity as T  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from gym_so100 import SO100VecEnv  # noqa: E402
from gym_so100.model import build_model  # noqa: E402


def main():
    Z = np.load(sys.argv[1])
    s = Z[sys.argv[2]]
    solver = sys.argv[3] if len(sys.argv) > 3 else "newton"
    nsub = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    q0, v0, w0, act = s[:13], s[13:25], s[25:37], s[37:43].astype(np.float32)
    model = build_model(solver=solver, nsubstep=1)
    env = SO100VecEnv(1, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver=solver, nsubstep=1)
    env.reset(seed=3)
    env.set_state(q0[None].astype(np.float32), v0[None].astype(np.float32), w0[None].astype(np.float32))
    ors = {"fp64": Oracle(64), "fp32": Oracle(32), "fma": Oracle(32, fma=True)}
    ds = {}
    for k, o in ors.items():
        ds[k] = o.new_data()
        o.set_state(ds[k], q0, v0, w0)
    a = torch.as_tensor(act[None]).cuda()
    for sub in range(nsub):
        env.step(a)
        torch.cuda.synchronize()
        dbg = env.debug.cpu().numpy()[0]
        gp, gf, _, gqa = T._gpu_solve(dbg)
        gd = dbg[16:16 + min(len(gp), 16)]
        res = {}
        for k, o in ors.items():
            o.env_step(model, ds[k], 0, act)
            res[k] = o.last_solve(ds[k])
        p64, f64, _, qa64, _ = res["fp64"]
        line = (f"sub {sub}: ncon GPU {len(gp)} fp64 {len(p64)} | GPU iters {int(dbg[1])} impr {dbg[2]:.2e}, fp64 "
                f"{ds['fp64'].solver_iter} {ds['fp64'].solver_improvement:.2e}, fp32 {ds['fp32'].solver_iter} "
                f"{ds['fp32'].solver_improvement:.2e} | qacc |GPU-fp64| {np.abs(gqa - qa64).max():.3e}")
        for k in ("fp32", "fma"):
            line += f" |{k}-fp64| {np.abs(res[k][3] - qa64).max():.3e}"
        print(line)
        print(f"   qacc GPU {np.array2string(gqa, precision=4)}\n   qacc fp64 {np.array2string(qa64, precision=4)}")
        for c in range(max(len(gp), len(p64))):
            g = f"{gp[c]:3d} d {gd[c]: .5e} f {np.array2string(gf[c], precision=3)}" if c < len(gp) and c < 16 else "-"
            o = f"{p64[c]:3d} f {np.array2string(f64[c], precision=3)}" if c < len(p64) else "-"
            print(f"   c{c:2d} GPU {g} | fp64 {o}")
        # teacher forcing: every side continues from the GPU's state
        qg, vg, wg = (env.qpos.cpu().numpy()[0].astype(np.float64), env.qvel.cpu().numpy()[0].astype(np.float64),
                      env.qacc_warmstart.cpu().numpy()[0].astype(np.float64))
        for k, o in ors.items():
            o.set_state(ds[k], qg, vg, wg)
    env.close()


if __name__ == "__main__":
    main()
