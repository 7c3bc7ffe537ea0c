#!/usr/bin/env python3
"""GPU-vs-oracle parity report (test infrastructure; run on the GPU box).

Teacher-forced: before every env step the oracle env is set to the GPU state (fp32 values), both take
the same action, and the per-step differences in qpos/qvel/reward/contacts are recorded.  Prints a
summary and writes gpurun_out/parity_report.json.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from gym_so100 import SO100VecEnv  # noqa: E402
from gym_so100.model import build_model  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402


def main(n=64, steps=60, bits=64, task=0, seed=1000):
    t0 = time.time()
    env = SO100VecEnv(n, device="cuda:0", autoreset=False, debug=True, max_episode_steps=0)
    model = build_model()
    o = Oracle(bits)
    obs, _ = env.reset(seed=seed)
    torch.cuda.synchronize()
    # reset parity
    d = o.new_data()
    max_reset = 0.0
    for i in range(n):
        o.reset(model, d, o.spawn_pose(seed + i))
        ob = o.observe(model, d)
        max_reset = max(max_reset, float(np.abs(ob - obs[i].cpu().numpy()).max()))
    print(f"reset obs max|diff| = {max_reset:.3e}")
    rng = np.random.default_rng(0)
    errs = {"qpos": [], "qvel": [], "reward_mismatch": 0, "bits_mismatch": 0, "ncon_mismatch": 0, "iters": []}
    datas = [o.new_data() for _ in range(n)]
    for step in range(steps):
        qpos = env.qpos.cpu().numpy().astype(np.float64)
        qvel = env.qvel.cpu().numpy().astype(np.float64)
        warm = env.qacc_warmstart.cpu().numpy().astype(np.float64)
        # mostly-tracking random actions: hold near the start pose with noise, some full random
        if step % 20 < 10:
            act = rng.uniform(-1, 1, size=(n, 6)).astype(np.float32)
        else:
            act = np.clip(rng.normal(0, 0.3, size=(n, 6)), -1, 1).astype(np.float32)
        _, rew, term, trunc, info = env.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gq = env.qpos.cpu().numpy().astype(np.float64)
        gv = env.qvel.cpu().numpy().astype(np.float64)
        gr = rew.cpu().numpy()
        gb = info["contact_bits"].cpu().numpy().astype(np.uint32)
        dbg = env.debug.cpu().numpy()
        for i in range(n):
            dd = datas[i]
            o.set_state(dd, qpos[i], qvel[i], warm[i])
            ob, r, t = o.env_step(model, dd, task, act[i])
            oq, ov, _, _ = o.get_state(dd)
            errs["qpos"].append(np.abs(oq - gq[i]))
            errs["qvel"].append(np.abs(ov - gv[i]) / (1.0 + np.abs(ov)))
            if abs(r - gr[i]) > 1e-5:
                errs["reward_mismatch"] += 1
            if o.contact_bits(dd) != gb[i]:
                errs["bits_mismatch"] += 1
            errs["iters"].append((dd.solver_iter, dbg[i, 1]))
    qp = np.array(errs["qpos"])
    qv = np.array(errs["qvel"])
    rep = {
        "n": n, "steps": steps, "oracle_bits": bits,
        "qpos_absdiff_max": float(qp.max()), "qpos_absdiff_p99": float(np.quantile(qp.max(1), 0.99)),
        "qpos_absdiff_median": float(np.median(qp.max(1))),
        "qvel_reldiff_max": float(qv.max()), "qvel_reldiff_p99": float(np.quantile(qv.max(1), 0.99)),
        "qvel_reldiff_median": float(np.median(qv.max(1))),
        "reward_mismatch": errs["reward_mismatch"], "bits_mismatch": errs["bits_mismatch"],
        "frac_qvel_within_1e-4": float(np.mean(qv.max(1) < 1e-4)),
        "frac_qvel_within_1e-3": float(np.mean(qv.max(1) < 1e-3)),
        "seconds": time.time() - t0,
    }
    print(json.dumps(rep, indent=1))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"parity_report_{bits}.json"), "w") as f:
        json.dump(rep, f, indent=1)
    worst = np.argsort(qv.max(1))[-5:]
    for w in worst:
        print("worst", w, "step", w // n, "env", w % n, "qvel rel", qv[w].round(5))


if __name__ == "__main__":
    bits = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    main(bits=bits)
