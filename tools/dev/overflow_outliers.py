"""The largest GPU errors of test_overflow_contact_parity's states (contact lists longer than 16), with the fp32
restatement's error, the ensemble of 1-ulp perturbations and the contact lists of each (GPU box; test-side tool).

    python tools/dev/overflow_outliers.py [newton|pgs] [nsubstep]
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
        T._arm_contact_parity(solver, o64, o32, 0, NPAIR, "overflow", 29, nsubstep=nsub, select=lambda d: d.ncon > 16)
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
        print(f"step {i}: GPU qvel err {r.qv[i]:.3e} qacc {r.qa[i]:.3e} | fp32 oracle {r.fqv[i]:.3e} | ensemble "
              f"{np.array2string(np.asarray(r.eqv[i]), precision=2)} | ncon GPU {len(gp)} oracle {len(p64)} same {r.same[i]}")
        if len(gp) != len(p64) or not np.array_equal(gp, p64):
            print("   pairs GPU ", list(gp))
            print("   pairs fp64", list(p64))


if __name__ == "__main__":
    main()
