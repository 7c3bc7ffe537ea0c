"""Where the 16-contacts-per-env cap bites (dev probe, CPU): the fp64 oracle runs the bench workload
(env i reset with RandomState(1000 + i), U[-1,1]^6 actions) and reports, per env step, the envs whose
position stages dropped contacts, with the pair classes of their contact lists.

    python tools/dev/contact_drops.py [nenv] [steps]
"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))
from oracle.oracle import Oracle  # noqa: E402
from gym_so100 import model as M  # noqa: E402


def pair_class(p):
    if p < M.NPAIR_BOX:
        return f"box{p}"
    if p < M.PAIR_MPR0:
        return "hull-table"
    if p < M.PAIR_SELF0:
        return "box-hull"
    if p < M.PAIR_BASE0:
        return "self"
    if p < M.PAIR_PADLINK0:
        return "base"
    if p < M.PAIR_PAD0:
        return "pad-link"
    if p < M.PAIR_PADBIN0:
        return "pad-table"
    return "pad-bin"


def main():
    nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    o = Oracle(64)
    m = M.build_model()
    datas = (o.Data * nenv)()
    for i in range(nenv):
        o.reset(m, datas[i], o.spawn_pose(1000 + i))
    rng = np.random.default_rng(0)
    drops, hist, ncon_hist = 0, collections.Counter(), collections.Counter()
    for s in range(steps):
        acts = rng.uniform(-1, 1, size=(1, nenv, 6)).astype(np.float32)
        o.batch_run(m, datas, nenv, 1, 0, acts, nthreads=os.cpu_count())
        for i in range(nenv):
            d = datas[i]
            ncon_hist[d.snap_ncon] += 1
            if d.snap_ndrop:
                drops += d.snap_ndrop
                cls = collections.Counter(pair_class(d.snap_pair[c]) for c in range(d.snap_ncon))
                hist[tuple(sorted(cls.items()))] += 1
                if sum(hist.values()) <= 5:
                    print(f"step {s} env {i}: dropped {d.snap_ndrop}, list {dict(cls)}")
    print(f"{nenv} envs x {steps} steps: dropped {drops} ({drops / (nenv * steps):.2e} per env step)")
    print("last-substep contact count histogram:", dict(sorted(ncon_hist.items())))
    for k, v in hist.most_common(10):
        print(v, dict(k))


if __name__ == "__main__":
    main()
