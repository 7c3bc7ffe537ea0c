"""Per-step device time of the benchmark's workload from reset (GPU box only): the bench's setup (env i reset with
RandomState(1000 + i), the seeded U[-1,1]^6 action pool), then one HIP-event pair around every step on the launch
stream, steps 0..S-1, no warmup.  Shows where in the episode the driver's 20-step window (--warmup 5) sits against
the builder's 300-step window (--warmup 30).

    python tools/gpurun/step_series.py <tree root> <envs> <steps> <out.json>

The tree root's own gym_so100 is imported, so an old revision's tree (abtree/<name>) runs its own library."""
import json
import os
import sys

root, n, steps, out = os.path.abspath(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
sys.path.insert(0, os.path.join(root, "gym-so100-c_amd"))
import torch  # noqa: E402
from gym_so100 import SO100VecEnv  # noqa: E402

dev = torch.device("cuda", 0)
env = SO100VecEnv(n, device="cuda:0", seed=0)
env.reset(seed=1000)
g = torch.Generator(device=dev)
g.manual_seed(0)
pool = [(torch.rand(n, 6, generator=g, device=dev) * 2 - 1).contiguous() for _ in range(16)]
stream = torch.cuda.current_stream(dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
torch.cuda.synchronize()
ev[0].record(stream)
for i in range(steps):
    env.set_action_buffer(pool[i % len(pool)])
    env.step_async_raw()
    ev[i + 1].record(stream)
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]
json.dump({"root": root, "envs": n, "ms": ms}, open(out, "w"))
w = lambda a, b: sum(ms[a:b]) / (b - a)
print(f"{root} n={n}: steps 0-4 {w(0, 5):.3f} ms, 5-24 (driver window) {w(5, 25):.3f} ms, 30-329 (builder window) "
      f"{w(30, min(330, steps)):.3f} ms")
env.close()
