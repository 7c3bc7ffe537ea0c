#!/usr/bin/env python3
"""Benchmark: env steps/sec (whole node) for 65,536 parallel bin-a-cube envs on 1/2/4/8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--total-envs 65536 | --envs-per-gpu E]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one batched env step of every env on every GPU: action prologue, 10 physics substeps
(kinematics, CRBA/RNE, box-box / hull / MPR contacts, the constraint solve -- primal Newton, MuJoCo's
default and so the reference's, or --solver pgs -- and semi-implicit Euler), the final position stage,
reward/obs epilogue, TimeLimit + in-kernel auto-reset.  With Newton (the default) the step is ONE fused kernel
launch at every shard size (so100_fused_kernel: every wave runs its 4 envs through all substeps with the state in
registers; waves launched heavy-first by their previous step's cost); with PGS or SO100_FUSED=0 it is 21 launches
per env chunk (per substep a stage kernel and a solver kernel, then the final stage kernel; 4 chunks on
concurrent streams).
Envs are sharded contiguously (global ids drive the seeds); there is no collective on the data path:
only the barrier + max-over-ranks timing reduction around the timed region.
Rank 0 prints ONE JSON line.  See DESIGN.md §6 for the roofline bytes and the CPU baseline.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))

METRIC = "env steps/sec (whole node), 65k parallel bin-a-cube envs at 1/2/4/8 MI355X"
# algorithmic HBM bytes per env step at the boundary.  Reads action 24 + qpos 52 + qvel 48
# + warmstart 48 + step counter 4 = 176; writes qpos 52 + qvel 48 + warmstart 48 + obs 60 + reward 4
# + terminated 1 + truncated 1 + step counter 4 = 218.  GoalEnv +24 (desired goal read, achieved goal
# written), domain randomisation +32 (params read, RNG state).  roofline.achieved = env steps/s per GPU x
# these bytes (never padded with intermediate traffic; the kernels' own record and PMC bytes are reported
# beside it as separate fields).
BYTES_PER_ENV_STEP = {"base": 394, "goal": 418, "dr": 426}
# the split path's stage -> solver HBM record (not algorithmic: an intermediate of the split launches),
# per Newton launch: per env the NewtonHdr (100 floats) read + qacc written, per contact 12 + 48 floats read
NEWTON_RECORD_BYTES_PER_ENV = 4 * 100 + 48
NEWTON_RECORD_BYTES_PER_CONTACT = 4 * (12 + 48)
PGS_RECORD_BYTES_PER_ENV = 640 + 48
PGS_RECORD_BYTES_PER_CONTACT = 160 + 192
HBM_PEAK = 8.0e12            # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
CLOCK_HZ = 2.4e9             # MI355X peak engine clock (valu_busy uses it: a lower real clock only raises the share)
SIMDS = 1024                 # 256 CUs x 4 SIMDs


def shard(total, world, rank):
    """Contiguous env shard [offset, offset+count) of rank (remainder spread over the first ranks)."""
    base, rem = divmod(total, world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--warmup", type=int, default=30)
    p.add_argument("--total-envs", type=int, default=65536)
    p.add_argument("--envs-per-gpu", type=int, default=0, help="weak scaling: fixed envs per GPU")
    p.add_argument("--task", default="so100_cube_to_bin")
    p.add_argument("--action-pool", type=int, default=16)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample duration")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-kernel-timing", action="store_true", help="skip the per-launch HIP events")
    p.add_argument("--contact-steps", type=int, default=10, help="untimed steps sampling contacts/env")
    p.add_argument("--fused-build", type=int, default=0, choices=[0, 2, 3],
                   help="the fused product build: 2 | 3 waves per SIMD, 0 = the library's choice by size")
    p.add_argument("--solver", default="newton", choices=["newton", "pgs"],
                   help="constraint solver: newton (MuJoCo's default, which the reference runs; default) or pgs")
    p.add_argument("--convex", default="epa", choices=["epa", "mpr"],
                   help="mesh-pair collider: epa (GJK + EPA, MuJoCo 3.3.3's default; default) or mpr (libccd)")
    p.add_argument("--dr", action="store_true",
                   help="configs[4]: domain-randomised cube mass / friction scales (0.8-1.2) and action noise (0.05)")
    p.add_argument("--dump-state", default="",
                   help="test hook: each rank saves its shard's final state to <dir>/state_rank<r>.npz")
    return p.parse_args(argv)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, solver="newton"):
    """Time the oracle (the fp64 clarity-first C restatement: dense 12x12 matrices, OpenMP over envs, one
    env per thread) on this host's cores: a reported, non-target baseline.  The reference's MuJoCo is not
    installed here, so it cannot be timed.  Threads: every CPU in this process's affinity set, capped by
    OMP_NUM_THREADS where the pool sets it (the GPU box's CPU share: 16 of its CPUs per GPU)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    from oracle.oracle import Oracle
    from gym_so100.model import build_model
    o = Oracle(64)
    m = build_model(solver=solver)
    allowed = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS") or allowed)
    cores = max(1, min(allowed, cap))
    nenv = 4 * cores
    datas = (o.Data * nenv)()
    for i in range(nenv):
        o.reset(m, datas[i], o.spawn_pose(1000 + i))
    rng = np.random.default_rng(0)
    steps_per_call = 5
    done, t_used = 0, 0.0
    while t_used < seconds:
        acts = rng.uniform(-1, 1, size=(steps_per_call, nenv, 6)).astype(np.float32)
        t0 = time.perf_counter()
        done += o.batch_run(m, datas, nenv, steps_per_call, 0, acts, nthreads=cores)
        t_used += time.perf_counter() - t0
    return {"value": done / t_used, "unit": "env_steps/s", "cores": cores, "kind": "port",
            "cpus_allowed": allowed, "cpu_count": os.cpu_count(), "cpu_model": _cpu_model(),
            "sample": f"{nenv} CubeToBin envs x {done // nenv} steps ({solver} solver, OpenMP {cores} threads, "
                      f"{t_used:.1f}s)",
            "note": "the repo's fp64 oracle (oracle/so100_oracle.c: a clarity-first restatement with dense 12x12 "
                    "matrices), not MuJoCo; a non-target baseline"}


def load_step_traffic(n_envs, mode, solver, lib_hash, kind="base"):
    """The committed rocprofv3 PMC measurement of one env step's HBM traffic at this size and step mode
    (profiles/r<NN>_pmc_step_*.json, the newest round's, tools/gpurun/pmc_step_traffic.py: FETCH_SIZE and WRITE_SIZE
    passes, summed over every kernel of a step) and whether it measured these kernels: the file records the
    so100_source_hash of the library it profiled, and traffic is reported only when that equals the loaded
    library's (a profile of older kernels is named in pmc_source but never quoted as traffic)."""
    tag = "" if kind == "base" else f"{kind}_"
    for rnd in ("r06", "r05", "r04", "r03"):
        path = os.path.join(ROOT, "profiles", f"{rnd}_pmc_step_{tag}{mode}_{solver}_{n_envs}.json")
        if os.path.exists(path):
            try:
                pmc = json.load(open(path))
            except ValueError:
                return None, False
            return pmc, pmc.get("lib_source_hash") == lib_hash
    return None, False


def workload(kind, total, world, count):
    """config.workload: the BASELINE.json config the line measures (configs[2] by default; --task so100_goal is
    configs[3], --dr configs[4]; a 1-GPU run of configs[4] benches one 4-GPU shard with --total-envs 8192)"""
    per = f"{total} envs over {world} GPU(s) ({count} per GPU)"
    if kind == "goal":
        return f"configs[3]: GoalEnv dict-obs (HER) variant, {per}, randomized cube spawn, sparse reward, auto-reset"
    if kind == "dr":
        return (f"configs[4]: domain-randomized cube mass / friction (x0.8-1.2) + action noise (sigma 0.05), {per}, "
                "CubeToBin reward, auto-reset")
    return f"configs[2]: {per} bin-a-cube envs, joint-space ctrl, fp32 state, CubeToBin reward, auto-reset"


def main(argv=None):
    args = parse(argv)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    if world > 1:
        # host-side barrier and MAX over ranks only: the env shards exchange nothing, so RCCL is never
        # initialised (north_star: no RCCL on the data path)
        dist.init_process_group("gloo", init_method="env://")
    # one process per GPU: rank -> device LOCAL_RANK.  SO100_BENCH_DEVICE (test hook only,
    # tests/test_gpu_multirank.py) puts every rank on one device to rehearse the multi-rank path on one GPU.
    device_index = int(os.environ.get("SO100_BENCH_DEVICE", local))
    torch.cuda.set_device(device_index)
    dev = torch.device("cuda", device_index)

    if args.envs_per_gpu > 0:
        count, offset = args.envs_per_gpu, rank * args.envs_per_gpu
        total = count * world
        scaling = "weak"
    else:
        total = args.total_envs
        offset, count = shard(total, world, rank)
        scaling = "strong"

    from gym_so100 import SO100VecEnv
    dr = dict(mass=(0.8, 1.2), friction=(0.8, 1.2), action_noise=0.05) if args.dr else None
    env = SO100VecEnv(count, task=args.task, device=str(dev), seed=args.seed, env_offset=offset, solver=args.solver,
                      convex=args.convex, domain_randomization=dr)
    if args.fused_build:
        env.fused_build = args.fused_build
    env.reset(seed=1000 + offset)   # env i <- RandomState(1000 + global id)
    # the action pool is drawn for all `total` envs from one seed and sliced to this shard, so env i's actions
    # (and its trajectory) do not depend on the number of ranks
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed * 1000003)
    pool = [(torch.rand(total, 6, generator=g, device=dev) * 2 - 1)[offset:offset + count].contiguous()
            for _ in range(args.action_pool)]
    stream = torch.cuda.current_stream(dev)

    for i in range(args.warmup):
        env.set_action_buffer(pool[i % len(pool)])
        env.step_async_raw()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    if not args.no_kernel_timing:
        env.profile_enable(args.steps)      # HIP events on the launch stream around every kernel
    env.pool_stats(reset=True)              # the fused step's contact-record pool counters, from the timed steps on
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for i in range(args.steps):
        env.set_action_buffer(pool[i % len(pool)])
        env.step_async_raw()
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    step_ms = ev[0].elapsed_time(ev[1]) / args.steps        # device time per env step on this stream
    solver_ms = stage_ms = float("nan")
    pool_st = env.pool_stats()
    if not args.no_kernel_timing:
        s_ms, s_n, t_ms, t_n = env.profile_read()
        env.profile_enable(0)
        solver_ms, stage_ms = s_ms / max(s_n, 1), t_ms / max(t_n, 1)
    # untimed: contacts per env per solver launch (the split record bytes) and contacts left out of an env's list
    # (a checked invariant: the list holds every contact since round 4, so this is 0)
    accum = torch.zeros(1, dtype=torch.int64, device=dev)
    dropped = torch.zeros(1, dtype=torch.int64, device=dev)
    for i in range(args.contact_steps):
        env.set_action_buffer(pool[i % len(pool)])
        env.step_async_raw()
        env.contact_count(accum)
        dropped += env.ncon_dropped.sum()
    torch.cuda.synchronize(dev)
    contacts_per_env = float(accum.item()) / max(1, args.contact_steps * count)
    dropped_per_env_step = float(dropped.item()) / max(1, args.contact_steps * count)
    if world > 1:
        t = torch.tensor([elapsed, step_ms, solver_ms, stage_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, step_ms, solver_ms, stage_ms = (float(x) for x in t)

    # sanity: the state stayed finite
    assert torch.isfinite(env.qpos).all().item(), "non-finite state after the benchmark"
    if args.dump_state:
        import numpy as np
        os.makedirs(args.dump_state, exist_ok=True)
        np.savez(os.path.join(args.dump_state, f"state_rank{rank}.npz"), offset=offset, count=count,
                 qpos=env.qpos.cpu().numpy(), qvel=env.qvel.cpu().numpy(), obs=env.obs.cpu().numpy(),
                 reward=env.reward.cpu().numpy(), episode=env.episode.cpu().numpy())

    if rank == 0:
        env_steps = total * args.steps
        value = env_steps / elapsed
        fused = env.fused
        nchunks, n0 = env.chunk_info()
        mode = "fused" if fused else "split"
        kind = "dr" if args.dr else ("goal" if args.task == "so100_goal" else "base")
        bpe = BYTES_PER_ENV_STEP[kind]
        # achieved = env steps/s per GPU x algorithmic bytes per env step.  Per GPU from this
        # rank's device time per step (HIP events on the launch stream around the timed steps: the fused
        # launch, or a split step's 21 launches per chunk with the chunks joined back to this stream)
        per_gpu_rate = count / (step_ms * 1e-3)
        achieved = per_gpu_rate * bpe
        from gym_so100 import _native
        lib_hash = _native.source_hash()
        pmc, pmc_current = load_step_traffic(count, mode, args.solver, lib_hash, kind)
        # per env step, like achieved; null unless the profile measured these kernels (the same source hash)
        traffic = pmc["hbm_bytes_per_step"] / count if (pmc and pmc_current) else None
        if fused:
            rec_per_launch = None
        else:
            per_env, per_con = ((PGS_RECORD_BYTES_PER_ENV, PGS_RECORD_BYTES_PER_CONTACT) if args.solver == "pgs" else
                                (NEWTON_RECORD_BYTES_PER_ENV, NEWTON_RECORD_BYTES_PER_CONTACT))
            rec_per_launch = n0 * (per_env + per_con * contacts_per_env)
        valu_insts = pmc.get("valu_insts_per_step") if (pmc and pmc_current) else None
        valu_busy = valu_insts * 2.0 / (step_ms * 1e-3 * CLOCK_HZ * SIMDS) if valu_insts else None
        line = {
            "metric": METRIC, "value": value, "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": workload(kind, total, world, count),
                       "envs_total": total, "envs_per_gpu": count, "task": args.task, "substeps": 10,
                       "domain_randomization": dr,
                       "solver": args.solver, "solver_iterations": env.model.iterations, "convex": args.convex,
                       "step_mode": mode, "fused_build": env.fused_build if fused else None,
                       "parallelism": f"env-sharded x{world}, no collectives (gloo barrier + MAX for timing)",
                       "actions": "U[-1,1]^6 pool resident in HBM"},
            "roofline": {"bound": "hbm",
                         "limiter": ("latency: each wave's dependent per-env chain (10 substeps of FK -> dynamics -> "
                                     "collision -> rows -> Newton steps); HBM is the roofline priced, not the limiter, "
                                     "valu_busy is the issue share (DESIGN.md §3.5, §8)"),
                         "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK, "traffic": traffic,
                         "bytes_per_env_step": bpe, "env_steps_per_s_per_gpu": per_gpu_rate,
                         "step_device_ms": step_ms,
                         "kernel": "so100_fused_kernel (one launch per env step)" if fused else
                                   f"split step: stage + so100_{args.solver}_kernel x 10 + final stage, {nchunks} chunks",
                         "traffic_over_algorithmic": (traffic / bpe) if traffic else None,
                         "pmc_source": pmc.get("file") if pmc else None,
                         "pmc_source_hash": pmc.get("lib_source_hash") if pmc else None,
                         "lib_source_hash": lib_hash,
                         "pmc_matches_lib": bool(pmc and pmc_current),
                         "valu_busy": valu_busy,
                         "solver_kernel_ms": None if fused else solver_ms,
                         "stage_kernel_ms": None if fused else stage_ms,
                         "fused_kernel_ms": solver_ms if fused else None,
                         "split_record_bytes_per_solver_launch": rec_per_launch, "envs_per_launch": n0,
                         "contacts_per_env": contacts_per_env,
                         "contacts_dropped_per_env_step": dropped_per_env_step,
                         "pool_entries_taken_per_step": pool_st["taken"] / args.steps if fused else None,
                         "pool_requests_none_free": pool_st["none_free"] if fused else None,
                         "pool_entries_per_xcd": pool_st["entries_per_xcd"] if fused else None,
                         "note": ("achieved = env steps/s per GPU x SURVEY §8(d)'s algorithmic bytes per env step "
                                  "(state/action in, state/outputs out; GoalEnv 418, DR 426): nothing else is "
                                  "algorithmic. traffic = measured HBM bytes per env step from rocprofv3 "
                                  "FETCH_SIZE + WRITE_SIZE over every kernel of a step (raw counters, the 16-B/lane x2 "
                                  "correction not applied), so traffic_over_algorithmic shows re-read and spill "
                                  "waste. The path is per-env dependent arithmetic (issue/latency-bound, DESIGN.md "
                                  "§3.5); valu_busy = PMC SQ_INSTS_VALU per step x 2 cyc / (step time x 2.4 GHz x "
                                  "1024 SIMDs)")},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.solver)
            except Exception as e:   # baseline is reported, never required for the GPU number
                line["cpu_baseline"] = {"value": None, "error": str(e)[:200]}
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
