"""Copy the round-2 measurement set (tools/gpurun/_gpu_round2.sh -> gpurun_out/r02) into profiles/r02_*."""
import json, os, shutil, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
S, P = os.path.join(ROOT, "gpurun_out", "r02"), os.path.join(ROOT, "profiles")
cp = {"bench.json": "r02_bench.json", "bench_pgs.json": "r02_bench_pgs.json", "smoke.log": "r02_smoke.log",
      "pytest_gpu.log": "r02_pytest_gpu.log", "lscpu.txt": "r02_gpu_host_lscpu.txt",
      "pmc_report_split.txt": "r02_pmc_report_split.txt", "pmc_report_fused.txt": "r02_pmc_report_fused.txt",
      "trace_report.txt": "r02_trace_report.txt", "pmc_traffic_newton.json": "pmc_traffic_newton.json",
      "pmc_traffic_fused.json": "pmc_traffic_fused.json", "trace/bench_kernel_stats.csv": "r02_kernel_stats.csv",
      "trace_fused/fused8192_kernel_stats.csv": "r02_kernel_stats_fused8192.csv",
      "trace_pgs/bench_pgs_kernel_stats.csv": "r02_kernel_stats_pgs.csv"}
for a, b in cp.items():
    shutil.copy(os.path.join(S, a), os.path.join(P, b))
lines = ["# round 2: env steps/s per GPU at the per-GPU shard sizes of the 1/2/4/8-GPU strong-scaling runs (65,536 envs total),",
         "# 1 MI355X, bench.py --total-envs N --steps 200 --warmup 20, both step modes on the same box (tools/gpurun/_gpu_round2.sh).",
         "# auto mode (the default) takes the fused step up to 49,152 envs per GPU.",
         "# envs  fused_env_steps/s  fused_ms/step  split_env_steps/s  split_ms/step  auto"]
per = {}
for n in (65536, 32768, 16384, 8192):
    f, s = (json.load(open(os.path.join(S, f"shard_f{k}_{n}.json"))) for k in (1, 0))
    per[n] = f["value"] if n <= 49152 else s["value"]
    lines.append(f"{n} {f['value']:.0f} {f['ms_per_step']:.3f} {s['value']:.0f} {s['ms_per_step']:.3f} "
                 f"{'fused' if n <= 49152 else 'split'}")
lines.append(f"# projected 8-GPU node (8 x the 8,192-env shard, no collectives): {8 * per[8192] / 1e6:.1f} M env steps/s")
open(os.path.join(P, "r02_shard_sizes.txt"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
