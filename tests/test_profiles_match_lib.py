"""Claims hygiene: the committed PMC step-traffic files the bench line quotes as roofline.traffic were
measured on the library this tree builds.  Each profiles/r06_pmc_step_*.json records the so100_source_hash of the
library its profiled bench.py runs loaded (tools/gpurun/pmc_step_traffic.py); bench.py quotes traffic only on a match,
so a kernel change without a new profile would silently drop traffic from the line.  CPU-only: loads the library and
reads its hash (no compute)."""
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_round6_pmc_files_match_the_built_library():
    from gym_so100 import _native
    h = _native.source_hash()                  # (as test_native_abi: the library must be built; it fails loudly if not)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r06_pmc_step_*.json")))
    assert len(files) >= 7, files              # 4 shard sizes, GoalEnv, DR, PGS
    for f in files:
        assert json.load(open(f))["lib_source_hash"] == h, (os.path.basename(f), h)
