"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer (the CPU restatement under
ASan/UBSan).  `make -C oracle asan` links so100_oracle.c into an instrumented driver (oracle/asan_driver.c);
this runs it over contact-rich states (folded arm poses, cubes in a bin corner and on the Base, random
actions, all three reward tasks, the batched OpenMP entry point) for both solvers, both model variants and
both precisions.  Any sanitizer finding aborts the driver (-fno-sanitize-recover=all)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.fixture(scope="module")
def asan_bins():
    r = subprocess.run(["make", "-s", "-C", ORACLE, "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("make -C oracle asan failed:\n" + r.stderr[-2000:])
    return {b: os.path.join(ORACLE, "build", f"oracle_asan_{b}") for b in (64, 32)}


@pytest.mark.parametrize("solver", ["newton", "pgs"])
@pytest.mark.parametrize("variant", ["joint", "ee"])
@pytest.mark.parametrize("bits", [64, 32])
def test_oracle_clean_under_asan_ubsan(asan_bins, tmp_path, solver, variant, bits):
    from gym_so100.model import build_model
    m = build_model(solver=solver, variant=variant)
    path = tmp_path / "model.bin"
    path.write_bytes(bytes(m))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24")
    r = subprocess.run([asan_bins[bits], str(path), "48", "20"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-1000:] + r.stderr[-4000:]
    assert r.stdout.startswith("ok:") and "ERROR" not in r.stderr and "runtime error" not in r.stderr
    contacts = int(r.stdout.split("contacts ")[1].split()[0])
    assert contacts > 48 * 20              # contact-rich: more than one contact per env step on average
