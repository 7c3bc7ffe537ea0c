"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/so100.h declares, its
struct layouts match the ctypes mirrors, and it fails loudly (no fallback) without a device."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "so100.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(so100_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from gym_so100 import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_native.EXPORTED_SYMBOLS)


def test_struct_layouts_match():
    from gym_so100 import _native
    from gym_so100.model import SO100Model
    lib = _native.load()      # load() itself raises on a layout mismatch
    mb, bb = ctypes.c_int(), ctypes.c_int()
    lib.so100_struct_sizes(ctypes.byref(mb), ctypes.byref(bb))
    assert mb.value == ctypes.sizeof(SO100Model)
    assert bb.value == ctypes.sizeof(_native.SO100Buffers)


def test_oracle_model_layout_matches(oracle64):
    from gym_so100.model import SO100Model
    assert oracle64.lib.so100o_sizeof_model() == ctypes.sizeof(SO100Model)


def test_create_validates_and_fails_loudly_without_device(model):
    import torch
    from gym_so100 import _native
    lib = _native.load()
    assert lib.so100_create(None, 4, 0) is None
    assert b"model is NULL" in lib.so100_last_error()
    assert lib.so100_create(ctypes.byref(model), 0, 0) is None
    if not torch.cuda.is_available():
        assert lib.so100_create(ctypes.byref(model), 4, 0) is None
        assert b"no HIP device" in lib.so100_last_error()


def test_model_structure_check_rejects_bad_model(model):
    import copy
    from gym_so100 import _native
    lib = _native.load()
    bad = copy.deepcopy(model)
    bad.pair_condim[0] = 3
    assert lib.so100_create(ctypes.byref(bad), 4, 0) is None
    err = lib.so100_last_error()
    assert b"condim" in err or b"no HIP device" in err


def test_vec_env_requires_native_library(monkeypatch):
    from gym_so100 import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/libso100_hip.so")
    from gym_so100 import SO100VecEnv
    with pytest.raises(_native.NativeLibraryError):
        SO100VecEnv(4)


def test_product_never_imports_the_oracle():
    pat = re.compile(r"^\s*(from\s+oracle|import\s+oracle|#\s*include\s*[<\"].*oracle)|liboracle|so100o_", re.M)
    pkg = os.path.join(ROOT, "gym-so100-c_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h", "Makefile")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not pat.search(txt), os.path.join(dirpath, f)


def test_sb3_adapter_interface():
    """The SB3 adapter exposes SB3's VecEnv surface (constructed only on a GPU: test_gpu_sb3.py)."""
    from gym_so100.sb3 import SO100SB3VecEnv
    for name in ("reset", "step_async", "step_wait", "step", "close", "seed", "get_attr", "set_attr",
                 "env_method", "env_is_wrapped", "get_images"):
        assert callable(getattr(SO100SB3VecEnv, name)), name


@pytest.mark.parametrize("case", ["solimp_power", "marker_pair", "marker_off_centre"])
def test_model_check_rejects_what_the_kernels_do_not_handle(model, case):
    """so100_create's model check (before any device call) rejects a solimp power other than 1 or 2 (the kernels'
    impedance has no general powf path), a marker pair that is not (marker, hull k), and a marker box off its
    body's origin (the kernels take its pose as the mocap pose)."""
    import copy
    from gym_so100 import _native
    from gym_so100.model import MOCAP_GEOM, PAIR_MOCAPHULL0
    lib = _native.load()
    bad = copy.deepcopy(model)
    if case == "solimp_power":
        bad.pair_solimp[5][4] = 3.0
        want = b"solimp power"
    elif case == "marker_pair":
        bad.pair_geom2[PAIR_MOCAPHULL0 + 2] = -1
        want = b"marker, hull k"
    else:
        bad.geom_pos[MOCAP_GEOM][0] = 0.01
        want = b"centred"
    assert lib.so100_create(ctypes.byref(bad), 4, 0) is None
    assert want in lib.so100_last_error()
