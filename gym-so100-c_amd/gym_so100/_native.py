"""ctypes binding of libso100_hip.so (include/so100.h).

The HIP library is the only compute path: if it cannot be loaded, every env constructor raises.
There is no CPU fallback in the product.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SO100_LIB") or os.path.join(HERE, "_lib", "libso100_hip.so")

SO100_FLAG_AUTORESET = 1
SO100_FLAG_DR = 2
SO100_DBG_OVF = 160                   # include/so100.h: the debug entries of contacts >= 16
SO100_DBG_STRIDE = 160 + 6 * (643 - 16)
TASKS = {"so100_cube_to_bin": 0, "so100_touch_cube": 1, "so100_touch_cube_sparse": 2, "so100_goal": 3}

_P = ctypes.c_void_p


class SO100Buffers(ctypes.Structure):
    """Mirror of ``so100_buffers`` (include/so100.h): device pointers, NULL = not requested."""
    _fields_ = [(n, _P) for n in (
        "qpos", "qvel", "qacc_warmstart", "elapsed", "episode", "action",
        "obs", "reward", "terminated", "truncated", "success", "final_obs", "diverged", "contact_bits",
        "achieved_goal", "desired_goal", "total_steps", "dr_params", "debug", "mocap", "reward64", "ncon_dropped",
        "ep_return", "ep_final", "ep_accum")]


SO100_MAX_LIGHTS = 4


class SO100Camera(ctypes.Structure):
    """Mirror of ``so100_camera`` (include/so100.h): pose, fovy, headlight and directional lights."""
    _fields_ = [("pos", ctypes.c_float * 3), ("mat", ctypes.c_float * 9), ("track", ctypes.c_int),
                ("fovy", ctypes.c_float),
                ("znear", ctypes.c_float), ("head_ambient", ctypes.c_float), ("head_diffuse", ctypes.c_float),
                ("nlight", ctypes.c_int), ("light_dir", (ctypes.c_float * 3) * SO100_MAX_LIGHTS),
                ("light_diffuse", ctypes.c_float * SO100_MAX_LIGHTS)]


class NativeLibraryError(RuntimeError):
    pass


_lib = None


ABI_VERSION = 17         # include/so100.h SO100_ABI_VERSION
HULL_CELLG = 8           # SO100_HULL_CELLG
HULL_NCELL = 6 * HULL_CELLG * HULL_CELLG


def load():
    """Load libso100_hip.so once; raise NativeLibraryError loudly if it is missing or broken."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `make -C gym-so100-c_amd/csrc` (or __graft_entry__.build()). "
            "The HIP kernels are the only compute path; there is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    lib.so100_abi_version.restype = ctypes.c_int
    lib.so100_last_error.restype = ctypes.c_char_p
    lib.so100_source_hash.restype = ctypes.c_char_p
    lib.so100_create.argtypes = [_P, ctypes.c_int, ctypes.c_int]
    lib.so100_create.restype = _P
    lib.so100_destroy.argtypes = [_P]
    lib.so100_num_envs.argtypes = [_P]
    lib.so100_configure.argtypes = [_P, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
    lib.so100_reset.argtypes = [_P, ctypes.POINTER(SO100Buffers), _P, _P, _P]
    lib.so100_step.argtypes = [_P, ctypes.POINTER(SO100Buffers), ctypes.c_int, _P]
    lib.so100_goal_reward.argtypes = [_P, ctypes.c_int, _P, _P, _P, _P]
    lib.so100_eval_reward.argtypes = [_P, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, _P]
    lib.so100_spawn_pose.argtypes = [_P, ctypes.c_int, _P, _P, _P]
    lib.so100_unnormalize.argtypes = [_P, ctypes.c_int, _P, _P, _P]
    lib.so100_profile_enable.argtypes = [_P, ctypes.c_int]
    lib.so100_profile_read.argtypes = [_P, _P, _P, _P, _P]
    lib.so100_contact_count.argtypes = [_P, _P, _P]
    lib.so100_contact_counts.argtypes = [_P, _P, _P]
    lib.so100_pool_stats.argtypes = [_P, _P, ctypes.c_int]
    lib.so100_chunk_info.argtypes = [_P, _P, _P]
    lib.so100_set_step_mode.argtypes = [_P, ctypes.c_int]
    lib.so100_step_mode.argtypes = [_P]
    lib.so100_render_mesh.argtypes = [_P, _P, _P, _P, ctypes.c_int]
    lib.so100_render.argtypes = [_P, _P, _P, ctypes.POINTER(SO100Camera), ctypes.c_int, ctypes.c_int, _P, _P]
    lib.so100_hull_cells.argtypes = [_P, _P, _P, ctypes.c_int]
    lib.so100_set_fused_build.argtypes = [_P, ctypes.c_int]
    lib.so100_fused_build.argtypes = [_P, ctypes.c_int]
    for fn in ("so100_destroy", "so100_num_envs", "so100_configure", "so100_reset", "so100_step",
               "so100_goal_reward", "so100_eval_reward", "so100_spawn_pose", "so100_unnormalize",
               "so100_profile_enable", "so100_profile_read", "so100_contact_count", "so100_contact_counts",
               "so100_pool_stats", "so100_chunk_info", "so100_render_mesh", "so100_render", "so100_set_step_mode", "so100_step_mode", "so100_hull_cells",
               "so100_set_fused_build", "so100_fused_build"):
        getattr(lib, fn).restype = ctypes.c_int
    lib.so100_struct_sizes.argtypes = [_P, _P]
    lib.so100_struct_sizes.restype = ctypes.c_int
    if lib.so100_abi_version() != ABI_VERSION:
        raise NativeLibraryError("libso100_hip.so ABI mismatch")
    mb, bb = ctypes.c_int(0), ctypes.c_int(0)
    lib.so100_struct_sizes(ctypes.byref(mb), ctypes.byref(bb))
    from .model import SO100Model
    if mb.value != ctypes.sizeof(SO100Model) or bb.value != ctypes.sizeof(SO100Buffers):
        raise NativeLibraryError(f"struct layout mismatch: so100_model {mb.value} vs {ctypes.sizeof(SO100Model)}, "
                                 f"so100_buffers {bb.value} vs {ctypes.sizeof(SO100Buffers)}")
    _lib = lib
    return lib


EXPORTED_SYMBOLS = ("so100_abi_version", "so100_last_error", "so100_source_hash", "so100_struct_sizes", "so100_create", "so100_destroy", "so100_num_envs",
                    "so100_configure", "so100_reset", "so100_step", "so100_goal_reward", "so100_eval_reward",
                    "so100_spawn_pose", "so100_unnormalize", "so100_profile_enable", "so100_profile_read",
                    "so100_contact_count", "so100_contact_counts", "so100_pool_stats", "so100_chunk_info", "so100_render_mesh",
                    "so100_render",
                    "so100_set_step_mode", "so100_step_mode", "so100_hull_cells", "so100_set_fused_build",
                    "so100_fused_build")


def source_hash():
    """The content hash of the sources the loaded library was built from (so100_source_hash)."""
    return load().so100_source_hash().decode()


def check(rc, what):
    if rc != 0:
        msg = load().so100_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Device pointer of a torch tensor (or None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(torch_mod, device):
    s = torch_mod.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)
