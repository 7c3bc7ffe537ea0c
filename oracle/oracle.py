"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

ORACLE: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
It loads oracle/build/liboracle{64,32}.so (built by oracle/Makefile from so100_oracle.c).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
NBODY, NHINGE, NQ, NV, NU, NGEOM, CONDIM, NOBS = 9, 6, 13, 12, 6, 16, 4, 15
NPAIR = 209                           # include/so100_model.h SO100_NPAIR
NCON_MAX = 62 * 8 + 209 - 62         # include/so100_model.h SO100_NCON_MAX: every pair at its collider's maximum
NEFC = NV + NHINGE + NCON_MAX * CONDIM


def _arr(t, *dims):
    for n in reversed(dims):
        t = t * n
    return t


def _make_types(real):
    class Contact(ctypes.Structure):
        _fields_ = [("pos", _arr(real, 3)), ("frame", _arr(real, 9)), ("dist", real), ("pair", ctypes.c_int)]

    i = ctypes.c_int

    class Data(ctypes.Structure):
        _fields_ = [
            ("qpos", _arr(real, NQ)), ("qvel", _arr(real, NV)), ("qacc_warmstart", _arr(real, NV)),
            ("ctrl", _arr(real, NU)),
            ("xpos", _arr(real, NBODY, 3)), ("xquat", _arr(real, NBODY, 4)), ("xmat", _arr(real, NBODY, 9)),
            ("xipos", _arr(real, NBODY, 3)), ("ximat", _arr(real, NBODY, 9)),
            ("xanchor", _arr(real, NHINGE, 3)), ("xaxis", _arr(real, NHINGE, 3)),
            ("geom_xpos", _arr(real, NGEOM, 3)), ("geom_xmat", _arr(real, NGEOM, 9)),
            ("site_cube", _arr(real, 3)), ("site_ee", _arr(real, 3)),
            ("cinert", _arr(real, NBODY, 13)), ("cdof", _arr(real, NV, 6)),
            ("qM", _arr(real, NV, NV)), ("qL", _arr(real, NV, NV)),
            ("ncon", i), ("ncon_dropped", i), ("con", _arr(Contact, NCON_MAX)),
            ("nefc", i), ("efc_type", _arr(i, NEFC)), ("efc_id", _arr(i, NEFC)), ("efc_dim", _arr(i, NEFC)),
            ("efc_J", _arr(real, NEFC, NV)),
            ("efc_pos", _arr(real, NEFC)), ("efc_margin", _arr(real, NEFC)), ("efc_frictionloss", _arr(real, NEFC)),
            ("efc_diagApprox", _arr(real, NEFC)), ("efc_R", _arr(real, NEFC)), ("efc_D", _arr(real, NEFC)),
            ("efc_K", _arr(real, NEFC)), ("efc_B", _arr(real, NEFC)), ("efc_imp", _arr(real, NEFC)),
            ("efc_mu", _arr(real, NEFC, 3)),
            ("cvel", _arr(real, NBODY, 6)), ("cdof_dot", _arr(real, NV, 6)), ("qfrc_bias", _arr(real, NV)),
            ("efc_vel", _arr(real, NEFC)),
            ("actuator_force", _arr(real, NU)), ("qfrc_actuator", _arr(real, NV)), ("qacc_smooth", _arr(real, NV)),
            ("efc_aref", _arr(real, NEFC)), ("efc_b", _arr(real, NEFC)),
            ("efc_force", _arr(real, NEFC)), ("qacc", _arr(real, NV)),
            ("solver_iter", i), ("solver_improvement", real), ("elapsed_steps", i),
            ("mocap_pos", _arr(real, 3)), ("mocap_quat", _arr(real, 4)),
            ("weld_pos", _arr(real, 6)), ("weld_J", _arr(real, 6, NV)), ("weld_D", _arr(real, 6)),
            ("weld_aref", _arr(real, 6)), ("weld_f", _arr(real, NV)),
            ("snap_ncon", i), ("snap_ndrop", i), ("snap_pair", _arr(i, NCON_MAX)),
            ("snap_force", _arr(real, NCON_MAX, 4)), ("snap_frf", _arr(real, NV)), ("snap_qacc", _arr(real, NV)),
            ("sep_on", i), ("sep_hits", i), ("sep_sep", i), ("sep", _arr(real, NPAIR, 4)),
        ]
    return Contact, Data


def ensure_built():
    libs = [os.path.join(HERE, "build", f"liboracle{b}.so") for b in ("64", "32", "32fma")]
    if not all(os.path.exists(p) for p in libs):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return libs


class Oracle:
    """One precision flavour of the oracle library (bits=64 default, 32 = same code in float)."""

    def __init__(self, bits=64, fma=False, path=None):
        """fma (bits=32 only): the build with multiply-adds contracted to FMAs, as the GPU compiler does; path: another
        build of the same precision (tools/dev experiments)"""
        ensure_built()
        self.bits = bits
        self.real = ctypes.c_double if bits == 64 else ctypes.c_float
        self.np_real = np.float64 if bits == 64 else np.float32
        self.lib = ctypes.CDLL(path or os.path.join(HERE, "build", f"liboracle{bits}{'fma' if fma else ''}.so"))
        self.Contact, self.Data = _make_types(self.real)
        L = self.lib
        P = ctypes.c_void_p
        L.so100o_sizeof_data.restype = ctypes.c_int
        assert L.so100o_sizeof_data() == ctypes.sizeof(self.Data), (L.so100o_sizeof_data(), ctypes.sizeof(self.Data))
        L.so100o_sizeof_model.restype = ctypes.c_int
        L.so100o_unnormalize.argtypes = [P, P, P]
        L.so100o_spawn_pose.argtypes = [ctypes.c_uint32, P]
        L.so100o_reward.argtypes = [P, ctypes.c_int, P, P, P, ctypes.c_uint32]
        L.so100o_reward.restype = ctypes.c_double
        for fn in ("so100o_fwd_position", "so100o_fwd_velocity", "so100o_fwd_acceleration", "so100o_euler",
                   "so100o_substep"):
            getattr(L, fn).argtypes = [P, P]
        L.so100o_reset.argtypes = [P, P, P]
        L.so100o_contact_bits.argtypes = [P]
        L.so100o_contact_bits.restype = ctypes.c_uint32
        L.so100o_env_step.argtypes = [P, P, ctypes.c_int, P, P, P]
        L.so100o_env_step.restype = ctypes.c_double
        L.so100o_observe.argtypes = [P, P, P]
        L.so100o_batch_run.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
        L.so100o_batch_run.restype = ctypes.c_long
        L.so100o_box_box.argtypes = [P, P, P, P, P, P, self.real, P]
        L.so100o_box_box.restype = ctypes.c_int

    # --- helpers -------------------------------------------------------------------------
    @staticmethod
    def _p(x):
        return ctypes.cast(ctypes.pointer(x), ctypes.c_void_p) if not isinstance(x, np.ndarray) else \
            ctypes.c_void_p(x.ctypes.data)

    def new_data(self):
        return self.Data()

    def unnormalize(self, model, action):
        a = np.ascontiguousarray(action, dtype=np.float32)
        c = np.zeros(6, np.float32)
        self.lib.so100o_unnormalize(self._p(model), self._p(a), self._p(c))
        return c

    def spawn_pose(self, seed):
        out = np.zeros(7)
        self.lib.so100o_spawn_pose(ctypes.c_uint32(int(seed)), self._p(out))
        return out

    def reward(self, model, task, cube_f32, cube, ee, bits):
        cf = np.ascontiguousarray(cube_f32, np.float32)
        c = np.ascontiguousarray(cube, np.float64)
        e = np.ascontiguousarray(ee, np.float64)
        return self.lib.so100o_reward(self._p(model), int(task), self._p(cf), self._p(c), self._p(e), int(bits))

    def reset(self, model, d, box_pose):
        bp = np.ascontiguousarray(box_pose, np.float64)
        self.lib.so100o_reset(self._p(model), self._p(d), self._p(bp))

    def env_step(self, model, d, task, action):
        a = np.ascontiguousarray(action, np.float32)
        obs = np.zeros(NOBS, np.float32)
        term = ctypes.c_int(0)
        r = self.lib.so100o_env_step(self._p(model), self._p(d), int(task), self._p(a), self._p(obs),
                                     ctypes.cast(ctypes.pointer(term), ctypes.c_void_p))
        return obs, r, bool(term.value)

    def call(self, fn, model, d):
        getattr(self.lib, fn)(self._p(model), self._p(d))

    def contact_bits(self, d):
        return int(self.lib.so100o_contact_bits(self._p(d)))

    def observe(self, model, d):
        obs = np.zeros(NOBS, np.float32)
        self.lib.so100o_observe(self._p(model), self._p(d), self._p(obs))
        return obs

    def batch_run(self, model, datas, nenv, steps, task, actions, nthreads=0):
        a = np.ascontiguousarray(actions, np.float32)
        assert a.shape == (steps, nenv, 6)
        return self.lib.so100o_batch_run(self._p(model), ctypes.c_void_p(ctypes.addressof(datas)), nenv, steps,
                                         int(task), self._p(a), int(nthreads))

    def last_solve(self, d):
        """so100o_env_step's record of its last substep's solve: (pairs [ncon], forces [ncon, 4] (normal,
        friction rows), dof frictionloss forces [12], qacc [12], contacts dropped over the step)."""
        n = d.snap_ncon
        return (np.array(d.snap_pair[:n], np.int64), np.array([d.snap_force[c][:] for c in range(n)], np.float64).reshape(n, 4),
                np.array(d.snap_frf[:], np.float64), np.array(d.snap_qacc[:], np.float64), int(d.snap_ndrop))

    # state <-> numpy
    def get_state(self, d):
        return (np.array(d.qpos[:], np.float64), np.array(d.qvel[:], np.float64),
                np.array(d.qacc_warmstart[:], np.float64), np.array(d.ctrl[:], np.float64))

    def set_state(self, d, qpos, qvel, warm, ctrl=None):
        for k in range(NQ):
            d.qpos[k] = float(qpos[k])
        for k in range(NV):
            d.qvel[k] = float(qvel[k])
            d.qacc_warmstart[k] = float(warm[k])
        if ctrl is not None:
            for k in range(NU):
                d.ctrl[k] = float(ctrl[k])
