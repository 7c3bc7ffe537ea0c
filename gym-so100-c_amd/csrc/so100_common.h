// so100_common.h — device-side pieces shared by the stage and solver kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "so100_device.h"

namespace so100 {
#define DEV __device__ __forceinline__

// Diagnostic build only (-DSO100_STAMPS): per-wave cycle attribution by phase (s_memtime), written to
// the debug buffer's tail.  The product build compiles these to nothing.
#ifdef SO100_STAMPS
#define STAMP_DECL unsigned long long st_prev_ = 0, st_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define STAMP(slot)                                                                              \
  do {                                                                                           \
    unsigned long long t_;                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                  \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    if ((slot) >= 0) st_acc_[(slot)] += t_ - st_prev_;                                           \
    st_prev_ = t_;                                                                               \
  } while (0)
#else
#define STAMP_DECL
#define STAMP(slot) do {} while (0)
#endif
// an opaque copy: the compiler can neither fold nor hoist what is computed from it (the fused kernel's
// substep loop would otherwise keep loop-invariant results live across it, spilling)
DEV void opaque(float& v) { asm volatile("" : "+v"(v)); }
// a value the compiler cannot see through (so it cannot hoist what derives from it out of a loop): a uniform pointer kept
// scalar (+ an opaque scalar zero), a per-lane value in a VGPR
template <class T> DEV T* launder_s(T* p) {
  int zero;
  asm volatile("s_mov_b32 %0, 0" : "=s"(zero));
  return reinterpret_cast<T*>(reinterpret_cast<char*>(const_cast<void*>(static_cast<const void*>(p))) + zero);
}
DEV int launder_v(int v) { asm volatile("" : "+v"(v)); return v; }
template <class T> DEV T* launder_v(T* p) { asm volatile("" : "+v"(p)); return p; }
constexpr float kMinVal = 1e-15f;
constexpr float kMinImp = 0.0001f;
constexpr float kMaxImp = 0.9999f;

// ------------------------------------------------------------------ cross-lane (16-lane row) primitives
template <int CTRL>
DEV float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// sum over the 16 lanes of this DPP row; result in every lane of the row
DEV float rowsum16(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}
template <int CTRL>
DEV int dppi(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true); }
// one butterfly step of arg_best16: keep the better (score, index) of this lane and its DPP partner, the
// lower index among equal scores; the point (x, y, z) follows its score
template <int CTRL, bool kMin>
DEV void arg_best_step(float& s, int& i, float& x, float& y, float& z) {
  const float os = dpp<CTRL>(s), ox = dpp<CTRL>(x), oy = dpp<CTRL>(y), oz = dpp<CTRL>(z);
  const int oi = dppi<CTRL>(i);
  const bool t = (kMin ? os < s : os > s) || (os == s && oi < i);
  s = t ? os : s; i = t ? oi : i; x = t ? ox : x; y = t ? oy : y; z = t ? oz : z;
}
// the best (max, or min with kMin) score of the 16 lanes of this DPP row, first index among ties, with its
// point, in every lane of the row (the selection is commutative, so all lanes agree bitwise).  The whole
// row must be active.
template <bool kMin>
DEV void arg_best16(float& s, int& i, float& x, float& y, float& z) {
  arg_best_step<0xB1, kMin>(s, i, x, y, z);    // quad_perm [1,0,3,2]
  arg_best_step<0x4E, kMin>(s, i, x, y, z);    // quad_perm [2,3,0,1]
  arg_best_step<0x141, kMin>(s, i, x, y, z);   // row_half_mirror
  arg_best_step<0x140, kMin>(s, i, x, y, z);   // row_mirror
}
// ------------------------------------------------------------------ row broadcast (DPP row_newbcast, gfx90a+)
template <int L>
DEV float bcast_row_c(float v) { return dpp<0x150 + L>(v); }
// j must fold to a constant after unrolling; every lane of each 16-lane row receives lane j of that row
DEV float bcast_row(float v, int j) {
  switch (j) {
    case 0: return bcast_row_c<0>(v);
    case 1: return bcast_row_c<1>(v);
    case 2: return bcast_row_c<2>(v);
    case 3: return bcast_row_c<3>(v);
    case 4: return bcast_row_c<4>(v);
    case 5: return bcast_row_c<5>(v);
    case 6: return bcast_row_c<6>(v);
    case 7: return bcast_row_c<7>(v);
    case 8: return bcast_row_c<8>(v);
    case 9: return bcast_row_c<9>(v);
    case 10: return bcast_row_c<10>(v);
    case 11: return bcast_row_c<11>(v);
    case 12: return bcast_row_c<12>(v);
    case 13: return bcast_row_c<13>(v);
    case 14: return bcast_row_c<14>(v);
    default: return bcast_row_c<15>(v);
  }
}
DEV float4 bcast_row4(float4 v, int j) {
  return make_float4(bcast_row(v.x, j), bcast_row(v.y, j), bcast_row(v.z, j), bcast_row(v.w, j));
}
// ds_bpermute byte address of lane src (0..15) of this lane's 16-lane row.  The lane id comes from an opaque
// v_mbcnt pair at each use: __shfl's own lane id is computed once per kernel and, held across the narrowphase and
// the solve, was a spilled value reloaded inside their loops (3-wave build)
DEV int row_lane() {
  int t;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(t));
  return t & 15;
}
DEV int row_lane_addr(int src) {
  int t;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(t));
  return ((t & ~15) | (src & 15)) << 2;
}
DEV float shfl_at(float v, int addr) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, v)));
}
// max over the wave of a value uniform within each env's 16-lane row (contact and candidate counts); result uniform.
// Four scalar lane reads: no lane id (__shfl_xor's, computed once per kernel and held across the fused substep loop,
// was a spilled value of the 3-wave build reloaded every substep)
DEV int wave_max_row(int v) {
  const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return max(max(a, b), max(c, d));
}
DEV float bcast16(float v, int src) { return __shfl(v, src, kLanes); }
DEV int bcast16i(int v, int src) { return __shfl(v, src, kLanes); }

// MuJoCo mju_QCQP3 restated (engine_util_solve.c): min 0.5 x'Ax + x'b s.t. sum (x_i/d_i)^2 <= r^2.
// The minimiser is y(la) = -(As + la I)^-1 D b for the multiplier la >= 0 that puts y on the sphere
// |y| = r (As = D A D, D = diag(mu0, mu0, mu1)).  In the eigenbasis of As (precomputed per substep,
// with P = Q' D and 1/lam) y_i(la) = c_i / (lam_i + la) with c = -P b, so an iterate costs three
// reciprocals, and x = D Q w = P' w.
// Root finding: MuJoCo's Newton on |y|^2 - r^2 from la = 0 (its 20-step cap included, so an unconverged
// search stops where MuJoCo's does; rounds 1-2 solved the secular equation instead).
// Returns the number of Newton steps taken.
DEV int qcqp3_eig(float* x, const float* P, const float* lam, const float* laminv, const float* b, float r,
                  bool live = true) {
  int nit = 0;
  float c[3], w[3], d[3];
#pragma unroll
  for (int i = 0; i < 3; i++) c[i] = -(P[3 * i] * b[0] + P[3 * i + 1] * b[1] + P[3 * i + 2] * b[2]);   // -P b
#pragma unroll
  for (int i = 0; i < 3; i++) { d[i] = laminv[i]; w[i] = c[i] * d[i]; }
  float s = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  // MuJoCo's iteration (mju_QCQP3; oracle qcqp): Newton on val = |y|^2 - r^2 from la = 0, at most 20 steps,
  // stops val < 1e-10 or delta < 1e-10; after the 20th step y stays at the la it was evaluated at.  In the
  // eigenbasis |y|^2 = sum w_i^2 and y' (A + la I)^-1 y = sum w_i^2 d_i, so delta = -val / deriv = val / 2t.
  if (live && s - r * r >= 1e-10f) {
    float la = 0.f;
    for (int it = 0; it < 20; it++) {
      const float val = s - r * r;
      if (val < 1e-10f) break;
      const float t = w[0] * w[0] * d[0] + w[1] * w[1] * d[1] + w[2] * w[2] * d[2];
      // (hardware reciprocals, 1 ulp, on the iteration's serial chain: one v_rcp each instead of the IEEE division
      // sequence, as the Newton solve's chains since round 3; round 5, PGS)
      const float delta = val * __builtin_amdgcn_rcpf(2.f * t);
      if (delta < 1e-10f) break;
      nit++;
      la += delta;
      if (it == 19) break;
#pragma unroll
      for (int i = 0; i < 3; i++) { d[i] = __builtin_amdgcn_rcpf(lam[i] + la); w[i] = c[i] * d[i]; }
      s = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    }
  }
  // x = D Q w = P' w
#pragma unroll
  for (int j = 0; j < 3; j++) x[j] = P[j] * w[0] + P[3 + j] * w[1] + P[6 + j] * w[2];
  return nit;
}

// ------------------------------------------------------------------ 4-lane (quad) primitives
DEV float quad_swap1(float v) { return dpp<0xB1>(v); }   // quad_perm [1,0,3,2]
DEV float quad_swap2(float v) { return dpp<0x4E>(v); }   // quad_perm [2,3,0,1]
// sum over the 4 lanes of a quad; every lane gets the bitwise-same value (fp add is commutative)
DEV float quadsum(float v) {
  v += quad_swap1(v);
  v += quad_swap2(v);
  return v;
}
template <int L>
DEV float quad_bcast(float v) { return dpp<L | (L << 2) | (L << 4) | (L << 6)>(v); }

}  // namespace so100
