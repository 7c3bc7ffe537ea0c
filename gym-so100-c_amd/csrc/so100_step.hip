// so100_step.hip — MI355X (gfx950) batched SO-ARM100 bin-a-cube simulator: the hot path.
//
// Replaces, for N envs per launch, gym_so100/env.py:172-182 SO100Env.step ->
// single_arm.py:33-38 before_step -> dm_control Physics.step(10) (MuJoCo mj_step x10 + mj_step1)
// -> single_arm.py get_reward / get_observation -> env.py:130-146 packing.
//
// Execution model:
//   * one wave64 workgroup = 4 envs; each env owns a 16-lane "lane group" = one DPP row.
//   * lane k of a group owns dof k (k < 12) for the solver, contact-pair k (k < 14) for collision,
//     contact k for per-contact constraint setup; small serial work (kinematic chain, 6x6 CRBA/RNE)
//     runs on lane 0 of the group with results staged in LDS.
//   * per-env state lives in registers for the whole env step (10 substeps) — HBM is touched once
//     to load the state/action and once to store state/outputs.
//   * the constraint solve is projected Gauss-Seidel (MuJoCo mj_solPGS semantics) with
//     J·qacc dot products reduced across the 16-lane row by DPP (quad_perm, row_half_mirror,
//     row_mirror): 4 VALU ops per reduction, no LDS round trip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "so100_device.h"
#include "so100.h"
#include "so100_common.h"
#include "so100_kin.h"
#include "so100_newton.h"

// hull supports through the direction cells in the split path's stage kernel too (the fused kernel always)
#ifndef SO100_SPLIT_CELLS
#define SO100_SPLIT_CELLS 0
#endif
namespace so100 {

DEV void cross_motion(float* r, const float* v, const float* u) {
  float a[3], b[3], c[3];
  cross3(a, v, u); cross3(b, v, u + 3); cross3(c, v + 3, u);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
DEV void cross_force(float* r, const float* v, const float* f) {
  float a[3], b[3], c[3];
  cross3(a, v, f); cross3(b, v + 3, f + 3); cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
// spatial inertia in[13] = I(9) about the reference point, m*d (3), m
DEV void mul_inert(float* r, const float* in, const float* v) {
  float Iw[3], mdv[3], mdw[3];
  mulmv3(Iw, in, v);
  cross3(mdv, in + 9, v + 3);
  cross3(mdw, in + 9, v);
#pragma unroll
  for (int k = 0; k < 3; k++) { r[k] = Iw[k] + mdv[k]; r[3 + k] = in[12] * v[3 + k] - mdw[k]; }
}

// ------------------------------------------------------------------ impedance / reference (MuJoCo restated)
DEV float getimpedance(const float* solimp, float pos, float margin) {
  float dmin = fminf(fmaxf(solimp[0], kMinImp), kMaxImp);
  float dmax = fminf(fmaxf(solimp[1], kMinImp), kMaxImp);
  float width = solimp[2];
  float mid = fminf(fmaxf(solimp[3], kMinImp), kMaxImp);
  float power = fmaxf(solimp[4], 1.0f);
  if (dmin == dmax || width <= kMinVal) return 0.5f * (dmin + dmax);
  float x = fabsf((pos - margin) * __builtin_amdgcn_rcpf(width));
  if (x >= 1.0f) return dmax;
  if (x <= 0.0f) return dmin;
  float y;
  if (power == 1.0f) y = x;
  else if (power == 2.0f) y = x <= mid ? x * x * __builtin_amdgcn_rcpf(mid)          // the model's solimp power
                                       : 1.0f - (1.0f - x) * (1.0f - x) * __builtin_amdgcn_rcpf(1.0f - mid);
  else if (x <= mid) y = powf(x, power) / powf(mid, power - 1.0f);
  else y = 1.0f - powf(1.0f - x, power) / powf(1.0f - mid, power - 1.0f);
  return dmin + y * (dmax - dmin);
}

// ------------------------------------------------------------------ task prologue / epilogue
// constants.py:44-47,78-86 applied to a float32 copy (single_arm.py:33-38): float32 ops, no FMA.
// span = fp32(max_val - min_val) with the subtraction in double (python floats), as numpy does.
DEV float unnormalize_f32(float a, float lo, float hi, float span) {
#pragma clang fp contract(off)
  float t = a + 1.0f;
  float u = t / 2.0f;
  float v = u * span;
  float w = v + lo;
  w = w < lo ? lo : w;
  return w > hi ? hi : w;
}

// reward ladders — single_arm.py:322-380 / :149-215 / :246-285 (double, exactly as the reference)
DEV double task_reward(const DevModel* __restrict__ m, int task, const float* cube_f, const float* ee_f,
                       uint32_t bits) {
#pragma clang fp contract(off)
  double bmin[3], bmax[3];
  const double hw = m->bin_hw, h = m->bin_h;
  bmin[0] = m->bin_center[0] + -hw; bmin[1] = m->bin_center[1] + -hw; bmin[2] = m->bin_center[2] + 0.0;
  bmax[0] = m->bin_center[0] + hw;  bmax[1] = m->bin_center[1] + hw;  bmax[2] = m->bin_center[2] + h;
  const bool touch_gripper = (bits & ((1u << SO100_NPAIR_GRIPPER) - 1u)) != 0u;
  const bool touch_table = ((bits >> SO100_PAIR_TABLE) & 1u) != 0u;
  if (task == SO100_TASK_CUBE_TO_BIN || task == SO100_TASK_GOAL) {
    double c[3] = {(double)cube_f[0], (double)cube_f[1], (double)cube_f[2]};
    bool over = (bmin[0] < c[0] && c[0] < bmax[0]) && (bmin[1] < c[1] && c[1] < bmax[1]);
    bool inside = true;
    const float half = (float)m->cube_half;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      float lower = cube_f[k] - half, upper = cube_f[k] + half;
      inside = inside && ((double)lower > bmin[k]) && ((double)upper < bmax[k]);
    }
    bool released = inside && !touch_gripper;
    double r = 0.0;
    if (touch_gripper) r = 1.0;
    if (touch_gripper && !touch_table) r = 2.0;
    if (over) r = 2.5;
    if (inside) r = 3.0;
    if (released) r = 4.0;
    return r;
  }
  double dx = (double)ee_f[0] - (double)cube_f[0], dy = (double)ee_f[1] - (double)cube_f[1];
  double dz = (double)ee_f[2] - (double)cube_f[2];
  double dist = sqrt(dx * dx + dy * dy + dz * dz);
  bool success = touch_gripper && dist < 0.05;
  if (task == SO100_TASK_TOUCH_CUBE_SPARSE) return success ? m->max_reward : -0.2;
  double r = 0.0;
  if (dist < 0.7) r = fmax(r, 0.1 * (1.0 - dist / 0.7));
  if (dist < 0.5) r = fmax(r, 0.2 * (1.0 - dist / 0.5));
  if (dist < 0.3) r = fmax(r, 0.5 * (1.0 - dist / 0.3));
  if (dist < 0.1) r = fmax(r, 1.0 * (1.0 - dist / 0.1));
  if (dist < 0.05) r = fmax(r, 2.0 * (1.0 - dist / 0.05));
  if (touch_gripper) r += 1.0;
  if (success) return m->max_reward;
  return r - 0.2;
}

// ------------------------------------------------------------------ RNG: numpy legacy MT19937 spawn
// RandomState(seed).uniform(lo, hi) for 3 components (utils.py:18-29): init_genrand, one twist of the
// first 6 words (needs mt[0..6] and mt[397..402]), tempering, 53-bit doubles.
DEV uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
DEV void spawn_pose(const DevModel* __restrict__ m, uint32_t seed, double* pose) {
#pragma clang fp contract(off)
  uint32_t lo[7], hi[6];
  uint32_t s = seed;
  lo[0] = s;
#pragma unroll
  for (int i = 1; i < 7; i++) { s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i; lo[i] = s; }
  for (int i = 7; i < 397; i++) s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
#pragma unroll
  for (int i = 397; i < 403; i++) { s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i; hi[i - 397] = s; }
  uint32_t out[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    uint32_t y = (lo[i] & 0x80000000u) | (lo[i + 1] & 0x7fffffffu);
    uint32_t v = hi[i] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    out[i] = mt_temper(v);
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    uint32_t a = out[2 * k] >> 5, b = out[2 * k + 1] >> 6;
    // no contraction: numpy evaluates (a*2^26 + b) / 2^53 and low + (high-low)*u with rounded ops
    double u = ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
    double range = m->spawn_hi[k] - m->spawn_lo[k];
    double scaled = range * u;
    pose[k] = m->spawn_lo[k] + scaled;
  }
  pose[3] = 1.0; pose[4] = 0.0; pose[5] = 0.0; pose[6] = 0.0;
}
DEV uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
DEV uint32_t episode_seed(uint64_t base, uint32_t env, uint32_t episode) {
  return (uint32_t)splitmix64(base ^ splitmix64(((uint64_t)env << 32) | episode));
}
DEV float hash_uniform(uint64_t key) { return (float)(splitmix64(key) >> 40) * (1.0f / 16777216.0f); }
DEV float hash_normal(uint64_t key) {
  float u1 = fmaxf(hash_uniform(key), 1e-7f), u2 = hash_uniform(key ^ 0xA5A5A5A5A5A5A5A5ull);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// Diagnostic builds only: SSTAMP_RAW accumulates the shader cycles since the last stamp into slot (-1: none).
// With -DSO100_DYN_STAMPS the stage stamps cover the position / dynamics stage's phases instead (DSTAMP,
// slots 0..7: sincos, FK, comPos, CRBA, Cholesky, M^-1 + RNE velocities, RNE forces, bias + qacc_smooth).
#ifdef SO100_STAGE_STAMPS
#define SSTAMP_RAW(slot)                                                                         \
  do {                                                                                           \
    unsigned long long t_;                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                  \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    if ((slot) >= 0) sst_acc_[(slot) & 7] += t_ - sst_prev_;                                     \
    sst_prev_ = t_;                                                                              \
  } while (0)
#endif
#if defined(SO100_STAGE_STAMPS) && defined(SO100_DYN_STAMPS)
#define DSTAMP_PARAMS , unsigned long long &sst_prev_, unsigned long long *sst_acc_
#define DSTAMP_ARGS , sst_prev_, sst_acc_
#define DSTAMP(slot) SSTAMP_RAW(slot)
#else
#define DSTAMP_PARAMS
#define DSTAMP_ARGS
#define DSTAMP(slot) do {} while (0)
#endif

// Lane-parallel dynamics stage (all 16 lanes of the env's row; lanes 0..5 = bodies/dofs of the arm):
// comPos, CRBA, Cholesky (lane 0) + M^-1 columns, RNE and actuation, with every sum in the serial
// order of the lane-0 version (prefix sums of cvel/cacc, suffix sums of crb/bias) so results are the
// same bit-for-bit.  Requires fk_stage first and a barrier.
// ------------------------------------------------------------------ EE / mocap variant: weld equality
// MuJoCo's mju_mat2Quat with the sign w >= 0 (oracle mat2quat_pos)
DEV void mat2quat_pos(float* q, const float* r) {
  const float tr = r[0] + r[4] + r[8];
  if (tr > 0.f) {
    q[0] = 0.5f * sqrtf(tr + 1.f);
    const float i4 = 1.f / (4.f * q[0]);
    q[1] = (r[7] - r[5]) * i4; q[2] = (r[2] - r[6]) * i4; q[3] = (r[3] - r[1]) * i4;
  } else if (r[0] > r[4] && r[0] > r[8]) {
    q[1] = 0.5f * sqrtf(1.f + r[0] - r[4] - r[8]);
    const float i4 = 1.f / (4.f * q[1]);
    q[0] = (r[7] - r[5]) * i4; q[2] = (r[1] + r[3]) * i4; q[3] = (r[2] + r[6]) * i4;
  } else if (r[4] > r[8]) {
    q[2] = 0.5f * sqrtf(1.f - r[0] + r[4] - r[8]);
    const float i4 = 1.f / (4.f * q[2]);
    q[0] = (r[2] - r[6]) * i4; q[1] = (r[1] + r[3]) * i4; q[3] = (r[5] + r[7]) * i4;
  } else {
    q[3] = 0.5f * sqrtf(1.f - r[0] - r[4] + r[8]);
    const float i4 = 1.f / (4.f * q[3]);
    q[0] = (r[3] - r[1]) * i4; q[1] = (r[2] + r[6]) * i4; q[2] = (r[5] + r[7]) * i4;
  }
  quat_normalize(q);
  if (q[0] < 0.f) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
}

// [3P] mj_makeEquality mjEQ_WELD for so_arm100_ee.xml:171-173 (site1 on the mocap body, site2 = ee_site on
// Fixed_Jaw), restated as oracle weld_fold: 6 always-active quadratic rows, eliminated exactly into the arm
// block of M (M += J'DJ) and the joint force (J'D aref, added to tau at the end of dynamics_par; DESIGN.md
// §4 deviation 10).  Called between the CRBA and the Cholesky; scratch: S.X (J rows, dead until the
// M^-1 columns), S.F (dead after the CRBA).  Uniform per block (m->ee), so its barriers are safe.
DEV void weld_fold(const DevModel* __restrict__ m, EnvShared& sh, int lane) {
  SerialScratch& S = sh.ser;
  float (*J)[8] = S.X;                       // J[row][dof 0..5]
  // F[0][0..5] residual, F[1][0..3] e, F[2][0..7] + F[3][0] R2, F[3][4..6] p2, F[4] D, F[5] D aref
  if (lane == 0) {
    float R2[9], p2[3], t[3], q1[4], R1[9], Rr[9], e[4];
    mulmm3(R2, S.xm[4], m->weld_mat2);
    mulmv3(t, S.xm[4], m->weld_pos2);
#pragma unroll
    for (int k = 0; k < 3; k++) p2[k] = S.xp[4][k] + t[k];
#pragma unroll
    for (int k = 0; k < 4; k++) q1[k] = sh.mocap[3 + k];
    quat_normalize(q1);
    quat2mat(R1, q1);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) Rr[3 * i + j] = R2[i] * R1[j] + R2[3 + i] * R1[3 + j] + R2[6 + i] * R1[6 + j];
    mat2quat_pos(e, Rr);
#pragma unroll
    for (int k = 0; k < 3; k++) { S.F[0][k] = sh.mocap[k] - p2[k]; S.F[0][3 + k] = m->weld_ts * e[1 + k]; }
#pragma unroll
    for (int k = 0; k < 4; k++) S.F[1][k] = e[k];
#pragma unroll
    for (int k = 0; k < 8; k++) S.F[2][k] = R2[k];
    S.F[3][0] = R2[8];
#pragma unroll
    for (int k = 0; k < 3; k++) S.F[3][4 + k] = p2[k];
  }
  __syncthreads();
  // columns: lane j = hinge j (the Jaw hinge, j = 5, is not on the ee chain)
  if (lane < 6) {
    const int j = lane;
    float R2[9], p2[3], e[4], ax[3], dp[3], c[3], a[3], v[3], vc[3];
#pragma unroll
    for (int k = 0; k < 8; k++) R2[k] = S.F[2][k];
    R2[8] = S.F[3][0];
#pragma unroll
    for (int k = 0; k < 3; k++) { p2[k] = S.F[3][4 + k]; ax[k] = sh.axis[j][k]; dp[k] = p2[k] - sh.anchor[j][k]; a[k] = -ax[k]; }
#pragma unroll
    for (int k = 0; k < 4; k++) e[k] = S.F[1][k];
    cross3(c, ax, dp);
    mulmtv3(v, R2, a);
    cross3(vc, v, e + 1);
    const bool on = j < 5;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      J[k][j] = on ? -c[k] : 0.f;
      J[3 + k][j] = on ? 0.5f * m->weld_ts * (e[0] * v[k] + vc[k]) : 0.f;
    }
  }
  __syncthreads();
  // rows: lane i
  if (lane < 6) {
    const int i = lane;
    float vel = 0.f;
#pragma unroll
    for (int j = 0; j < 6; j++) vel += J[i][j] * sh.qvel[j];
    const float pos = S.F[0][i];
    const float imp = getimpedance(m->weld_solimp, pos, 0.f);
    const float R = fmaxf(kMinVal, (1.f - imp) / imp * m->weld_invw[i < 3 ? 0 : 1]);
    const float D = 1.f / R;
    S.F[4][i] = D;
    S.F[5][i] = D * (-m->weld_B * vel - m->weld_K * imp * pos);
  }
  __syncthreads();
  // M += J'DJ (lane i: entries j <= i and their mirrors, as the CRBA), J'D aref -> F[1]
  if (lane < 6) {
    const int i = lane;
    float f = 0.f;
#pragma unroll
    for (int r = 0; r < 6; r++) f += J[r][i] * S.F[5][r];
#pragma unroll
    for (int j = 0; j < 6; j++) {
      if (j <= i) {
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < 6; r++) v += J[r][i] * S.F[4][r] * J[r][j];
        S.M[i][j] += v;
        if (j != i) S.M[j][i] += v;
      }
    }
    sh.qacc_smooth[i] = f;                    // staged here until tau (qacc_smooth is written last)
  }
  __syncthreads();
}

DEV void dynamics_par_lds(const DevModel* __restrict__ m, EnvShared& sh, int lane, float mscale DSTAMP_PARAMS) {
  SerialScratch& S = sh.ser;
  // ---- comPos (body a = lane): cinert about the tree reference point r = Base xpos; cdof
  if (lane < 6) {
    const int a = lane;
    const float* r = m->base_pos;
    float xm[9], xp[3], ax[3];
#pragma unroll
    for (int k = 0; k < 9; k++) xm[k] = S.xm[a][k];
#pragma unroll
    for (int k = 0; k < 3; k++) { xp[k] = S.xp[a][k]; ax[k] = sh.axis[a][k]; }
    float ip[3], xi[3], IM[9], diag[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, Ib[9], RT[9], Iw[9];
    mulmv3(ip, xm, m->body_ipos[a]);
#pragma unroll
    for (int k = 0; k < 3; k++) xi[k] = xp[k] + ip[k] - r[k];
    mulmm3(IM, xm, m->body_imat[a]);
    diag[0] = m->body_inertia[a][0]; diag[4] = m->body_inertia[a][1]; diag[8] = m->body_inertia[a][2];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) RT[3 * i + j] = IM[3 * j + i];
    mulmm3(Ib, IM, diag);
    mulmm3(Iw, Ib, RT);
    const float mass = m->body_mass[a];
    const float dd2 = dot3(xi, xi);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) S.cin[a][3 * i + j] = Iw[3 * i + j] + mass * ((i == j ? dd2 : 0.f) - xi[i] * xi[j]);
#pragma unroll
    for (int k = 0; k < 3; k++) S.cin[a][9 + k] = mass * xi[k];
    S.cin[a][12] = mass;
    float off[3] = {r[0] - xp[0], r[1] - xp[1], r[2] - xp[2]}, lin[3];
    cross3(lin, ax, off);
#pragma unroll
    for (int k = 0; k < 3; k++) { S.cdof[a][k] = ax[k]; S.cdof[a][3 + k] = lin[k]; }
  }
  __syncthreads();
  DSTAMP(2);
  // ---- CRBA: composite inertia crb_i = cin_5 + ... + cin_i (that order), F_i = crb_i cdof_i
  if (lane < 6) {
    const int i = lane;
    float crb[13];
#pragma unroll
    for (int k = 0; k < 13; k++) crb[k] = 0.f;
#pragma unroll
    for (int b = 5; b >= 0; b--) {
      if (b >= i) {
#pragma unroll
        for (int k = 0; k < 13; k++) crb[k] += S.cin[b][k];
      }
    }
    float F[6], cd[6];
#pragma unroll
    for (int k = 0; k < 6; k++) cd[k] = S.cdof[i][k];
    mul_inert(F, crb, cd);
#pragma unroll
    for (int k = 0; k < 6; k++) S.F[i][k] = F[k];
    // row i of M (j <= i) and its mirror: M(i,j) = cdof_j . F_i
#pragma unroll
    for (int j = 0; j < 6; j++) {
      if (j <= i) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 6; k++) v += S.cdof[j][k] * F[k];
        if (j == i) v += m->armature[i];
        S.M[i][j] = v;
        S.M[j][i] = v;
      }
    }
  }
  __syncthreads();
  DSTAMP(3);
  if (m->ee) weld_fold(m, sh, lane);
  // ---- Cholesky of the 6x6 on each of lanes 0..5 (the same instructions on the same values: no serial lane,
  // no barrier, no LDS round trip), then lane c solves M x = e_c for the M^-1 column c
  DSTAMP(4);
  if (lane < 6) {
    const int c = lane;
    float L[6][6], Linv[6], z[6], x[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
      float sdiag = S.M[j][j];
#pragma unroll
      for (int k = 0; k < j; k++) sdiag -= L[j][k] * L[j][k];
      const float sd = fmaxf(sdiag, kMinVal);
      Linv[j] = __builtin_amdgcn_rsqf(sd);          // 1 / L_jj by v_rsq (1 ulp), L_jj = sd / L_jj
      L[j][j] = sd * Linv[j];
#pragma unroll
      for (int i = j + 1; i < 6; i++) {
        float t = S.M[i][j];
#pragma unroll
        for (int k = 0; k < j; k++) t -= L[i][k] * L[j][k];
        L[i][j] = t * Linv[j];
      }
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
      float sacc = (i == c) ? 1.f : 0.f;
#pragma unroll
      for (int k = 0; k < i; k++) sacc -= L[i][k] * z[k];
      z[i] = sacc * Linv[i];
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
      float sacc = z[i];
#pragma unroll
      for (int k = i + 1; k < 6; k++) sacc -= L[k][i] * x[k];
      x[i] = sacc * Linv[i];
    }
#pragma unroll
    for (int i = 0; i < 6; i++) S.X[c][i] = x[i];
  }
  // ---- RNE (flg_acc = 0), part 1: cvel_a = sum_{k<=a} cdof_k qd_k, cdof_dot_a = cvel_a x cdof_a
  if (lane < 6) {
    const int a = lane;
    float cvel[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 6; b++) {
      if (b <= a) {
        const float qd = sh.qvel[b];
#pragma unroll
        for (int k = 0; k < 6; k++) cvel[k] += S.cdof[b][k] * qd;
      }
    }
    float cd[6], cdd[6];
#pragma unroll
    for (int k = 0; k < 6; k++) cd[k] = S.cdof[a][k];
    cross_motion(cdd, cvel, cd);
#pragma unroll
    for (int k = 0; k < 6; k++) S.cdd[a][k] = cdd[k];
  }
  __syncthreads();
  DSTAMP(5);
  // symmetrised M^-1 -> LDS (minv), RNE part 2: cacc_a = -g + sum_{k<=a} cdd_k qd_k, body forces
  if (lane < 6) {
    const int a = lane;
#pragma unroll
    for (int j = 0; j < 6; j++) sh.minv[a][j] = 0.5f * (S.X[j][a] + S.X[a][j]);
    float cvel[6] = {0, 0, 0, 0, 0, 0};
    float cacc[6] = {0, 0, 0, -m->gravity[0], -m->gravity[1], -m->gravity[2]};
#pragma unroll
    for (int b = 0; b < 6; b++) {
      if (b <= a) {
        const float qd = sh.qvel[b];
#pragma unroll
        for (int k = 0; k < 6; k++) cvel[k] += S.cdof[b][k] * qd;
#pragma unroll
        for (int k = 0; k < 6; k++) cacc[k] += S.cdd[b][k] * qd;
      }
    }
    float cin[13];
#pragma unroll
    for (int k = 0; k < 13; k++) cin[k] = S.cin[a][k];
    float f1[6], Iv[6], f2[6];
    mul_inert(f1, cin, cacc);
    mul_inert(Iv, cin, cvel);
    cross_force(f2, cvel, Iv);
#pragma unroll
    for (int k = 0; k < 6; k++) S.cfrc[a][k] = f1[k] + f2[k];
  }
  __syncthreads();
  DSTAMP(6);
  // ---- bias_a = cdof_a . sum_{k>=a} cfrc_k (suffix, from body 5 down); actuation
  float tau = 0.f;
  if (lane < 6) {
    const int a = lane;
    float acc[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int b = 5; b >= 0; b--) {
      if (b >= a) {
#pragma unroll
        for (int k = 0; k < 6; k++) acc[k] += S.cfrc[b][k];
      }
    }
    float bias = 0.f;
#pragma unroll
    for (int k = 0; k < 6; k++) bias += S.cdof[a][k] * acc[k];
    const float c = fminf(fmaxf(sh.ctrl[a], m->act_clo[a]), m->act_chi[a]);
    float f = m->act_kp[a] * c - m->act_kp[a] * sh.qpos[a] - m->act_kv[a] * sh.qvel[a];
    f = fminf(fmaxf(f, m->act_flo[a]), m->act_fhi[a]);
    tau = f - bias + (m->ee ? sh.qacc_smooth[a] : 0.f);   // + J'D aref of the weld (weld_fold)
  }
  // tau_j to every lane by DPP broadcasts, taken by the whole row before any lane branches (no barrier and
  // no LDS round trip; minv was written before the last barrier)
  float tj[6];
#pragma unroll
  for (int j = 0; j < 6; j++) tj[j] = bcast_row(tau, j);
  if (lane < 6) {
    const int i = lane;
    float sacc = 0.f;
#pragma unroll
    for (int j = 0; j < 6; j++) sacc += sh.minv[i][j] * tj[j];
    sh.qacc_smooth[i] = sacc;
  } else if (lane < 9) {
    // cube (free body): -bias / m = g, gyroscopic term on the rotational dofs
    const int k = lane - 6;
    const float mc = m->cube_mass * mscale;
    const float I3[3] = {m->cube_inertia[0] * mscale, m->cube_inertia[1] * mscale, m->cube_inertia[2] * mscale};
    const float w[3] = {sh.qvel[9], sh.qvel[10], sh.qvel[11]};
    float Iw3[3] = {I3[0] * w[0], I3[1] * w[1], I3[2] * w[2]}, gyro[3];
    cross3(gyro, w, Iw3);
    const float gk = k == 0 ? gyro[0] : (k == 1 ? gyro[1] : gyro[2]);
    const float Ik = k == 0 ? I3[0] : (k == 1 ? I3[1] : I3[2]);
    sh.qacc_smooth[6 + k] = (mc * m->gravity[k]) / mc;
    sh.qacc_smooth[9 + k] = -gk / Ik;
    sh.inv_mcube[k] = 1.0f / mc;
    sh.inv_mcube[3 + k] = 1.0f / Ik;
  }
}

DEV void dynamics_par_bcast(const DevModel* __restrict__ m, EnvShared& sh, int lane, float mscale DSTAMP_PARAMS) {
  SerialScratch& S = sh.ser;
  // ---- comPos (body a = lane): cinert about the tree reference point r = Base xpos; cdof.  Lanes >= 6 hold
  // zeros (the CRBA's row scans read them).
  float cin_r[13], cdof_r[6];
#pragma unroll
  for (int k = 0; k < 13; k++) cin_r[k] = 0.f;
#pragma unroll
  for (int k = 0; k < 6; k++) cdof_r[k] = 0.f;
  if (lane < 6) {
    const int a = lane;
    const float* r = m->base_pos;
    float xm[9], xp[3], ax[3];
#pragma unroll
    for (int k = 0; k < 9; k++) xm[k] = S.xm[a][k];
#pragma unroll
    for (int k = 0; k < 3; k++) { xp[k] = S.xp[a][k]; ax[k] = sh.axis[a][k]; }
    float ip[3], xi[3], IM[9], diag[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, Ib[9], RT[9], Iw[9];
    mulmv3(ip, xm, m->body_ipos[a]);
#pragma unroll
    for (int k = 0; k < 3; k++) xi[k] = xp[k] + ip[k] - r[k];
    mulmm3(IM, xm, m->body_imat[a]);
    diag[0] = m->body_inertia[a][0]; diag[4] = m->body_inertia[a][1]; diag[8] = m->body_inertia[a][2];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) RT[3 * i + j] = IM[3 * j + i];
    mulmm3(Ib, IM, diag);
    mulmm3(Iw, Ib, RT);
    const float mass = m->body_mass[a];
    const float dd2 = dot3(xi, xi);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) cin_r[3 * i + j] = Iw[3 * i + j] + mass * ((i == j ? dd2 : 0.f) - xi[i] * xi[j]);
#pragma unroll
    for (int k = 0; k < 3; k++) cin_r[9 + k] = mass * xi[k];
    cin_r[12] = mass;
    float off[3] = {r[0] - xp[0], r[1] - xp[1], r[2] - xp[2]}, lin[3];
    cross3(lin, ax, off);
#pragma unroll
    for (int k = 0; k < 3; k++) { cdof_r[k] = ax[k]; cdof_r[3 + k] = lin[k]; }
#pragma unroll
    for (int k = 0; k < 13; k++) S.cin[a][k] = cin_r[k];
#pragma unroll
    for (int k = 0; k < 6; k++) S.cdof[a][k] = cdof_r[k];
  }
  DSTAMP(2);
  // ---- CRBA: composite inertia crb_i = cin_5 + ... + cin_i (that order) from the bodies' lanes by row broadcasts
  // (round 2 read them from LDS after a barrier; the same sums bit for bit), F_i = crb_i cdof_i; row i of M
  // (j <= i) from the row's cdof_j broadcasts, and its mirror
  {
    float crb[13];
#pragma unroll
    for (int k = 0; k < 13; k++) crb[k] = 0.f;
#pragma unroll
    for (int b = 5; b >= 0; b--) {                 // the serial order (cin_5 first): bitwise the LDS version's sums
#pragma unroll
      for (int k = 0; k < 13; k++) {
        const float x = bcast_row(cin_r[k], b);
        crb[k] = b >= lane ? crb[k] + x : crb[k];
      }
    }
    float F[6];
    mul_inert(F, crb, cdof_r);
    float mrow[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < 6; k++) v += bcast_row(cdof_r[k], j) * F[k];
      mrow[j] = v;
    }
    if (lane < 6) {
      const int i = lane;
#pragma unroll
      for (int j = 0; j < 6; j++) {
        if (j <= i) {
          const float v = mrow[j] + (j == i ? m->armature[i] : 0.f);
          S.M[i][j] = v;
          S.M[j][i] = v;
        }
      }
    }
  }
  __syncthreads();
  DSTAMP(3);
  if (m->ee) weld_fold(m, sh, lane);
  // ---- Cholesky of the 6x6 on each of lanes 0..5 (the same instructions on the same values: no serial lane,
  // no barrier, no LDS round trip), then lane c solves M x = e_c for the M^-1 column c
  DSTAMP(4);
  if (lane < 6) {
    const int c = lane;
    float L[6][6], Linv[6], z[6], x[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
      float sdiag = S.M[j][j];
#pragma unroll
      for (int k = 0; k < j; k++) sdiag -= L[j][k] * L[j][k];
      const float sd = fmaxf(sdiag, kMinVal);
      Linv[j] = __builtin_amdgcn_rsqf(sd);          // 1 / L_jj by v_rsq (1 ulp), L_jj = sd / L_jj
      L[j][j] = sd * Linv[j];
#pragma unroll
      for (int i = j + 1; i < 6; i++) {
        float t = S.M[i][j];
#pragma unroll
        for (int k = 0; k < j; k++) t -= L[i][k] * L[j][k];
        L[i][j] = t * Linv[j];
      }
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
      float sacc = (i == c) ? 1.f : 0.f;
#pragma unroll
      for (int k = 0; k < i; k++) sacc -= L[i][k] * z[k];
      z[i] = sacc * Linv[i];
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
      float sacc = z[i];
#pragma unroll
      for (int k = i + 1; k < 6; k++) sacc -= L[k][i] * x[k];
      x[i] = sacc * Linv[i];
    }
#pragma unroll
    for (int i = 0; i < 6; i++) S.X[c][i] = x[i];
  }
  // ---- RNE (flg_acc = 0) from the bodies' lanes by row broadcasts, summed in the serial order (bitwise the sums
  // of round 2, which read the other bodies' cdof / cdd / cfrc from LDS after two barriers): cvel_a = sum_{k<=a}
  // cdof_k qd_k, cdof_dot_a = cvel_a x cdof_a, cacc_a = -g + sum_{k<=a} cdd_k qd_k, the body forces,
  // bias_a = cdof_a . sum_{k>=a} cfrc_k
  const float qd_own = lane < 6 ? sh.qvel[lane] : 0.f;
  float cvel[6], cdd[6], cacc[6];
#pragma unroll
  for (int k = 0; k < 6; k++) cvel[k] = 0.f;
#pragma unroll
  for (int b = 0; b < 6; b++) {                   // serial order, as the LDS version
    const float qd = bcast_row(qd_own, b);
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const float x = bcast_row(cdof_r[k], b);
      cvel[k] = b <= lane ? cvel[k] + x * qd : cvel[k];
    }
  }
  cross_motion(cdd, cvel, cdof_r);
  cacc[0] = cacc[1] = cacc[2] = 0.f;
  cacc[3] = -m->gravity[0]; cacc[4] = -m->gravity[1]; cacc[5] = -m->gravity[2];
#pragma unroll
  for (int b = 0; b < 6; b++) {
    const float qd = bcast_row(qd_own, b);
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const float x = bcast_row(cdd[k], b);
      cacc[k] = b <= lane ? cacc[k] + x * qd : cacc[k];
    }
  }
  float cfrc[6];
  {
    float f1[6], Iv[6], f2[6];
    mul_inert(f1, cin_r, cacc);
    mul_inert(Iv, cin_r, cvel);
    cross_force(f2, cvel, Iv);
#pragma unroll
    for (int k = 0; k < 6; k++) cfrc[k] = f1[k] + f2[k];
  }
  float facc[6];                                  // sum_{k>=a} cfrc_k, from body 5 down (serial order)
#pragma unroll
  for (int k = 0; k < 6; k++) facc[k] = 0.f;
#pragma unroll
  for (int b = 5; b >= 0; b--) {
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const float x = bcast_row(cfrc[k], b);
      facc[k] = b >= lane ? facc[k] + x : facc[k];
    }
  }
  __syncthreads();               // the M^-1 columns of the other lanes (S.X)
  DSTAMP(5);
  // symmetrised M^-1 -> LDS (minv; each lane its own row, read back only by itself)
  if (lane < 6) {
    const int a = lane;
#pragma unroll
    for (int j = 0; j < 6; j++) sh.minv[a][j] = 0.5f * (S.X[j][a] + S.X[a][j]);
  }
  DSTAMP(6);
  // ---- actuation
  float tau = 0.f;
  if (lane < 6) {
    const int a = lane;
    float bias = 0.f;
#pragma unroll
    for (int k = 0; k < 6; k++) bias += cdof_r[k] * facc[k];
    const float c = fminf(fmaxf(sh.ctrl[a], m->act_clo[a]), m->act_chi[a]);
    float f = m->act_kp[a] * c - m->act_kp[a] * sh.qpos[a] - m->act_kv[a] * sh.qvel[a];
    f = fminf(fmaxf(f, m->act_flo[a]), m->act_fhi[a]);
    tau = f - bias + (m->ee ? sh.qacc_smooth[a] : 0.f);   // + J'D aref of the weld (weld_fold)
  }
  // tau_j to every lane by DPP broadcasts, taken by the whole row before any lane branches (no barrier and
  // no LDS round trip; minv was written before the last barrier)
  float tj[6];
#pragma unroll
  for (int j = 0; j < 6; j++) tj[j] = bcast_row(tau, j);
  if (lane < 6) {
    const int i = lane;
    float sacc = 0.f;
#pragma unroll
    for (int j = 0; j < 6; j++) sacc += sh.minv[i][j] * tj[j];
    sh.qacc_smooth[i] = sacc;
  } else if (lane < 9) {
    // cube (free body): -bias / m = g, gyroscopic term on the rotational dofs
    const int k = lane - 6;
    const float mc = m->cube_mass * mscale;
    const float I3[3] = {m->cube_inertia[0] * mscale, m->cube_inertia[1] * mscale, m->cube_inertia[2] * mscale};
    const float w[3] = {sh.qvel[9], sh.qvel[10], sh.qvel[11]};
    float Iw3[3] = {I3[0] * w[0], I3[1] * w[1], I3[2] * w[2]}, gyro[3];
    cross3(gyro, w, Iw3);
    const float gk = k == 0 ? gyro[0] : (k == 1 ? gyro[1] : gyro[2]);
    const float Ik = k == 0 ? I3[0] : (k == 1 ? I3[1] : I3[2]);
    sh.qacc_smooth[6 + k] = (mc * m->gravity[k]) / mc;
    sh.qacc_smooth[9 + k] = -gk / Ik;
    sh.inv_mcube[k] = 1.0f / mc;
    sh.inv_mcube[3 + k] = 1.0f / Ik;
  }
}

// The arm's dynamics, two schedules of the same arithmetic (bitwise the same results, tools/dev/lib_states.py):
// dynamics_par_lds exchanges the bodies' cinert / cdof / cdd / cfrc through LDS with barriers; dynamics_par_bcast
// takes them from the bodies' lanes by row broadcasts, summed in the same serial order.  The broadcast schedule has
// the shorter latency chain and more VALU instructions: +0.8 % env steps/s at 8,192 envs (2-wave fused build, every
// wave resident, the step latency-bound), -2.0 % at 65,536 (3-wave build, issue-bound), same-box A/B
// (profiles/r03_ab_dyn_bcast.txt); the 2-wave fused build takes it (+0.9 % at 8,192, profiles/r03_ab_dyn_bcast_w2.txt).
template <bool kBcast>
DEV void dynamics_par(const DevModel* __restrict__ m, EnvShared& sh, int lane, float mscale DSTAMP_PARAMS) {
  if constexpr (kBcast) dynamics_par_bcast(m, sh, lane, mscale DSTAMP_ARGS);
  else dynamics_par_lds(m, sh, lane, mscale DSTAMP_ARGS);
}

// ------------------------------------------------------------------ box-box narrowphase (one pair per lane)
struct PairContacts {
  int n;
  float normal[3];
  float pos[SO100_MAXCONPAIR][3];
  float dist[SO100_MAXCONPAIR];
};

// Register-resident polygons: fixed 8 slots written by select chains (static indices only), so the
// clipping never touches scratch memory.  Same Sutherland-Hodgman order and 8-vertex cap as the oracle.
struct Poly8 {
  float x[8], y[8];
  int n;
};
DEV void poly_push(Poly8& p, float x, float y) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const bool w = (k == p.n);
    p.x[k] = w ? x : p.x[k];
    p.y[k] = w ? y : p.y[k];
  }
  p.n = p.n + 1;
}
// clip polygon q by the half-plane sign * coord[dir] < h (rectangle side), result in r
DEV void clip_stage(const Poly8& q, Poly8& r, int dir, float sign, float h) {
  r.n = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (i < q.n && r.n < 8) {
      const float ax = q.x[i], ay = q.y[i];
      const bool last = (i + 1 >= q.n);
      const float bx = last ? q.x[0] : q.x[(i + 1) & 7], by = last ? q.y[0] : q.y[(i + 1) & 7];
      const float ad = dir ? ay : ax, bd = dir ? by : bx;
      const bool ina = sign * ad < h, inb = sign * bd < h;
      if (ina) poly_push(r, ax, ay);
      if (ina != inb && r.n < 8) {
        const float lim = sign * h;
        const float ao = dir ? ax : ay, bo = dir ? bx : by;
        const float o = ao + (bo - ao) / (bd - ad) * (lim - ad);
        if (dir) poly_push(r, o, lim); else poly_push(r, lim, o);
      }
    }
  }
}

// Runtime-indexed reads of small register arrays as masked blends a0 w0 + a1 w1 + a2 w2 (one weight 1,
// exact for finite values).  A pointer, a dynamic index, or a select chain (which the compiler folds back
// into an index) would force the array into scratch memory.
DEV void onehot3(int i, float* w) { w[0] = i == 0 ? 1.f : 0.f; w[1] = i == 1 ? 1.f : 0.f; w[2] = i == 2 ? 1.f : 0.f; }
DEV float sel3(const float* a, int i) {
  float w[3];
  onehot3(i, w);
  return a[0] * w[0] + a[1] * w[1] + a[2] * w[2];
}
DEV void col3(float* o, const float* R, int c) {          // column c of a row-major 3x3
  float w[3];
  onehot3(c, w);
#pragma unroll
  for (int t = 0; t < 3; t++) o[t] = R[3 * t] * w[0] + R[3 * t + 1] * w[1] + R[3 * t + 2] * w[2];
}

// collapse: the pair is the cube against the table's mesh, one contact (MuJoCo's convex collider; the oracle's
// collide_box_pair): the mean of the kept points' positions and the deepest distance, summed in clip order as
// the kept points would be, without their compaction and 8-slot output (bitwise the same contact)
DEV void box_box(const float* p1, const float* R1, const float* A, const float* p2, const float* R2,
                 const float* B, float margin, PairContacts& out, bool collapse) {
  out.n = 0;
  float pd[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]}, pp[3], R[9], Q[9];
  mulmtv3(pp, R1, pd);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      R[3 * i + j] = R1[i] * R2[j] + R1[3 + i] * R2[3 + j] + R1[6 + i] * R2[6 + j];
      Q[3 * i + j] = fabsf(R[3 * i + j]) + 1e-6f;
    }
  float best = -1e30f, nb[3] = {0, 0, 0};
  int code = 0;
  bool invert = false;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    float s = fabsf(pp[i]) - (A[i] + B[0] * Q[3 * i] + B[1] * Q[3 * i + 1] + B[2] * Q[3 * i + 2]);
    if (s > margin) return;
    if (s > best) { best = s; code = 1 + i; invert = pp[i] < 0; nb[0] = nb[1] = nb[2] = 0; nb[i] = 1; }
  }
#pragma unroll
  for (int j = 0; j < 3; j++) {
    float e = pp[0] * R[j] + pp[1] * R[3 + j] + pp[2] * R[6 + j];
    float s = fabsf(e) - (A[0] * Q[j] + A[1] * Q[3 + j] + A[2] * Q[6 + j] + B[j]);
    if (s > margin) return;
    if (s > best) { best = s; code = 4 + j; invert = e < 0; nb[0] = R[j]; nb[1] = R[3 + j]; nb[2] = R[6 + j]; }
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      float n[3] = {0, 0, 0};
      n[i1] = -R[3 * i2 + j];
      n[i2] = R[3 * i1 + j];
      const float l2 = n[i1] * n[i1] + n[i2] * n[i2];
      if (l2 < 1e-10f) continue;                   // |n| < 1e-5
      const float linv = __builtin_amdgcn_rsqf(l2);   // v_rsq (1 ulp): one instruction on the env's chain
      float e = pp[i2] * R[3 * i1 + j] - pp[i1] * R[3 * i2 + j];
      float ex = A[i1] * Q[3 * i2 + j] + A[i2] * Q[3 * i1 + j] + B[j1] * Q[3 * i + j2] + B[j2] * Q[3 * i + j1];
      float s = (fabsf(e) - ex) * linv;
      if (s > margin) return;
      if (s * 1.05f > best) {
        best = s; code = 7 + 3 * i + j; invert = e < 0;
        nb[0] = n[0] * linv; nb[1] = n[1] * linv; nb[2] = n[2] * linv;
      }
    }
  }
  if (code == 0) return;
  float normal[3];
  mulmv3(normal, R1, nb);
  if (invert) { normal[0] = -normal[0]; normal[1] = -normal[1]; normal[2] = -normal[2]; }
  out.normal[0] = normal[0]; out.normal[1] = normal[1]; out.normal[2] = normal[2];
  const float depth0 = -best;

  if (code > 6) {
    const int i = (code - 7) / 3, j = (code - 7) % 3;
    float pa[3] = {p1[0], p1[1], p1[2]}, pb[3] = {p2[0], p2[1], p2[2]};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      {
        float ax[3] = {R1[k], R1[3 + k], R1[6 + k]};
        float sg = k == i ? 0.f : (dot3(normal, ax) > 0 ? 1.f : -1.f);
#pragma unroll
        for (int t = 0; t < 3; t++) pa[t] += sg * A[k] * ax[t];
      }
      {
        float ax[3] = {R2[k], R2[3 + k], R2[6 + k]};
        float sg = k == j ? 0.f : (dot3(normal, ax) > 0 ? -1.f : 1.f);
#pragma unroll
        for (int t = 0; t < 3; t++) pb[t] += sg * B[k] * ax[t];
      }
    }
    float ua[3], ub[3];
    col3(ua, R1, i);
    col3(ub, R2, j);
    float pq[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
    float uaub = dot3(ua, ub), q1 = dot3(ua, pq), q2 = -dot3(ub, pq);
    float den = 1.f - uaub * uaub, al = 0.f, be = 0.f;
    if (den > 1e-4f) { den = 1.f / den; al = (q1 + uaub * q2) * den; be = (uaub * q1 + q2) * den; }
    float pc0[3];
#pragma unroll
    for (int t = 0; t < 3; t++) {
      pa[t] += ua[t] * al;
      pb[t] += ub[t] * be;
      pc0[t] = 0.5f * (pa[t] + pb[t]);
    }
    // every slot, in the face path's store order (only slot 0 counts: n = 1): the compiler merges the two
    // exits' stores, and stores to different slots became one store at a run-time slot index (scratch)
#pragma unroll
    for (int c = 0; c < SO100_MAXCONPAIR; c++) {
#pragma unroll
      for (int t = 0; t < 3; t++) out.pos[c][t] = pc0[t];
      out.dist[c] = -depth0;
    }
    out.n = 1;
    return;
  }

  // reference box (face normal) and incident box, selected by value (no pointer / dynamic index)
  const bool ref1 = code <= 3;
  float pR[3], RR[9], SR[3], pI[3], RI[9], SI[3], nref[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    pR[k] = ref1 ? p1[k] : p2[k]; pI[k] = ref1 ? p2[k] : p1[k];
    SR[k] = ref1 ? A[k] : B[k];   SI[k] = ref1 ? B[k] : A[k];
    nref[k] = ref1 ? normal[k] : -normal[k];
  }
#pragma unroll
  for (int k = 0; k < 9; k++) { RR[k] = ref1 ? R1[k] : R2[k]; RI[k] = ref1 ? R2[k] : R1[k]; }
  const int codeN = ref1 ? code - 1 : code - 4;
  float nr[3], anr[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    float ax[3] = {RI[k], RI[3 + k], RI[6 + k]};
    nr[k] = dot3(nref, ax);
    anr[k] = fabsf(nr[k]);
  }
  int lanr = (anr[1] > anr[0]) ? ((anr[1] > anr[2]) ? 1 : 2) : ((anr[0] > anr[2]) ? 0 : 2);
  float center[3], ril[3];
  col3(ril, RI, lanr);
  const float sil = sel3(SI, lanr), nrl = sel3(nr, lanr);
#pragma unroll
  for (int t = 0; t < 3; t++) center[t] = pI[t] - pR[t] + (nrl < 0 ? sil : -sil) * ril[t];
  const int c1 = (codeN == 0) ? 1 : 0, c2 = (codeN == 2) ? 1 : 2;
  const int a1 = (lanr == 0) ? 1 : 0, a2 = (lanr == 2) ? 1 : 2;
  float u1[3], u2[3], v1[3], v2[3];
  col3(u1, RR, c1);
  col3(u2, RR, c2);
  col3(v1, RI, a1);
  col3(v2, RI, a2);
  float cc1 = dot3(center, u1), cc2 = dot3(center, u2);
  float m11 = dot3(u1, v1), m12 = dot3(u1, v2), m21 = dot3(u2, v1), m22 = dot3(u2, v2);
  const float sia1 = sel3(SI, a1), sia2 = sel3(SI, a2);
  float k1 = m11 * sia1, k2 = m21 * sia1, k3 = m12 * sia2, k4 = m22 * sia2;
  Poly8 P, Pq;
  P.n = 4;
  P.x[0] = cc1 - k1 - k3; P.y[0] = cc2 - k2 - k4;
  P.x[1] = cc1 - k1 + k3; P.y[1] = cc2 - k2 + k4;
  P.x[2] = cc1 + k1 + k3; P.y[2] = cc2 + k2 + k4;
  P.x[3] = cc1 + k1 - k3; P.y[3] = cc2 + k2 - k4;
#pragma unroll
  for (int k = 4; k < 8; k++) { P.x[k] = 0.f; P.y[k] = 0.f; }
  const float src1 = sel3(SR, c1), src2 = sel3(SR, c2), srcN = sel3(SR, codeN);
  // an incident face inside the reference face's rectangle (the cube resting on the table) passes the
  // four clip stages unchanged, in order: skip them (bitwise the same polygon)
  bool inside = true;
#pragma unroll
  for (int k = 0; k < 4; k++) inside = inside && -P.x[k] < src1 && P.x[k] < src1 && -P.y[k] < src2 && P.y[k] < src2;
  if (!inside) {
    clip_stage(P, Pq, 0, -1.f, src1);
    clip_stage(Pq, P, 0, 1.f, src1);
    clip_stage(P, Pq, 1, -1.f, src2);
    clip_stage(Pq, P, 1, 1.f, src2);
  }
  const int n = P.n;
  if (n < 1) return;
  float det = m11 * m22 - m12 * m21;
  if (fabsf(det) < 1e-12f) return;
  det = 1.f / det;
  const float i11 = m22 * det, i12 = -m12 * det, i21 = -m21 * det, i22 = m11 * det;
  if (collapse) {
    float sp[3] = {0.f, 0.f, 0.f}, dmin = 0.f;
    int cnum = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (k < n) {
        const float x = P.x[k] - cc1, y = P.y[k] - cc2;
        const float s1 = i11 * x + i12 * y, s2 = i21 * x + i22 * y;
        float pt[3];
        for (int t = 0; t < 3; t++) pt[t] = center[t] + s1 * v1[t] + s2 * v2[t];
        const float dp = srcN - dot3(nref, pt);
        if (dp > -margin) {
#pragma unroll
          for (int t = 0; t < 3; t++) sp[t] += pt[t] + pR[t] + 0.5f * dp * nref[t];
          dmin = (cnum == 0 || -dp < dmin) ? -dp : dmin;
          cnum++;
        }
      }
    }
    if (cnum < 1) return;
    const float nf = (float)cnum;
#pragma unroll
    for (int c = 0; c < SO100_MAXCONPAIR; c++) {     // every slot (no run-time slot index: see below)
#pragma unroll
      for (int t = 0; t < 3; t++) out.pos[c][t] = sp[t] / nf;
      out.dist[c] = dmin;
    }
    out.n = 1;
    return;
  }
  // keep the penetrating points (compacted in order; 2D coords in K, depth in D)
  Poly8 K;
  K.n = 0;
  float D[8];
#pragma unroll
  for (int k = 0; k < 8; k++) { K.x[k] = 0.f; K.y[k] = 0.f; D[k] = 0.f; }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (k < n) {
      const float x = P.x[k] - cc1, y = P.y[k] - cc2;
      const float s1 = i11 * x + i12 * y, s2 = i21 * x + i22 * y;
      float pt[3];
      for (int t = 0; t < 3; t++) pt[t] = center[t] + s1 * v1[t] + s2 * v2[t];
      const float dp = srcN - dot3(nref, pt);
      if (dp > -margin) {
#pragma unroll
        for (int q2 = 0; q2 < 8; q2++) D[q2] = (q2 == K.n) ? dp : D[q2];
        poly_push(K, P.x[k], P.y[k]);
      }
    }
  }
  const int cnum = K.n;
  if (cnum < 1) return;
  // every clipped point within the margin, in clip order (up to 8: mjc_BoxBox keeps them all).  Every slot is
  // written unconditionally (slots >= cnum are never read): stores under `c < cnum` were merged by the compiler
  // into one store with a run-time slot index, which put `out` in scratch memory
  static_assert(SO100_MAXCONPAIR == 8, "the clip polygon holds 8 points");
#pragma unroll
  for (int c = 0; c < SO100_MAXCONPAIR; c++) {
    const float x = K.x[c], y = K.y[c], dp = D[c];
    const float xr = x - cc1, yr = y - cc2;
    const float s1 = i11 * xr + i12 * yr, s2 = i21 * xr + i22 * yr;
#pragma unroll
    for (int t = 0; t < 3; t++) {
      const float pt = center[t] + s1 * v1[t] + s2 * v2[t];
      out.pos[c][t] = pt + pR[t] + 0.5f * dp * nref[t];
    }
    out.dist[c] = -dp;
  }
  out.n = cnum;
}

// geom world pose from the staged body frames; b = the geom's body (a pair's body id, pair_b1 / pair_b2, loaded
// beside its geom id instead of after it: so100_create checks pair_b = geom_body[pair_g])
DEV void geom_pose_b(const DevModel* __restrict__ m, const EnvShared& sh, int g, int b, float* pos, float* mat) {
  if (b == 0) {
#pragma unroll
    for (int k = 0; k < 3; k++) pos[k] = m->geom_pos[g][k];
#pragma unroll
    for (int k = 0; k < 9; k++) mat[k] = m->geom_mat[g][k];
    return;
  }
  const float* bp;
  const float* bm;
  if (b == SO100_CUBE_BODY) { bp = sh.cube_pos; bm = sh.cube_mat; }
  else { bp = sh.jaw_pos[b - 6]; bm = sh.jaw_mat[b - 6]; }
  float t[3];
  mulmv3(t, bm, m->geom_pos[g]);
#pragma unroll
  for (int k = 0; k < 3; k++) pos[k] = bp[k] + t[k];
  mulmm3(mat, bm, m->geom_mat[g]);
}
DEV void geom_pose(const DevModel* __restrict__ m, const EnvShared& sh, int g, float* pos, float* mat) {
  geom_pose_b(m, sh, g, m->geom_body[g], pos, mat);
}

DEV void collide_pair(const DevModel* __restrict__ m, const EnvShared& sh, int p, PairContacts& pc) {
  pc.n = 0;
  const int g1 = m->pair_g1[p], g2 = m->pair_g2[p];
  float p1[3], R1[9], p2[3], R2[9];
  geom_pose_b(m, sh, g1, m->pair_b1[p], p1, R1);
  geom_pose_b(m, sh, g2, m->pair_b2[p], p2, R2);
  const float* A = m->geom_size[g1];
  const float* B = m->geom_size[g2];
  float d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  const float margin = m->pair_margin[p];
  if (sqrtf(dot3(d, d)) > sqrtf(dot3(A, A)) + sqrtf(dot3(B, B)) + margin) return;
  // the cube against the table's mesh (geom2 = geom 0): MuJoCo's convex collider, one contact per pair (the
  // oracle's collide_box_pair): the SAT normal, the deepest distance, the mean of the clipped positions
  box_box(p1, R1, A, p2, R2, B, margin, pc, g2 == 0);
}

// Arm/jaw hulls vs the table top (pairs SO100_NPAIR_BOX + k; oracle collision()): hull k's lowest
// vertex inside the top face's x-y footprint, a contact when it is below the top.
//  * broadphase, in parallel: lane k < SO100_NHULL of each env tests hull k's body-frame bounding box
//    against the top; only hulls that are candidates in some env of the wave are scanned;
//  * scan: the 16 lanes of the env's row split the vertices (lane, lane + 16, ...) and a 16-lane
//    lexicographic (z, vertex index) min gives the oracle's first lowest vertex.
// Needs the link frames of fk_stage (sh.ser.xm / xp).  Lane k < SO100_NHULL returns hull k's contact
// flag and its lowest vertex.
DEV bool hull_table(const DevModel* __restrict__ m, const EnvShared& sh, int lane, int grp, bool valid, float& hx,
                    float& hy, float& hz) {
  bool found = false;
  hx = hy = hz = 0.f;
#ifdef SO100_EXPERIMENT_NO_HULLS
  return false;   // timing experiment only: hull contacts off
#endif
  const float top = m->table_top;
  bool cand = false;
  if (valid && lane < SO100_NHULL) {
    const int a = m->hull_body[lane] - 2;
    const float4 hc = reinterpret_cast<const float4*>(m->hull_center)[lane];
    const float4 hh = reinterpret_cast<const float4*>(m->hull_half)[lane];
    const float r6 = sh.ser.xm[a][6], r7 = sh.ser.xm[a][7], r8 = sh.ser.xm[a][8];
    const float cz = (r6 * hc.x + r7 * hc.y + r8 * hc.z) + sh.ser.xp[a][2];
    const float ext = fabsf(r6) * hh.x + fabsf(r7) * hh.y + fabsf(r8) * hh.z;
    cand = cz - ext < top + m->pair_margin[SO100_NPAIR_BOX + lane];
  }
  const uint64_t cm = __ballot(cand);
  const uint32_t env_cand = (uint32_t)(cm >> (grp * 16)) & 0xFFFFu;
  uint32_t wave_cand = (uint32_t)((cm | (cm >> 16) | (cm >> 32) | (cm >> 48)) & 0xFFFFull);
  const float lo0 = m->table_lo[0], lo1 = m->table_lo[1], hi0 = m->table_hi[0], hi1 = m->table_hi[1];
  const float4* __restrict__ verts = reinterpret_cast<const float4*>(m->hull_vert);
  while (wave_cand) {
    const int k = __builtin_ctz(wave_cand);
    wave_cand &= wave_cand - 1u;
    const bool mine = (env_cand >> k) & 1u;
    float bz = __builtin_inff(), bx = 0.f, by = 0.f;
    int bi = 0x7fffffff;
    if (mine) {
      const int a = m->hull_body[k] - 2;
      const float* R = sh.ser.xm[a];
      const float* P = sh.ser.xp[a];
      const float r0 = R[0], r1 = R[1], r2 = R[2], r3 = R[3], r4 = R[4], r5 = R[5], r6 = R[6], r7 = R[7], r8 = R[8];
      const float p0 = P[0], p1 = P[1], p2 = P[2];
      const int n = m->hull_count[k], s0 = m->hull_start[k];
      for (int i = lane; i < n; i += kLanes) {
        const float4 v = verts[s0 + i];
        const float wx = (r0 * v.x + r1 * v.y + r2 * v.z) + p0;
        const float wy = (r3 * v.x + r4 * v.y + r5 * v.z) + p1;
        const float wz = (r6 * v.x + r7 * v.y + r8 * v.z) + p2;
        const bool in = wx >= lo0 && wx <= hi0 && wy >= lo1 && wy <= hi1;
        if (in && wz < bz) { bz = wz; bx = wx; by = wy; bi = i; }
      }
    }
    arg_best16<true>(bz, bi, bx, by, bz);   // the score is the point's z (passed as both)
    if (lane == k) {
      found = mine && bi != 0x7fffffff && (bz - top < m->pair_margin[SO100_NPAIR_BOX + k]);
      hx = bx; hy = by; hz = bz;
    }
  }
  return found;
}

// ------------------------------------------------------------------ box vs convex hull: MPR (oracle mpr_*)
// MuJoCo mjc_Convex -> libccd ccdMPRPenetration, restated (oracle/so100_oracle.c):
// obj1 = the box (cube or a bin box), obj2 = hull k, in hull k's body frame H.  Every lane of the env's
// row runs the portal arithmetic redundantly; the hull support is lane-parallel (lanes split the
// vertices, a 16-lane (score, index) max keeps the oracle's first maximal vertex), so all 16 lanes hold
// bitwise-identical portals and take identical branches.  Portal slots are only ever addressed by
// constant indices (no scratch).
struct MprSup {
  float v[3], v1[3], v2[3];
  uint32_t id;                      // the supports: obj1 box corner signs (bits 0..2) or hull vertex (0..9), obj2 hull
                                    // vertex << 10 (EPA rebuilds a vertex from it: sup_from_id)
};
#ifndef SO100_SMALL_HULL_REG
#define SO100_SMALL_HULL_REG 0
#endif
struct MprObj {
  float c[3], ax[9], h[3];          // obj1 frame in H: origin (box centre / hull body origin), axes
                                    // (columns of ax); box half sizes
  float c1[3], bc[3], bh[3];        // obj1 centre (box centre / hull centroid), bounding box centre and half
                                    // extents (axes ax), in H
  float hc[3];                      // obj2 (hull) centroid in H
  int hull1;                        // obj1: -1 a box, else a hull (self-collision); uniform over the wave
  int s1, n1;                       // obj1 hull vertex range
  int k, s0, n;                     // obj2: hull index, vertex range
  bool cells;                       // hull supports through the direction cells (fused kernel) or full scans
#if SO100_SMALL_HULL_REG
  float4 v2r;                       // obj2 hull of at most 16 vertices: the lane's vertex, held for the item
#endif
};
constexpr float kCcdEps = 2.220446049250313e-16f;   // MuJoCo's double libccd CCD_EPS (absolute tests: see oracle)
constexpr float kMprTol = 1e-6f;            // MuJoCo ccd_tolerance
constexpr int kMprIters = 50;               // MuJoCo ccd_iterations

DEV bool ccd_zero(float x) { return fabsf(x) < kCcdEps; }
DEV bool ccd_eq(float a, float b) {
  const float ab = fabsf(a - b);
  if (ab < kCcdEps) return true;
  const float fa = fabsf(a), fb = fabsf(b);
  return fb > fa ? ab < kCcdEps * fb : ab < kCcdEps * fa;
}
DEV void normalize3(float* v) {
  const float k = 1.0f / sqrtf(dot3(v, v));
  v[0] *= k; v[1] *= k; v[2] *= k;
}
DEV void sub3(float* r, const float* a, const float* b) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
// d = w ? s : d as unconditional selects: a conditional copy between portal slots would be folded into a
// store through a selected pointer, which puts the portal in scratch memory
DEV void sup_sel(MprSup& d, const MprSup& s, bool w) {
#pragma unroll
  for (int t = 0; t < 3; t++) {
    d.v[t] = w ? s.v[t] : d.v[t];
    d.v1[t] = w ? s.v1[t] : d.v1[t];
    d.v2[t] = w ? s.v2[t] : d.v2[t];
  }
  d.id = w ? s.id : d.id;
}

// A pointer read from the model (hull_cand, hull_blk) is generic to the compiler, so its loads were flat loads,
// which also count on lgkmcnt: every wait for them drained the LDS traffic too.  ld_global4 makes them global.
// (Device pass only: address spaces do not exist in the host pass of this translation unit.)
typedef float f4v __attribute__((ext_vector_type(4)));
DEV float4 ld_global4(const float4* p, size_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  const f4v v = ((const __attribute__((address_space(1))) f4v*)(const void*)p)[i];
  return make_float4(v.x, v.y, v.z, v.w);
#else
  return p[i];
#endif
}
// a vertex's support score n . v with one fixed rounding (explicit FMAs): the cell block, the cell list and the
// whole-hull scan must score a vertex bitwise alike, so that near-ties resolve alike (the fused and split paths
// use different ones and are bitwise equal)
DEV float sup_score(float n0, float n1, float n2, float x, float y, float z) {
  return __builtin_fmaf(n2, z, __builtin_fmaf(n1, y, n0 * x));
}
// first vertex of hull k (vertex range [s0, s0 + n)) maximising (n0, n1, n2) . v: lanes split the
// candidates, then a 16-lane (score, index) max keeps the oracle's first maximal vertex; every lane of the
// row gets it.  The candidates are those of the direction's cube-map cell (so100_hull_cells: a superset of
// the cell's possible supports, in vertex order, so the same vertex as a scan of the whole hull, which
// remains for a cell whose list did not fit and for a zero or non-finite direction).  The direction is
// uniform over the row, so is the path.
DEV float4 hull_support(const DevModel* __restrict__ m, bool cells, int k, int s0, int cnt, float n0, float n1, float n2,
                        int lane) {   // (x, y, z, vertex index within the hull as int bits)
  float best = -__builtin_inff(), bx = 0.f, by = 0.f, bz = 0.f;
  int bi = 0x7fffffff;
  {
    const float a0 = fabsf(n0), a1 = fabsf(n1), a2 = fabsf(n2);
    const bool fx = a0 >= a1 && a0 >= a2, fy = !fx && a1 >= a2;
    const float am = fx ? a0 : fy ? a1 : a2;
    uint32_t e = 0u;
#ifdef SO100_NO_HULL_CELLS
    if (false) {                             // A/B diagnostic builds only: the whole-hull scan
#else
    if (cells && am > 1e-30f && am < __builtin_inff()) {
#endif
      const float na = fx ? n0 : fy ? n1 : n2, nu = fx ? n1 : n0, nv = (fx || fy) ? n2 : n1;
      const float g = 0.5f * (float)SO100_HULL_CELLG / am;
      const int cu = min(max((int)((nu + am) * g), 0), SO100_HULL_CELLG - 1);
      const int cv = min(max((int)((nv + am) * g), 0), SO100_HULL_CELLG - 1);
      const int face = 2 * (fx ? 0 : fy ? 1 : 2) + (na >= 0.f ? 0 : 1);
      const int cell = k * SO100_HULL_NCELL + (face * SO100_HULL_CELLG + cu) * SO100_HULL_CELLG + cv;
      // the cell entry and the lane's candidate of the cell's block, loaded together (one memory latency)
      const float4 cb = ld_global4(reinterpret_cast<const float4*>(m->hull_blk), (size_t)cell * kCellBlk + lane);
      e = m->hull_cells[cell];
      const int cn = (int)(e & 255u);
      if (cn > 0 && cn <= kCellBlk) {
        // lanes beyond the list hold its last candidate again: the same (score, index), the same winner
        best = sup_score(n0, n1, n2, cb.x, cb.y, cb.z);
        bi = __float_as_int(cb.w); bx = cb.x; by = cb.y; bz = cb.z;
        arg_best16<false>(best, bi, bx, by, bz);
        return make_float4(bx, by, bz, __int_as_float(bi));
      }
    }
    const int cc = (int)(e & 255u);
    if (cc > 0) {
      const float4* __restrict__ cand = reinterpret_cast<const float4*>(m->hull_cand) + (e >> 8);
      for (int base = lane; base < cc; base += 2 * kLanes) {
        const float4 c0 = ld_global4(cand, base);
        const float4 c1 = ld_global4(cand, min(base + kLanes, cc - 1));
        const float s0c = sup_score(n0, n1, n2, c0.x, c0.y, c0.z);
        if (s0c > best) { best = s0c; bi = __float_as_int(c0.w); bx = c0.x; by = c0.y; bz = c0.z; }
        const float s1c = sup_score(n0, n1, n2, c1.x, c1.y, c1.z);
        if (base + kLanes < cc && s1c > best) { best = s1c; bi = __float_as_int(c1.w); bx = c1.x; by = c1.y; bz = c1.z; }
      }
      arg_best16<false>(best, bi, bx, by, bz);
      return make_float4(bx, by, bz, __int_as_float(bi));
    }
  }
  const float4* __restrict__ verts = reinterpret_cast<const float4*>(m->hull_vert) + s0;
  for (int base = lane; base < cnt; base += 8 * kLanes) {
    float4 vb[8];
#pragma unroll
    for (int u = 0; u < 8; u++) vb[u] = verts[min(base + u * kLanes, cnt - 1)];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int i = base + u * kLanes;
      const float sc = sup_score(n0, n1, n2, vb[u].x, vb[u].y, vb[u].z);
      const bool t = i < cnt && sc > best;
      best = t ? sc : best; bi = t ? i : bi;
      bx = t ? vb[u].x : bx; by = t ? vb[u].y : by; bz = t ? vb[u].z : bz;
    }
  }
  arg_best16<false>(best, bi, bx, by, bz);
  return make_float4(bx, by, bz, __int_as_float(bi));
}

#if SO100_SMALL_HULL_REG
// the support of a hull of at most 16 vertices from the row's register-held vertices (lane l: vertex min(l, n - 1)):
// the whole-hull scan's arithmetic and tie rule (first maximal vertex), without a memory access per support
DEV float4 hull_support_reg(float4 v, int idx, float n0, float n1, float n2) {
  float best = -__builtin_inff(), bx = 0.f, by = 0.f, bz = 0.f;
  int bi = 0x7fffffff;
  const float sc = sup_score(n0, n1, n2, v.x, v.y, v.z);
  if (sc > best) { best = sc; bi = idx; bx = v.x; by = v.y; bz = v.z; }
  arg_best16<false>(best, bi, bx, by, bz);
  return make_float4(bx, by, bz, __int_as_float(bi));
}
#endif
DEV void mpr_support(const DevModel* __restrict__ m, const MprObj& o, const float* d, MprSup& s, int lane) {
  uint32_t id = 0u;
#pragma unroll
  for (int t = 0; t < 3; t++) s.v1[t] = o.c[t];
  if (o.hull1 < 0) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const float l = o.ax[i] * d[0] + o.ax[3 + i] * d[1] + o.ax[6 + i] * d[2];
      const float sz = l >= 0.f ? o.h[i] : -o.h[i];
      id |= l >= 0.f ? 1u << i : 0u;
#pragma unroll
      for (int t = 0; t < 3; t++) s.v1[t] += sz * o.ax[3 * t + i];
    }
  } else {
    // obj1 hull: the direction into its body frame, its support back into H
    float dl[3], w[3];
    mulmtv3(dl, o.ax, d);
    const float4 v = hull_support(m, o.cells, o.hull1, o.s1, o.n1, dl[0], dl[1], dl[2], lane);
    const float vv[3] = {v.x, v.y, v.z};
    id = (uint32_t)__float_as_int(v.w);
    mulmv3(w, o.ax, vv);
#pragma unroll
    for (int t = 0; t < 3; t++) s.v1[t] += w[t];
  }
#if SO100_SMALL_HULL_REG
  const float4 v = o.n <= kLanes ? hull_support_reg(o.v2r, min(lane, o.n - 1), -d[0], -d[1], -d[2])
                                 : hull_support(m, o.cells, o.k, o.s0, o.n, -d[0], -d[1], -d[2], lane);
#else
  const float4 v = hull_support(m, o.cells, o.k, o.s0, o.n, -d[0], -d[1], -d[2], lane);
#endif
  s.v2[0] = v.x; s.v2[1] = v.y; s.v2[2] = v.z;
  s.id = id | (uint32_t)__float_as_int(v.w) << 10;
  sub3(s.v, s.v1, s.v2);
}
// the support point of mpr_support with these ids, rebuilt by the same arithmetic (bitwise the same point)
DEV void sup_from_id(const DevModel* __restrict__ m, const MprObj& o, uint32_t id, MprSup& s) {
#pragma unroll
  for (int t = 0; t < 3; t++) s.v1[t] = o.c[t];
  if (o.hull1 < 0) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const float sz = (id >> i) & 1u ? o.h[i] : -o.h[i];
#pragma unroll
      for (int t = 0; t < 3; t++) s.v1[t] += sz * o.ax[3 * t + i];
    }
  } else {
    const float4 hv = reinterpret_cast<const float4*>(m->hull_vert)[o.s1 + (int)(id & 1023u)];
    const float vv[3] = {hv.x, hv.y, hv.z};
    float w[3];
    mulmv3(w, o.ax, vv);
#pragma unroll
    for (int t = 0; t < 3; t++) s.v1[t] += w[t];
  }
  const float4 v2 = reinterpret_cast<const float4*>(m->hull_vert)[o.s0 + (int)((id >> 10) & 1023u)];
  s.v2[0] = v2.x; s.v2[1] = v2.y; s.v2[2] = v2.z;
  s.id = id;
  sub3(s.v, s.v1, s.v2);
}
DEV void portal_dir(const MprSup* P, float* dir) {
  float a[3], b[3];
  sub3(a, P[2].v, P[1].v);
  sub3(b, P[3].v, P[1].v);
  cross3(dir, a, b);
  normalize3(dir);
}
DEV bool portal_reach_tol(const MprSup* P, const MprSup& v4, const float* dir) {
  const float d4 = dot3(v4.v, dir);
  float d1 = d4 - dot3(P[1].v, dir);
  const float d2 = d4 - dot3(P[2].v, dir), d3 = d4 - dot3(P[3].v, dir);
  d1 = d1 < d2 ? d1 : d2;
  d1 = d1 < d3 ? d1 : d3;
  return ccd_eq(d1, kMprTol) || d1 < kMprTol;
}
DEV void portal_expand(MprSup* P, const MprSup& v4) {
  float v4v0[3];
  cross3(v4v0, v4.v, P[0].v);
  const bool a = dot3(P[1].v, v4v0) > 0.f, b = dot3(P[2].v, v4v0) > 0.f, c = dot3(P[3].v, v4v0) > 0.f;
  sup_sel(P[1], v4, a ? b : !c);
  sup_sel(P[2], v4, !a && c);
  sup_sel(P[3], v4, a && !b);
}
// -1: no intersection, 0: portal, 1: touching on v1, 2: origin on the segment v0-v1
DEV int mpr_discover(const DevModel* __restrict__ m, const MprObj& o, MprSup* P, int lane) {
#pragma unroll
  for (int t = 0; t < 3; t++) { P[0].v1[t] = o.c1[t]; P[0].v2[t] = o.hc[t]; }
  sub3(P[0].v, P[0].v1, P[0].v2);
  if (ccd_zero(P[0].v[0]) && ccd_zero(P[0].v[1]) && ccd_zero(P[0].v[2])) P[0].v[0] += kCcdEps * 10.f;
  float dir[3] = {-P[0].v[0], -P[0].v[1], -P[0].v[2]}, va[3], vb[3];
  normalize3(dir);
  mpr_support(m, o, dir, P[1], lane);
  float dt = dot3(P[1].v, dir);
  if (ccd_zero(dt) || dt < 0.f) return -1;
  cross3(dir, P[0].v, P[1].v);
  if (ccd_zero(dot3(dir, dir))) return (ccd_zero(P[1].v[0]) && ccd_zero(P[1].v[1]) && ccd_zero(P[1].v[2])) ? 1 : 2;
  normalize3(dir);
  mpr_support(m, o, dir, P[2], lane);
  dt = dot3(P[2].v, dir);
  if (ccd_zero(dt) || dt < 0.f) return -1;
  sub3(va, P[1].v, P[0].v);
  sub3(vb, P[2].v, P[0].v);
  cross3(dir, va, vb);
  normalize3(dir);
  {
    const bool sw = dot3(dir, P[0].v) > 0.f;
    const MprSup t = P[1];
    sup_sel(P[1], P[2], sw);
    sup_sel(P[2], t, sw);
    const float sg = sw ? -1.f : 1.f;
    dir[0] *= sg; dir[1] *= sg; dir[2] *= sg;
  }
  for (int it = 0; it < kMprIters; it++) {
    mpr_support(m, o, dir, P[3], lane);
    dt = dot3(P[3].v, dir);
    if (ccd_zero(dt) || dt < 0.f) return -1;
    cross3(va, P[1].v, P[3].v);
    dt = dot3(va, P[0].v);
    const bool c1 = dt < 0.f && !ccd_zero(dt);
    cross3(va, P[3].v, P[2].v);
    dt = dot3(va, P[0].v);
    const bool c2 = !c1 && dt < 0.f && !ccd_zero(dt);     // tested against the unchanged v2, as libccd
    sup_sel(P[2], P[3], c1);
    sup_sel(P[1], P[3], c2);
    if (!c1 && !c2) return 0;
    sub3(va, P[1].v, P[0].v);
    sub3(vb, P[2].v, P[0].v);
    cross3(dir, va, vb);
    normalize3(dir);
  }
  return -1;
}
DEV float seg_dist2(const float* x0, const float* b, float* w) {
  float dd[3];
  sub3(dd, b, x0);
  float t = -dot3(x0, dd);
  t /= dot3(dd, dd);
  if (t < 0.f || ccd_zero(t)) { w[0] = x0[0]; w[1] = x0[1]; w[2] = x0[2]; }
  else if (t > 1.f || ccd_eq(t, 1.f)) { w[0] = b[0]; w[1] = b[1]; w[2] = b[2]; }
  else {
#pragma unroll
    for (int k = 0; k < 3; k++) w[k] = dd[k] * t + x0[k];
  }
  return dot3(w, w);
}
// ccdVec3PointTriDist2 of the origin, with the witness point
DEV float tri_dist2(const float* x0, const float* B, const float* C, float* w) {
  float d1[3], d2[3];
  sub3(d1, B, x0);
  sub3(d2, C, x0);
  const float v = dot3(d1, d1), ww = dot3(d2, d2), p = dot3(x0, d1), q = dot3(x0, d2), r = dot3(d1, d2);
  const float det = ww * v - r * r;
  float s, t;
  if (ccd_zero(det)) { s = -1.f; t = -1.f; }
  else { s = (q * r - ww * p) / det; t = (-s * r - q) / ww; }
  if ((ccd_zero(s) || s > 0.f) && (ccd_eq(s, 1.f) || s < 1.f) && (ccd_zero(t) || t > 0.f) &&
      (ccd_eq(t, 1.f) || t < 1.f) && (ccd_eq(t + s, 1.f) || t + s < 1.f)) {
#pragma unroll
    for (int k = 0; k < 3; k++) w[k] = x0[k] + d1[k] * s + d2[k] * t;
    return dot3(w, w);
  }
  float w2[3];
  float dist = seg_dist2(x0, B, w);
  float d2b = seg_dist2(x0, C, w2);
  if (d2b < dist) { dist = d2b; w[0] = w2[0]; w[1] = w2[1]; w[2] = w2[2]; }
  d2b = seg_dist2(B, C, w2);
  if (d2b < dist) { dist = d2b; w[0] = w2[0]; w[1] = w2[1]; w[2] = w2[2]; }
  return dist;
}
DEV void mpr_find_pos(const MprSup* P, float* pos) {
  float dir[3], vec[3], b[4];
  portal_dir(P, dir);
  cross3(vec, P[1].v, P[2].v); b[0] = dot3(vec, P[3].v);
  cross3(vec, P[3].v, P[2].v); b[1] = dot3(vec, P[0].v);
  cross3(vec, P[0].v, P[1].v); b[2] = dot3(vec, P[3].v);
  cross3(vec, P[2].v, P[1].v); b[3] = dot3(vec, P[0].v);
  float sum = b[0] + b[1] + b[2] + b[3];
  if (ccd_zero(sum) || sum < 0.f) {
    b[0] = 0.f;
    cross3(vec, P[2].v, P[3].v); b[1] = dot3(vec, dir);
    cross3(vec, P[3].v, P[1].v); b[2] = dot3(vec, dir);
    cross3(vec, P[1].v, P[2].v); b[3] = dot3(vec, dir);
    sum = b[1] + b[2] + b[3];
  }
  const float inv = 1.f / sum;
  float p1[3] = {0.f, 0.f, 0.f}, p2[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int t = 0; t < 3; t++) { p1[t] += P[i].v1[t] * b[i]; p2[t] += P[i].v2[t] * b[i]; }
#pragma unroll
  for (int t = 0; t < 3; t++) pos[t] = 0.5f * (p1[t] * inv + p2[t] * inv);
}
// ccdMPRPenetration: true and (depth, dir box -> hull, pos) on intersection with a defined normal
DEV bool mpr_penetration(const DevModel* __restrict__ m, const MprObj& o, float& depth, float* dir, float* pos,
                         int lane) {
  MprSup P[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
#pragma unroll
    for (int t = 0; t < 3; t++) { P[i].v[t] = 0.f; P[i].v1[t] = 0.f; P[i].v2[t] = 0.f; }
    P[i].id = 0u;
  }
  const int res = mpr_discover(m, o, P, lane);
  if (res < 0 || res == 1) return false;
  if (res == 2) {
#pragma unroll
    for (int t = 0; t < 3; t++) { pos[t] = 0.5f * (P[1].v1[t] + P[1].v2[t]); dir[t] = P[1].v[t]; }
    depth = sqrtf(dot3(dir, dir));
    if (ccd_zero(depth)) return false;
    normalize3(dir);
    return true;
  }
  // refine the portal until it holds the origin
  for (int it = 0;; it++) {
    if (it >= kMprIters) return false;
    float pd[3];
    portal_dir(P, pd);
    float dt = dot3(pd, P[1].v);
    if (ccd_zero(dt) || dt > 0.f) break;
    MprSup v4;
    mpr_support(m, o, pd, v4, lane);
    dt = dot3(v4.v, pd);
    if (!(ccd_zero(dt) || dt > 0.f) || portal_reach_tol(P, v4, pd)) return false;
    portal_expand(P, v4);
  }
  // penetration: expand towards the boundary until the tolerance (or the iteration cap)
  for (int it = 0;; it++) {
    float pd[3];
    portal_dir(P, pd);
    MprSup v4;
    mpr_support(m, o, pd, v4, lane);
    if (portal_reach_tol(P, v4, pd) || it > kMprIters) break;
    portal_expand(P, v4);
  }
  depth = sqrtf(tri_dist2(P[1].v, P[2].v, P[3].v, dir));
  if (ccd_zero(depth)) return false;
  normalize3(dir);
  mpr_find_pos(P, pos);
  return true;
}

// ------------------------------------------------------------------ mesh pairs: GJK + EPA (oracle epa_penetration)
// MuJoCo 3.3.3's default convex collider (native mjc_ccd): GJK decides the overlap and leaves a tetrahedron of
// Minkowski-difference support points around the origin; EPA grows it to the facet of A - B nearest the origin:
// the minimum penetration (depth, normal geom1 -> geom2), witness points from the origin's projection on that
// facet, one contact at their midpoint.  Row-redundant like MPR: every lane of the row runs the same scalar
// path on bitwise-identical values; the hull supports, the facet scans and the horizon are lane-parallel
// (lane l owns facet slots l, l + 16, l + 32: visibility, its edges' twin test against the visible facets,
// and the new facets on its horizon edges, ranked by row ballots).  The simplex lives in registers (constant
// slot indices, selects); the polytope in LDS, in the row's env's contact area (ConSlot con[kMaxCon], dead
// while the narrowphase runs): kEpaMaxF facet planes + vertex triples and kEpaMaxV vertex support ids; the
// vertex points in registers across the row (EpaVerts).
constexpr int kEpaMaxV = 24, kEpaMaxF = 44, kEpaMaxE = 48;   // oracle EPA_MAXV / EPA_MAXF / EPA_MAXE
// Diagnostic build only (-DSO100_EPA_STAMPS, tools/dev/epa_stamps.py): shader cycles of the convex collider's
// phases summed over the rows (lane 0) into a device counter array read by so100_dev_epa_cycles.
#ifdef SO100_EPA_STAMPS
__device__ unsigned long long so100_epa_cyc[12];  // GJK, EPA, items, EPA items, EPA iters, support, horizon+facets, scan,
                                                   // then inside the horizon: visibility + twins, masks, facets
#define ESTAMP_T() __builtin_amdgcn_s_memtime()
#define ESTAMP_ADD(k, v) do { if (lane == 0) atomicAdd(&so100_epa_cyc[k], (unsigned long long)(v)); } while (0)
#else
#define ESTAMP_T() 0ull
#define ESTAMP_ADD(k, v) do { (void)(v); } while (0)
#endif
struct EpaPoly {
  float4 plane[kEpaMaxF];           // outward normal, distance from the origin
  uint32_t fv[kEpaMaxF];            // vertex indices v0 | v1 << 5 | v2 << 10
  uint32_t vid[kEpaMaxV];           // the vertices' support ids (sup_from_id)
};
static_assert(sizeof(EpaPoly) <= sizeof(ConSlot) * kMaxCon, "an EPA polytope fits an env's contact area");

// A GJK simplex point: the Minkowski-difference point and its support ids (EPA starts from these; the witness
// points of EPA's final facet are rebuilt from the ids, sup_from_id), 4 registers per point instead of 10.
struct GjkPt {
  float v[3];
  uint32_t id;
};
DEV void pt_sel(GjkPt& d, const GjkPt& s, bool w) {
#pragma unroll
  for (int t = 0; t < 3; t++) d.v[t] = w ? s.v[t] : d.v[t];
  d.id = w ? s.id : d.id;
}

// the simplex part nearest the origin and the next search direction (oracle gjk_simplex); true when the
// tetrahedron S[0..3] encloses the origin.  S[n - 1] is the newest point.
DEV bool gjk_simplex(GjkPt* S, int& n, float* d) {
  if (n == 4) {                                   // A = S[3], B = S[2], C = S[1], D = S[0]
    float ao[3], ab[3], ac[3], ad[3], nabc[3], nacd[3], nadb[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      ao[k] = -S[3].v[k]; ab[k] = S[2].v[k] - S[3].v[k]; ac[k] = S[1].v[k] - S[3].v[k]; ad[k] = S[0].v[k] - S[3].v[k];
    }
    cross3(nabc, ab, ac);
    cross3(nacd, ac, ad);
    cross3(nadb, ad, ab);
    const float s1 = dot3(nabc, ad) > 0.f ? -1.f : 1.f, s2 = dot3(nacd, ab) > 0.f ? -1.f : 1.f;
    const float s3 = dot3(nadb, ac) > 0.f ? -1.f : 1.f;
#pragma unroll
    for (int k = 0; k < 3; k++) { nabc[k] *= s1; nacd[k] *= s2; nadb[k] *= s3; }
    const bool f1 = dot3(nabc, ao) > 0.f;
    const bool f2 = !f1 && dot3(nacd, ao) > 0.f;
    const bool f3 = !f1 && !f2 && dot3(nadb, ao) > 0.f;
    if (!f1 && !f2 && !f3) return true;
    const GjkPt t0 = S[0], t1 = S[1], t2 = S[2], t3 = S[3];
    // f1: (C, B, A); f2: (D, C, A); f3: (B, D, A)
    pt_sel(S[0], t1, f1); pt_sel(S[0], t2, f3);
    pt_sel(S[1], t2, f1); pt_sel(S[1], t0, f3);
    pt_sel(S[2], t3, true);
    n = 3;
  }
  if (n == 3) {                                   // A = S[2], B = S[1], C = S[0]
    float ao[3], ab[3], ac[3], abc[3], e1[3], e2[3];
#pragma unroll
    for (int k = 0; k < 3; k++) { ao[k] = -S[2].v[k]; ab[k] = S[1].v[k] - S[2].v[k]; ac[k] = S[0].v[k] - S[2].v[k]; }
    cross3(abc, ab, ac);
    cross3(e1, abc, ac);
    cross3(e2, ab, abc);
    const bool ce = dot3(e1, ao) > 0.f;
    const bool c_ac = ce && dot3(ac, ao) > 0.f;
    const bool ab_region = (ce && !c_ac) || (!ce && dot3(e2, ao) > 0.f);
    const bool c_ab = ab_region && dot3(ab, ao) > 0.f;
    const bool c_pt = ab_region && !c_ab;
    const bool face = !ce && !ab_region;
    const bool above = face && dot3(abc, ao) > 0.f;
    float t[3], dac[3], dab[3];
    cross3(t, ac, ao);
    cross3(dac, t, ac);
    cross3(t, ab, ao);
    cross3(dab, t, ab);
#pragma unroll
    for (int k = 0; k < 3; k++) d[k] = c_ac ? dac[k] : c_ab ? dab[k] : c_pt ? ao[k] : above ? abc[k] : -abc[k];
    const GjkPt t0 = S[0], t1 = S[1], t2 = S[2];
    // c_ac: (C, A); c_ab: (B, A); c_pt: (A); below: (B, C, A)
    pt_sel(S[0], t1, c_ab || (face && !above));
    pt_sel(S[0], t2, c_pt);
    pt_sel(S[1], t2, c_ac || c_ab);
    pt_sel(S[1], t0, face && !above);
    n = (c_ac || c_ab) ? 2 : c_pt ? 1 : 3;
    return false;
  }
  // line: A = S[1], B = S[0]
  float ao[3], ab[3], t[3], dl[3];
#pragma unroll
  for (int k = 0; k < 3; k++) { ao[k] = -S[1].v[k]; ab[k] = S[0].v[k] - S[1].v[k]; }
  const bool seg = dot3(ab, ao) > 0.f;
  cross3(t, ab, ao);
  cross3(dl, t, ab);
#pragma unroll
  for (int k = 0; k < 3; k++) d[k] = seg ? dl[k] : ao[k];
  const GjkPt t1 = S[1];
  pt_sel(S[0], t1, !seg);
  n = seg ? 2 : 1;
  return false;
}

// GJK (oracle gjk): true when A - B encloses the origin, S then holds the enclosing tetrahedron
DEV bool gjk_enclose(const DevModel* __restrict__ m, const MprObj& o, GjkPt* S, int lane) {
  float d[3];
#pragma unroll
  for (int k = 0; k < 3; k++) d[k] = o.hc[k] - o.c1[k];
  if (ccd_zero(dot3(d, d))) d[0] = 1.f;
  int n = 0;
  for (int it = 0; it < kMprIters; it++) {
    const float dd = dot3(d, d);
    if (dd < kCcdEps * kCcdEps) return false;       // ccd_zero(|d|)
    const float ind = __builtin_amdgcn_rsqf(dd);    // 1 / |d| (oracle gjk: one division), v_rsq
    const float du[3] = {d[0] * ind, d[1] * ind, d[2] * ind};
    MprSup as;
    mpr_support(m, o, du, as, lane);
    GjkPt a;
#pragma unroll
    for (int k = 0; k < 3; k++) a.v[k] = as.v[k];
    a.id = as.id;
    if (dot3(a.v, du) <= 0.f) return false;
#pragma unroll
    for (int k = 0; k < 4; k++) pt_sel(S[k], a, n == k);
    n++;
    if (n > 1 && gjk_simplex(S, n, d)) return true;
    if (n == 1) { d[0] = -a.v[0]; d[1] = -a.v[1]; d[2] = -a.v[2]; }
  }
  return false;
}

// a facet (a, b, c) of the polytope into slot f (oracle epa_face_set); false for a degenerate triangle
DEV bool epa_face_set(EpaPoly& P, int f, int a, int b, int c, const float* A, const float* B, const float* C) {
  float ab[3], ac[3], n[3];
  sub3(ab, B, A);
  sub3(ac, C, A);
  cross3(n, ab, ac);
  const float l2 = dot3(n, n);
  if (l2 < kCcdEps * kCcdEps) return false;       // ccd_zero(|n|)
  const float il = __builtin_amdgcn_rsqf(l2);     // 1 / |n| (oracle epa_face_set: one division), v_rsq
  n[0] = n[0] * il; n[1] = n[1] * il; n[2] = n[2] * il;
  P.plane[f] = make_float4(n[0], n[1], n[2], dot3(n, A));
  P.fv[f] = (uint32_t)a | (uint32_t)b << 5 | (uint32_t)c << 10;
  return true;
}

// The polytope's vertex positions (the Minkowski-difference points) across the row's lanes: vertex i on lane
// i & 15, slot i >> 4 (kEpaMaxV <= 32): the lanes building new facets fetch their vertices by row shuffles
// instead of dependent global loads of the supports (sup_from_id): bitwise the same points.
struct EpaVerts {
  float x[2], y[2], z[2];
};
DEV void everts_set(EpaVerts& V, int i, const float* v, int lane) {
  const bool mine = (i & 15) == lane;
#pragma unroll
  for (int s = 0; s < 2; s++) {
    const bool w = mine && (i >> 4) == s;
    V.x[s] = w ? v[0] : V.x[s];
    V.y[s] = w ? v[1] : V.y[s];
    V.z[s] = w ? v[2] : V.z[s];
  }
}

// EPA from GJK's tetrahedron (oracle epa_penetration, the same bookkeeping order): true and (depth, dir
// geom1 -> geom2, pos) on the facet reached.  P: the row's LDS polytope; lane: 0..15 in the row.
DEV bool epa_penetration(const DevModel* __restrict__ m, const MprObj& o, const GjkPt* S, float& depth, float* dir,
                         float* pos, EpaPoly& P, int lane, int grp) {
  uint64_t alive = 0ull;                        // live facet slots (row-uniform)
  // the initial tetrahedron: faces (0,1,2), (0,3,1), (0,2,3), (1,3,2), each outward (away from the 4th vertex)
  {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int a = i < 3 ? 0 : 1;
      int b = i == 0 ? 1 : i == 1 ? 3 : i == 2 ? 2 : 3;
      int c = i == 0 ? 2 : i == 1 ? 1 : i == 2 ? 3 : 2;
      const int e = 6 - a - b - c;
      GjkPt A = S[0], B = S[0], C = S[0], E = S[0];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        pt_sel(A, S[k], a == k); pt_sel(B, S[k], b == k); pt_sel(C, S[k], c == k); pt_sel(E, S[k], e == k);
      }
      float ab[3], ac[3], ae[3], n[3];
      sub3(ab, B.v, A.v);
      sub3(ac, C.v, A.v);
      sub3(ae, E.v, A.v);
      cross3(n, ab, ac);
      const bool flip = dot3(n, ae) > 0.f;
      const GjkPt Bt = B;
      pt_sel(B, C, flip);
      pt_sel(C, Bt, flip);
      const int bb = flip ? c : b, cc = flip ? b : c;
      ok = ok && epa_face_set(P, i, a, bb, cc, A.v, B.v, C.v);
      alive |= 1ull << i;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) P.vid[k] = S[k].id;
    if (!ok) return false;
  }
  EpaVerts V;
#pragma unroll
  for (int s = 0; s < 2; s++) { V.x[s] = 0.f; V.y[s] = 0.f; V.z[s] = 0.f; }
#pragma unroll
  for (int k = 0; k < 4; k++) everts_set(V, k, S[k].v, lane);
  int nv = 4, best = -1;
  float bn[3] = {0.f, 0.f, 0.f}, bd = 0.f;
  for (int it = 0; it < kMprIters; it++) {
    // the nearest live facet: lanes scan slots lane, lane + 16, lane + 32, then a row (dist, slot) min
    const unsigned long long et0 = ESTAMP_T();
    ESTAMP_ADD(4, 1);
    float dmin = __builtin_inff(), nx = 0.f, ny = 0.f, nz = 0.f;
    int fmin = 0x7fffffff;
#pragma unroll
    for (int s3 = 0; s3 < 3; s3++) {
      const int f = lane + kLanes * s3;
      if (f < kEpaMaxF && ((alive >> f) & 1ull)) {
        const float4 pl = P.plane[f];
        if (pl.w < dmin) { dmin = pl.w; fmin = f; nx = pl.x; ny = pl.y; nz = pl.z; }
      }
    }
    arg_best16<true>(dmin, fmin, nx, ny, nz);
    if (fmin == 0x7fffffff) return false;
    best = fmin; bd = dmin; bn[0] = nx; bn[1] = ny; bn[2] = nz;
    MprSup w;
    const unsigned long long et1 = ESTAMP_T();
    mpr_support(m, o, bn, w, lane);
    const float gain = dot3(w.v, bn) - bd;
    const unsigned long long et2 = ESTAMP_T();
    ESTAMP_ADD(7, et1 - et0);
    ESTAMP_ADD(5, et2 - et1);
    if (gain < kMprTol || nv >= kEpaMaxV) break;
    // the facets that see w (lane-parallel): lane l tests slots l, l + 16, l + 32; vis is the row-uniform mask
    uint64_t vis = 0ull;
    bool mv[3];
    uint32_t mfv[3];
#pragma unroll
    for (int s3 = 0; s3 < 3; s3++) {
      const int f = lane + kLanes * s3;
      mv[s3] = false;
      mfv[s3] = 0u;
      if (f < kEpaMaxF && ((alive >> f) & 1ull)) {
        const float4 pl = P.plane[f];
        mv[s3] = (pl.x * w.v[0] + pl.y * w.v[1] + pl.z * w.v[2]) - pl.w > 0.f;
        mfv[s3] = P.fv[f];
      }
      vis |= ((__ballot(mv[s3]) >> (grp * kLanes)) & 0xFFFFull) << (kLanes * s3);
    }
    // the horizon: the edges (a, b) of the visible facets whose twin (b, a) lies on no visible facet, in
    // (slot, edge) order (oracle epa_penetration).  Each lane holds its visible slots' 3 edges; one pass over
    // the visible facets (their vertex triples broadcast from LDS) marks the lanes' edges that have a twin.
    const unsigned long long eh0 = ESTAMP_T();
    uint32_t twin = 0u;                          // bit 3 s3 + k: edge k of the lane's slot s3 has a twin
    for (uint64_t vm = vis; vm != 0ull; vm &= vm - 1ull) {
      const uint32_t g = P.fv[__builtin_ctzll(vm)];
      const uint32_t g0 = g & 31u, g1 = (g >> 5) & 31u, g2 = (g >> 10) & 31u;
      // g's directed edges reversed: (g1, g0), (g2, g1), (g0, g2) as a | b << 5
      const uint32_t r0 = g1 | g0 << 5, r1 = g2 | g1 << 5, r2 = g0 | g2 << 5;
#pragma unroll
      for (int s3 = 0; s3 < 3; s3++)
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const uint32_t a = (mfv[s3] >> (5 * k)) & 31u, bb = (mfv[s3] >> (5 * ((k + 1) % 3))) & 31u;
          const uint32_t key = a | bb << 5;
          twin |= (mv[s3] && (key == r0 || key == r1 || key == r2)) ? 1u << (3 * s3 + k) : 0u;
        }
    }
    // horizon masks per (slot group, edge): bit l = edge k of slot l + 16 s3
    uint32_t hm[3][3];
    int ne = 0;
#pragma unroll
    for (int s3 = 0; s3 < 3; s3++)
#pragma unroll
      for (int k = 0; k < 3; k++) {
        hm[s3][k] = (uint32_t)((__ballot(mv[s3] && !((twin >> (3 * s3 + k)) & 1u)) >> (grp * kLanes)) & 0xFFFFull);
        ne += __popc(hm[s3][k]);
      }
    const unsigned long long eh1 = ESTAMP_T();
    ESTAMP_ADD(8, eh1 - eh0);
    if (ne > kEpaMaxE) break;                      // the horizon does not fit: stop at the nearest facet
    alive &= ~vis;
    const int iw = nv;
    P.vid[nv] = w.id;
    everts_set(V, nv, w.v, lane);
    nv++;
    // the new facets (a, b, w), one per horizon edge, built by the lanes that own the edges: the j-th
    // non-degenerate one (in horizon order) takes the j-th lowest free slot; slots run out -> the rest none
    const unsigned long long eh2 = ESTAMP_T();
    ESTAMP_ADD(9, eh2 - eh1);
    const uint64_t freem = ~alive & ((1ull << kEpaMaxF) - 1ull);
    const int nfree = __popcll(freem);
    const uint32_t below = (1u << lane) - 1u;
    int nvalid = 0;                               // non-degenerate facets so far (earlier slot groups)
#pragma unroll
    for (int s3 = 0; s3 < 3; s3++) {
      const uint32_t any = hm[s3][0] | hm[s3][1] | hm[s3][2];
      if (__ballot(any != 0u) == 0ull) continue;  // wave-uniform: no horizon edge in this slot group
      float pv[3][3];
#pragma unroll
      for (int q = 0; q < 3; q++) {
        const int vi = (int)((mfv[s3] >> (5 * q)) & 31u);
        const int src = vi & 15;
        const float x0 = __shfl(V.x[0], src, kLanes), x1 = __shfl(V.x[1], src, kLanes);
        const float y0 = __shfl(V.y[0], src, kLanes), y1 = __shfl(V.y[1], src, kLanes);
        const float z0 = __shfl(V.z[0], src, kLanes), z1 = __shfl(V.z[1], src, kLanes);
        pv[q][0] = vi >= 16 ? x1 : x0; pv[q][1] = vi >= 16 ? y1 : y0; pv[q][2] = vi >= 16 ? z1 : z0;
      }
      float4 fpl[3];
      uint32_t ok = 0u;                           // bit k: the lane's edge k makes a non-degenerate facet
#pragma unroll
      for (int k = 0; k < 3; k++) {
        fpl[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((hm[s3][k] >> lane) & 1u) {
          const float* A = pv[k];
          const float* B = pv[(k + 1) % 3];
          float ab[3], ac[3], n[3];
          sub3(ab, B, A);
          sub3(ac, w.v, A);
          cross3(n, ab, ac);
          const float l2 = dot3(n, n);
          if (!(l2 < kCcdEps * kCcdEps)) {
            const float il = __builtin_amdgcn_rsqf(l2);
            n[0] = n[0] * il; n[1] = n[1] * il; n[2] = n[2] * il;
            fpl[k] = make_float4(n[0], n[1], n[2], dot3(n, A));
            ok |= 1u << k;
          }
        }
      }
      // rank in (slot, edge) order among the non-degenerate facets: earlier groups, lower lanes, lower edges
      int lo = 0, cnt = 0;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const uint32_t mk = (uint32_t)((__ballot((ok >> k) & 1u) >> (grp * kLanes)) & 0xFFFFull);
        lo += __popc(mk & below);
        cnt += __popc(mk);
      }
      int rk = nvalid + lo;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        if ((ok >> k) & 1u) {
          if (rk < nfree) {
            uint64_t fm = freem;
            for (int t = 0; t < rk; t++) fm &= fm - 1ull;
            const int slot = __builtin_ctzll(fm);
            const uint32_t a = (mfv[s3] >> (5 * k)) & 31u, bb = (mfv[s3] >> (5 * ((k + 1) % 3))) & 31u;
            P.plane[slot] = fpl[k];
            P.fv[slot] = a | bb << 5 | (uint32_t)iw << 10;
          }
          rk++;
        }
      }
      nvalid += cnt;
    }
    {                                             // alive |= the lowest min(nvalid, nfree) free slots
      uint64_t fm = freem, taken = 0ull;
      for (int t = 0; t < nvalid && fm != 0ull; t++) {
        const uint64_t bit = fm & (~fm + 1ull);
        taken |= bit;
        fm ^= bit;
      }
      alive |= taken;
    }
    const unsigned long long eh3 = ESTAMP_T();
    ESTAMP_ADD(10, eh3 - eh2);
    ESTAMP_ADD(6, eh3 - et2);
  }
  if (best < 0) return false;
  depth = bd;
  if (ccd_zero(depth) || depth < 0.f) return false;
  // witness points: barycentric coordinates of the origin's projection p = n dist on the facet
  const uint32_t fv = P.fv[best];
  MprSup A, B, C;
  sup_from_id(m, o, P.vid[fv & 31u], A);
  sup_from_id(m, o, P.vid[(fv >> 5) & 31u], B);
  sup_from_id(m, o, P.vid[(fv >> 10) & 31u], C);
  const float p[3] = {bn[0] * bd, bn[1] * bd, bn[2] * bd};
  float l0, l1, l2;
  {
    float v0[3], v1[3], v2[3];
    sub3(v0, B.v, A.v); sub3(v1, C.v, A.v); sub3(v2, p, A.v);
    const float d00 = dot3(v0, v0), d01 = dot3(v0, v1), d11 = dot3(v1, v1), d20 = dot3(v2, v0), d21 = dot3(v2, v1);
    const float den = d00 * d11 - d01 * d01;
    if (ccd_zero(den)) { l0 = 1.f; l1 = 0.f; l2 = 0.f; }
    else { l1 = (d11 * d20 - d01 * d21) / den; l2 = (d00 * d21 - d01 * d20) / den; l0 = 1.f - l1 - l2; }
  }
#pragma unroll
  for (int t = 0; t < 3; t++) {
    float w1 = 0.f, w2 = 0.f;
    w1 += l0 * A.v1[t]; w2 += l0 * A.v2[t];
    w1 += l1 * B.v1[t]; w2 += l1 * B.v2[t];
    w1 += l2 * C.v1[t]; w2 += l2 * C.v2[t];
    pos[t] = 0.5f * (w1 + w2);
    dir[t] = bn[t];
  }
  return true;
}

// the mesh pairs' collider of the model (so100_model.convex): GJK + EPA (MuJoCo 3.3.3's default) or MPR
DEV bool convex_penetration(const DevModel* __restrict__ m, const MprObj& o, float& depth, float* dir, float* pos,
                            EpaPoly& P, int lane, int grp) {
  if (m->convex == SO100_CONVEX_MPR) return mpr_penetration(m, o, depth, dir, pos, lane);
  GjkPt S[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
#pragma unroll
    for (int t = 0; t < 3; t++) S[i].v[t] = 0.f;
    S[i].id = 0u;
  }
  const unsigned long long gt0 = ESTAMP_T();
  ESTAMP_ADD(2, 1);
  const bool enc = gjk_enclose(m, o, S, lane);
  const unsigned long long gt1 = ESTAMP_T();
  ESTAMP_ADD(0, gt1 - gt0);
  if (!enc) return false;
  ESTAMP_ADD(3, 1);
  const bool hit = epa_penetration(m, o, S, depth, dir, pos, P, lane, grp);
  ESTAMP_ADD(1, ESTAMP_T() - gt1);
  return hit;
}

// world frame of a hull's body: an arm link (bodies 2..7, fk_stage's frames in LDS) or the static Base
// (body 1, hull SO100_HULL_BASE)
DEV void hull_frame(const DevModel* __restrict__ m, const EnvShared& sh, int b, float* R, float* P) {
  if (b == 1) {
#pragma unroll
    for (int t = 0; t < 9; t++) R[t] = m->base_xmat[t];
#pragma unroll
    for (int t = 0; t < 3; t++) P[t] = m->base_xpos[t];
  } else {
    const int a = b - 2;
#pragma unroll
    for (int t = 0; t < 9; t++) R[t] = sh.ser.xm[a][t];
#pragma unroll
    for (int t = 0; t < 3; t++) P[t] = sh.ser.xp[a][t];
  }
}

// Convex pair p (23..142): obj1 = box geom (cube, bin box, finger pad) or hull k1 (self-collision, the Base), obj2 = hull k, both
// in hull k's body frame H.  Oracle collision().
DEV void mpr_obj_setup(const DevModel* __restrict__ m, const EnvShared& sh, int p, MprObj& o) {
  const int g = m->pair_g1[p], k = -1 - m->pair_g2[p];
  float RH[9], pH[3];
  hull_frame(m, sh, m->hull_body[k], RH, pH);
  float pb[3], Rb[9];
  if (g == SO100_CUBE_GEOM) {
#pragma unroll
    for (int t = 0; t < 3; t++) pb[t] = sh.cube_pos[t];
#pragma unroll
    for (int t = 0; t < 9; t++) Rb[t] = sh.cube_mat[t];
  } else if (g >= 0 && m->geom_body[g] == 0) {       // a bin box (static)
#pragma unroll
    for (int t = 0; t < 3; t++) pb[t] = m->geom_pos[g][t];
#pragma unroll
    for (int t = 0; t < 9; t++) Rb[t] = m->geom_mat[g][t];
  } else if (g >= 0) {                               // a finger pad on a jaw (pad / link-hull pairs)
    geom_pose(m, sh, g, pb, Rb);
  } else {
    hull_frame(m, sh, m->hull_body[-1 - g], Rb, pb);
  }
  float dp[3];
  sub3(dp, pb, pH);
  mulmtv3(o.c, RH, dp);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int jj = 0; jj < 3; jj++) o.ax[3 * i + jj] = RH[i] * Rb[jj] + RH[3 + i] * Rb[3 + jj] + RH[6 + i] * Rb[6 + jj];
  o.hull1 = g >= 0 ? -1 : -1 - g;
  if (g >= 0) {
#pragma unroll
    for (int t = 0; t < 3; t++) { o.h[t] = m->geom_size[g][t]; o.c1[t] = o.c[t]; o.bc[t] = o.c[t]; o.bh[t] = o.h[t]; }
    o.s1 = 0; o.n1 = 0;
  } else {
    const int k1 = o.hull1;
    const float4 c4 = reinterpret_cast<const float4*>(m->hull_centroid)[k1];
    const float4 b4 = reinterpret_cast<const float4*>(m->hull_center)[k1];
    const float4 h4 = reinterpret_cast<const float4*>(m->hull_half)[k1];
    const float cl[3] = {c4.x, c4.y, c4.z}, bl[3] = {b4.x, b4.y, b4.z};
    float t1[3], t2[3];
    mulmv3(t1, o.ax, cl);
    mulmv3(t2, o.ax, bl);
#pragma unroll
    for (int t = 0; t < 3; t++) { o.h[t] = 0.f; o.c1[t] = t1[t] + o.c[t]; o.bc[t] = t2[t] + o.c[t]; }
    o.bh[0] = h4.x; o.bh[1] = h4.y; o.bh[2] = h4.z;
    o.s1 = m->hull_start[k1];
    o.n1 = m->hull_count[k1];
  }
  const float4 hc = reinterpret_cast<const float4*>(m->hull_centroid)[k];
  o.hc[0] = hc.x; o.hc[1] = hc.y; o.hc[2] = hc.z;
  o.k = k;
  o.cells = false;
  o.s0 = m->hull_start[k];
  o.n = m->hull_count[k];
}
// conservative broadphase, stage 1 (oracle mpr_broadphase): bounding spheres in the world frame: obj1's
// centre (box centre / hull box centre) against hull k's box centre; radii precomputed (hull_half.w,
// |half sizes| of a box)
DEV bool mpr_sphere(const DevModel* __restrict__ m, const EnvShared& sh, int p) {
  const int g = m->pair_g1[p], k = -1 - m->pair_g2[p];
  float RH[9], pH[3];
  hull_frame(m, sh, m->hull_body[k], RH, pH);
  const float4 hb4 = reinterpret_cast<const float4*>(m->hull_center)[k];
  const float hb[3] = {hb4.x, hb4.y, hb4.z};
  float w[3], c1[3], r1;
  mulmv3(w, RH, hb);
  if (g == SO100_CUBE_GEOM) {
#pragma unroll
    for (int t = 0; t < 3; t++) c1[t] = sh.cube_pos[t];
    r1 = m->geom_rbound[g];
  } else if (g >= 0 && m->geom_body[g] == 0) {       // a bin box
#pragma unroll
    for (int t = 0; t < 3; t++) c1[t] = m->geom_pos[g][t];
    r1 = m->geom_rbound[g];
  } else if (g >= 0) {                               // a finger pad on a jaw
    float Rp[9];
    geom_pose(m, sh, g, c1, Rp);
    r1 = m->geom_rbound[g];
  } else {
    const int k1 = -1 - g;
    float R1[9], P1[3];
    hull_frame(m, sh, m->hull_body[k1], R1, P1);
    const float4 b4 = reinterpret_cast<const float4*>(m->hull_center)[k1];
    const float bl[3] = {b4.x, b4.y, b4.z};
    float t1[3];
    mulmv3(t1, R1, bl);
#pragma unroll
    for (int t = 0; t < 3; t++) c1[t] = t1[t] + P1[t];
    r1 = reinterpret_cast<const float4*>(m->hull_half)[k1].w;
  }
  float T[3];
#pragma unroll
  for (int t = 0; t < 3; t++) T[t] = c1[t] - (w[t] + pH[t]);
  const float rs = reinterpret_cast<const float4*>(m->hull_half)[k].w + r1;
  return dot3(T, T) <= rs * rs;
}
// stage 2: OBB-OBB separating axes in H (hull k's box vs the box)
DEV bool mpr_broadphase(const DevModel* __restrict__ m, const MprObj& o, int k) {
  const float4 hb4 = reinterpret_cast<const float4*>(m->hull_center)[k];
  const float4 hh4 = reinterpret_cast<const float4*>(m->hull_half)[k];
  const float hb[3] = {hb4.x, hb4.y, hb4.z}, hh[3] = {hh4.x, hh4.y, hh4.z};
  float T[3];
  sub3(T, o.bc, hb);
  float A[9];
#pragma unroll
  for (int i = 0; i < 9; i++) A[i] = fabsf(o.ax[i]) + 1e-5f;
#pragma unroll
  for (int i = 0; i < 3; i++)
    if (fabsf(T[i]) > hh[i] + o.bh[0] * A[3 * i] + o.bh[1] * A[3 * i + 1] + o.bh[2] * A[3 * i + 2]) return false;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const float s = T[0] * o.ax[j] + T[1] * o.ax[3 + j] + T[2] * o.ax[6 + j];
    if (fabsf(s) > hh[0] * A[j] + hh[1] * A[3 + j] + hh[2] * A[6 + j] + o.bh[j]) return false;
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      const float ra = hh[i1] * A[3 * i2 + j] + hh[i2] * A[3 * i1 + j];
      const float rb = o.bh[j1] * A[3 * i + j2] + o.bh[j2] * A[3 * i + j1];
      const float s = T[i2] * o.ax[3 * i1 + j] - T[i1] * o.ax[3 * i2 + j];
      if (fabsf(s) > ra + rb) return false;
    }
  }
  return true;
}

// Broadphase bounding spheres (oracle mpr_broadphase stage 1), one per collision object: hull k at k (< 10,
// the Base hull at 9), geom g (1..14: pads, cube, bin boxes) at 9 + g.  World centre (hull: its bounding box
// centre; box: its centre) and radius (hull_half.w / geom_rbound), by the arithmetic mpr_sphere uses.
constexpr int kSphObj = SO100_NHULL_ALL + SO100_NGEOM - 1;   // 24
DEV float4 sphere_obj(const DevModel* __restrict__ m, const EnvShared& sh, int o) {
  float c[3], r;
  if (o < SO100_NHULL_ALL) {
    float R[9], P[3], w[3];
    hull_frame(m, sh, m->hull_body[o], R, P);
    const float4 b4 = reinterpret_cast<const float4*>(m->hull_center)[o];
    const float bl[3] = {b4.x, b4.y, b4.z};
    mulmv3(w, R, bl);
#pragma unroll
    for (int t = 0; t < 3; t++) c[t] = w[t] + P[t];
    r = reinterpret_cast<const float4*>(m->hull_half)[o].w;
  } else {
    const int g = o - (SO100_NHULL_ALL - 1);
    if (g == SO100_CUBE_GEOM) {
#pragma unroll
      for (int t = 0; t < 3; t++) c[t] = sh.cube_pos[t];
    } else if (m->geom_body[g] == 0) {               // a bin box (static)
#pragma unroll
      for (int t = 0; t < 3; t++) c[t] = m->geom_pos[g][t];
    } else {                                         // a finger pad on a jaw
      float Rp[9];
      geom_pose(m, sh, g, c, Rp);
    }
    r = m->geom_rbound[g];
  }
  return make_float4(c[0], c[1], c[2], r);
}

// The MPR pairs 23..142 of one substep ((cube | bin box, hull), hull-hull self-collision, the Base hull, the
// finger pads vs the arm's link hulls),
// contacts staged in sh.mpr in pair order.
//  * broadphase stage 1, bounding spheres: lane l of the env's row computes objects l and l + 16 of the
//    env's sphere table (sphere_obj, in its MPR staging area, dead until the narrowphase's hits), then tests
//    pairs 23 + l + 16 r (r < 8) by two table reads each; the survivors form a wave-wide list (env by env,
//    pairs ascending);
//  * broadphase stage 2, OBB separating axes (mpr_broadphase), one list item per lane of the wave (64 per
//    batch; round 2 ran both stages on the env's own row, 8 rounds of 16 pairs, each round paying the sphere
//    and OBB paths of every pair class: 28 % of the average wave's assembly); the OBB survivors go to their
//    env's candidate list in pair order;
//  * narrowphase, shared across the wave: the 4 envs' candidates form one list (env by env, pairs ascending,
//    in the LDS contact area of env 0, dead until the compaction); each round the 4 rows take the next 4
//    items, whichever env they belong to, and run MPR on that env's frames.  A wave whose envs hold c_e
//    candidates runs ceil(sum c_e / 4) rounds: the envs' own rows share a heavy env's pairs (this was one
//    pair of the wave's union per round, on the rows holding it: 60 % of the slowest waves' assembly);
//  * each round's hits go to their env's staging slots in list order, so each env keeps its pair order.
// The candidate lists are the pairs passing both stages, in pair order, as before: the same contacts.
// Returns the env's number of MPR contacts (uniform across its row; those beyond kMaxCon are not staged and
// count as dropped).
template <bool kCells>
DEV int mpr_contacts(const DevModel* __restrict__ m, EnvShared* shm, int lane, int grp, bool valid) {
#ifdef SO100_EXPERIMENT_NO_MPR
  return 0;   // timing experiment only: box-hull contacts off
#endif
#ifdef SO100_NO_PADLINK
  constexpr int kConvex = SO100_NPAIR_CONVEX - SO100_NPAIR_PADLINK;   // A/B diagnostic builds only
#else
  constexpr int kConvex = SO100_NPAIR_CONVEX;
#endif
  constexpr int kRounds = (kConvex + kLanes - 1) / kLanes;   // 8
  static_assert(kRounds <= 8, "candidate masks hold 128 pairs");
  // each env's candidates go to its dynamics scratch (RNE cdd + tau: dead from the collision on; the contact
  // area holds the rows' EPA polytopes)
  static_assert(kConvex <= (int)(sizeof(shm[0].ser.cdd) + sizeof(shm[0].ser.tau)), "an env's candidate list fits");
  static_assert(__builtin_offsetof(SerialScratch, cdd) >= sizeof(ConArea), "the candidate lists do not alias the contact area");
  // the sphere table and the sphere survivors' list in the env's MPR staging area
  static_assert(kSphObj * sizeof(float4) + kConvex <= sizeof(shm[0].mpr), "sphere table + list fit the staging area");
  const EnvShared& sh = shm[grp];
  {
    float4* tab = reinterpret_cast<float4*>(&shm[grp].mpr[0]);
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
      const int o = lane + kLanes * pass;
      if (o < kSphObj) tab[o] = sphere_obj(m, sh, o);
    }
  }
  __syncthreads();
  uint64_t env_cand[2] = {0ull, 0ull};
  uint32_t mine = 0u;                           // bit r: this lane's pair of round r passes the spheres
  {
    const float4* tab = reinterpret_cast<const float4*>(&shm[grp].mpr[0]);
#pragma unroll
    for (int r = 0; r < kRounds; r++) {
      const int q = lane + kLanes * r;
      bool cand = false;
      if (valid && q < kConvex) {
        const int g = m->pair_g1[SO100_PAIR_MPR0 + q], k = -1 - m->pair_g2[SO100_PAIR_MPR0 + q];
        const float4 a = tab[g >= 0 ? SO100_NHULL_ALL - 1 + g : -1 - g], b = tab[k];
        const float T[3] = {a.x - b.x, a.y - b.y, a.z - b.z};
        const float rs = b.w + a.w;
        cand = dot3(T, T) <= rs * rs;
      }
      const uint64_t bl = __ballot(cand);
      mine |= cand ? 1u << r : 0u;
      env_cand[r / 4] |= ((bl >> (grp * 16)) & 0xFFFFull) << (16 * (r % 4));
    }
  }
  // the wave's list of sphere survivors: env e's at [spre_e, spre_e + s_e), in its own staging area
  const int scnt = __popcll(env_cand[0]) + __popcll(env_cand[1]);
  const int s0c = __builtin_amdgcn_readlane(scnt, 0), s1c = __builtin_amdgcn_readlane(scnt, 16);
  const int s2c = __builtin_amdgcn_readlane(scnt, 32), s3c = __builtin_amdgcn_readlane(scnt, 48);
  const int spre1 = s0c, spre2 = s0c + s1c, spre3 = s0c + s1c + s2c, stotal = spre3 + s3c;
  if (stotal == 0) return 0;
  {
    uint8_t* slist = reinterpret_cast<uint8_t*>(&shm[grp].mpr[0]) + kSphObj * sizeof(float4);
#pragma unroll
    for (int r = 0; r < kRounds; r++) {
      if ((mine >> r) & 1u) {
        const int q = lane + kLanes * r;     // rank = sphere survivors of this env below pair q
        const uint64_t below0 = q >= 64 ? env_cand[0] : (env_cand[0] & ((1ull << q) - 1ull));
        const uint64_t below1 = q >= 64 ? (env_cand[1] & ((1ull << (q - 64)) - 1ull)) : 0ull;
        slist[__popcll(below0) + __popcll(below1)] = (uint8_t)q;
      }
    }
  }
  __syncthreads();
  // stage 2 over the survivors, one per lane of the wave; the OBB survivors to their env's list in order
  int c0 = 0, c1 = 0, c2 = 0, c3 = 0;           // candidates per env (wave-uniform)
  {
    const int tid = grp * kLanes + lane;
    const uint64_t below_me = (1ull << tid) - 1ull;
    for (int b0 = 0; b0 < stotal; b0 += kThreads) {
      const int item = b0 + tid;
      const bool act = item < stotal;
      const int ie = item >= spre3 ? 3 : item >= spre2 ? 2 : item >= spre1 ? 1 : 0;
      int q = 0;
      bool pass = false;
      if (act) {
        const int spre_ie = ie == 0 ? 0 : ie == 1 ? spre1 : ie == 2 ? spre2 : spre3;
        q = (reinterpret_cast<const uint8_t*>(&shm[ie].mpr[0]) + kSphObj * sizeof(float4))[item - spre_ie];
        MprObj o;
        mpr_obj_setup(m, shm[ie], SO100_PAIR_MPR0 + q, o);
        pass = mpr_broadphase(m, o, -1 - m->pair_g2[SO100_PAIR_MPR0 + q]);
      }
      const uint64_t pb = __ballot(pass);
      const uint64_t e0 = __ballot(act && ie == 0), e1 = __ballot(act && ie == 1);
      const uint64_t e2 = __ballot(act && ie == 2), e3 = __ballot(act && ie == 3);
      if (pass) {
        const uint64_t mie = ie == 0 ? e0 : ie == 1 ? e1 : ie == 2 ? e2 : e3;
        const int base = ie == 0 ? c0 : ie == 1 ? c1 : ie == 2 ? c2 : c3;
        reinterpret_cast<uint8_t*>(&shm[ie].ser.cdd[0][0])[base + __popcll(pb & mie & below_me)] = (uint8_t)q;
      }
      c0 += __popcll(pb & e0); c1 += __popcll(pb & e1); c2 += __popcll(pb & e2); c3 += __popcll(pb & e3);
    }
  }
  const int pre1 = c0, pre2 = c0 + c1, pre3 = c0 + c1 + c2;
  int total = pre3 + c3;
#ifdef SO100_EXPERIMENT_MPR_BROAD_ONLY
  asm volatile("" ::"v"(total));   // keeps the broadphase live
  total = 0;   // timing experiment only: broadphase without the narrowphase
#endif
  if (total == 0) return 0;
  __syncthreads();
  int f0 = 0, f1 = 0, f2 = 0, f3 = 0;           // staged contacts per env (wave-uniform)
  const int rounds = (total + kEnvsPerBlock - 1) / kEnvsPerBlock;
  auto env_of = [&](int item) { return item >= pre3 ? 3 : item >= pre2 ? 2 : item >= pre1 ? 1 : 0; };
  for (int rd = 0; rd < rounds; rd++) {
    const int item = kEnvsPerBlock * rd + grp;
    const bool act = item < total;
    const int ie = env_of(item);
    float depth = 0.f, dir[3] = {0.f, 0.f, 0.f}, pos[3] = {0.f, 0.f, 0.f};
    bool hit = false;
    int p = SO100_PAIR_MPR0;
    if (act) {
      const int pre_ie = ie == 0 ? 0 : ie == 1 ? pre1 : ie == 2 ? pre2 : pre3;
      p = SO100_PAIR_MPR0 + reinterpret_cast<const uint8_t*>(&shm[ie].ser.cdd[0][0])[item - pre_ie];
      MprObj o;
      mpr_obj_setup(m, shm[ie], p, o);
      o.cells = kCells;
#if SO100_SMALL_HULL_REG
      o.v2r = o.n <= kLanes ? ld_global4(reinterpret_cast<const float4*>(m->hull_vert), o.s0 + min(lane, o.n - 1))
                            : make_float4(0.f, 0.f, 0.f, 0.f);
#endif
      hit = convex_penetration(m, o, depth, dir, pos, *reinterpret_cast<EpaPoly*>(&shm[grp].con[0]), lane, grp);
    }
    // this round's hits, row g at bit 16 g; rows earlier in the list with the same env come first
    const uint64_t hb = __ballot(hit);
    int slot = ie == 0 ? f0 : ie == 1 ? f1 : ie == 2 ? f2 : f3;
#pragma unroll
    for (int g = 0; g < kEnvsPerBlock; g++) {
      const int it = kEnvsPerBlock * rd + g;
      const bool h = it < total && ((hb >> (16 * g)) & 1ull);
      if (g < grp && h && env_of(it) == ie) slot++;
    }
    if (hit && lane == 0 && slot < kMaxCon) {
      const int k = -1 - m->pair_g2[p];
      float RH[9], pH[3], wn[3], wp[3];
      hull_frame(m, shm[ie], m->hull_body[k], RH, pH);
      mulmv3(wn, RH, dir);
      mulmv3(wp, RH, pos);
      MprStage& st = shm[ie].mpr[slot];
      st.pos[0] = wp[0] + pH[0]; st.pos[1] = wp[1] + pH[1];
      st.pos[2] = wp[2] + pH[2]; st.pos[3] = -depth;
      st.nrm[0] = wn[0]; st.nrm[1] = wn[1]; st.nrm[2] = wn[2];
      st.nrm[3] = __int_as_float(p);
    }
#pragma unroll
    for (int g = 0; g < kEnvsPerBlock; g++) {
      const int it = kEnvsPerBlock * rd + g;
      if (it < total && ((hb >> (16 * g)) & 1ull)) {
        const int e = env_of(it);
        f0 += e == 0; f1 += e == 1; f2 += e == 2; f3 += e == 3;
      }
    }
  }
  return grp == 0 ? f0 : grp == 1 ? f1 : grp == 2 ? f2 : f3;
}

// the contact frame (oracle make_frame; MuJoCo mju_makeFrame): the two normalisations by v_rsq (1 ulp)
DEV void make_frame(float* f) {
  float* n = f;
  float* t1 = f + 3;
  const float in = __builtin_amdgcn_rsqf(dot3(n, n));
  n[0] *= in; n[1] *= in; n[2] *= in;
  if (fabsf(n[1]) < 0.5f) { t1[0] = 0.f; t1[1] = 1.f; t1[2] = 0.f; }
  else { t1[0] = 0.f; t1[1] = 0.f; t1[2] = 1.f; }
  float pr = dot3(n, t1);
  t1[0] -= pr * n[0]; t1[1] -= pr * n[1]; t1[2] -= pr * n[2];
  const float it = __builtin_amdgcn_rsqf(dot3(t1, t1));
  t1[0] *= it; t1[1] *= it; t1[2] *= it;
  cross3(f + 6, n, t1);
}

// (M^-1 J')[dof] for the 4 rows of a contact: arm dofs use the dense 6x6 M^-1 row (row broadcasts of
// the other arm lanes' J), cube dofs the diagonal inverse mass.
DEV float4 minv_times(float4 J, const float* minv_row, float invmc, int lane) {
  float4 acc = make_float4(J.x * invmc, J.y * invmc, J.z * invmc, J.w * invmc);
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const float4 Jj = bcast_row4(J, j);
    acc.x += minv_row[j] * Jj.x; acc.y += minv_row[j] * Jj.y;
    acc.z += minv_row[j] * Jj.z; acc.w += minv_row[j] * Jj.w;
  }
  return acc;
}

// contact c's Jacobian column for dof `lane` (rows: normal, t1, t2 on the point velocity; torsion on
// the angular velocity); J = frame . (jac(body of geom2) - jac(body of geom1)) at the contact point
DEV float4 contact_jac(const DevModel* __restrict__ m, const EnvShared& sh, int c, int lane) {
  const int p = sh.con_pair[c];
  const float* cp = sh.con[c].g.pos;
  const float* fr = sh.con[c].g.frame;
  float jp[3] = {0, 0, 0}, jr[3] = {0, 0, 0};
#pragma unroll
  for (int side = 0; side < 2; side++) {
    const int b = side ? m->pair_b2[p] : m->pair_b1[p];
    const float sg = side ? 1.f : -1.f;
    if (lane < 6) {
      if (b >= 2 && b <= 7 && lane + 2 <= b) {
        float off[3] = {cp[0] - sh.anchor[lane][0], cp[1] - sh.anchor[lane][1], cp[2] - sh.anchor[lane][2]};
        float v[3];
        cross3(v, sh.axis[lane], off);
#pragma unroll
        for (int t = 0; t < 3; t++) { jp[t] += sg * v[t]; jr[t] += sg * sh.axis[lane][t]; }
      }
    } else if (b == SO100_CUBE_BODY) {
      if (lane < 9) {
        jp[lane - 6] += sg;
      } else {
        const int k = lane - 9;
        float ax[3] = {sh.cube_mat[k], sh.cube_mat[3 + k], sh.cube_mat[6 + k]};
        float off[3] = {cp[0] - sh.cube_pos[0], cp[1] - sh.cube_pos[1], cp[2] - sh.cube_pos[2]};
        float v[3];
        cross3(v, ax, off);
#pragma unroll
        for (int t = 0; t < 3; t++) { jp[t] += sg * v[t]; jr[t] += sg * ax[t]; }
      }
    }
  }
  // condim 3 (hull-table): no torsion row.  A zero 4th row makes the 4-row block exactly the condim-3
  // block: its A row/column is R3 on the diagonal only, the eigen-component it adds to the QCQP carries
  // c = w = 0, and its force stays 0 (so100_pgs.hip)
  const float jt = m->pair_cond4[p] ? fr[0] * jr[0] + fr[1] * jr[1] + fr[2] * jr[2] : 0.f;
  return make_float4(fr[0] * jp[0] + fr[1] * jp[1] + fr[2] * jp[2], fr[3] * jp[0] + fr[4] * jp[1] + fr[5] * jp[2],
                     fr[6] * jp[0] + fr[7] * jp[1] + fr[8] * jp[2], jt);
}

// Symmetric 3x3 eigen-decomposition by cyclic Jacobi (5 sweeps: quadratic convergence reaches fp32
// round-off for 3x3): A = Q diag(lam) Q', columns of Q are the eigenvectors.
DEV void eig3_sym(const float A0[3][3], float lam[3], float Q[3][3]) {
  float a[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) { a[i][j] = A0[i][j]; Q[i][j] = (i == j) ? 1.f : 0.f; }
#pragma unroll
  for (int sweep = 0; sweep < 5; sweep++) {
#pragma unroll
    for (int pq = 0; pq < 3; pq++) {
      const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
      const float apq = a[p][q];
      if (fabsf(apq) > 1e-30f) {
        // hardware rcp / sqrt / rsq (~1 ulp): each rotation stays orthogonal to fp32 precision and the
        // cyclic sweeps correct any residual, at a fraction of the IEEE division / sqrt sequences
        const float theta = (a[q][q] - a[p][p]) * __builtin_amdgcn_rcpf(2.f * apq);
        const float t = copysignf(__builtin_amdgcn_rcpf(fabsf(theta) + __builtin_amdgcn_sqrtf(theta * theta + 1.f)), theta);
        const float c = __builtin_amdgcn_rsqf(t * t + 1.f), sn = t * c;
#pragma unroll
        for (int k = 0; k < 3; k++) {           // columns p, q
          const float akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - sn * akq;
          a[k][q] = sn * akp + c * akq;
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {           // rows p, q
          const float apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - sn * aqk;
          a[q][k] = sn * apk + c * aqk;
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const float qkp = Q[k][p], qkq = Q[k][q];
          Q[k][p] = c * qkp - sn * qkq;
          Q[k][q] = sn * qkp + c * qkq;
        }
      }
    }
  }
  lam[0] = a[0][0]; lam[1] = a[1][1]; lam[2] = a[2][2];
}

// ------------------------------------------------------------------ the step kernel
struct StageArgs {
  const DevModel* m;
  so100_buffers b;
  Workspace w;
  int n;
  int task;
  int flags;
  int max_steps;
  uint64_t base_seed;
  int env_offset;
  int sub;             // substep index (kMode 2: nsubstep)
  int par;             // substep parity (heavy-group list set)
};

DEV int wave_max_i(int v) {
  // max over the wave (all 4 lane groups); result uniform
  v = max(v, __shfl_xor(v, 16));
  v = max(v, __shfl_xor(v, 32));
  return __builtin_amdgcn_readfirstlane(v);
}

// reset one env (lane-group cooperative): arm start pose, cube spawn, zero velocity/warmstart
DEV void env_reset_state(const DevModel* __restrict__ m, EnvShared& sh, int lane, uint32_t seed, float& qpos_r,
                         float& qvel_r, float& warm_r, double* pose_out) {
  double pose[7];
  spawn_pose(m, seed, pose);
  if (pose_out) {
#pragma unroll
    for (int k = 0; k < 7; k++) pose_out[k] = pose[k];
  }
  float v = 0.f;
  if (lane < 6) v = m->start_qpos[lane];
#pragma unroll
  for (int k = 0; k < 7; k++) if (lane == 6 + k) v = (float)pose[k];
  qpos_r = v;
  qvel_r = 0.f;
  warm_r = 0.f;
}

// obs row: box(3) bin(3) ee(3) qpos[:6] — env.py:137-145.  qv = qpos[lane-9] gathered by the caller
// (bcast16 in uniform control flow).
DEV void write_obs(const DevModel* __restrict__ m, const EnvShared& sh, int lane, float qv, float* dst) {
  float v = qv;
  if (lane < 3) v = sh.site_cube[lane];
  else if (lane < 6) v = m->bin_center_f[lane - 3];
  else if (lane < 9) v = sh.site_ee[lane - 6];
  if (lane < SO100_NOBS) dst[lane] = v;
}

// Diagnostic build only (-DSO100_STAGE_STAMPS): per-phase cycle attribution of the stage kernel
// (substep nsubstep-1, mode 1), written to debug[88..93] (SSTAMP_RAW, DSTAMP: top of this file).
#ifdef SO100_STAGE_STAMPS
#define SSTAMP_DECL unsigned long long sst_prev_ = 0, sst_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#ifdef SO100_DYN_STAMPS
#define SSTAMP(slot) SSTAMP_RAW(-1)
#else
#define SSTAMP(slot) SSTAMP_RAW(slot)
#endif
#else
#define SSTAMP_DECL
#define SSTAMP(slot) do {} while (0)
#endif

// Euler (mj_Euler) of the previous substep on the state held in registers: qvel += h qacc, then qpos
// with the new qvel; the cube quaternion by the exponential map (lanes 9..12, staged through LDS).
DEV void euler_update(EnvShared& sh, int lane, float h, float qacc, float& qpos_r, float& qvel_r) {
  if (lane < SO100_NV) qvel_r += h * qacc;
  if (lane < 9) qpos_r += h * qvel_r;
  if (lane >= 9 && lane < 12) sh.vec[lane] = qvel_r;
  if (lane >= 9 && lane < 13) sh.qpos[lane] = qpos_r;
  __syncthreads();
  if (lane >= 9 && lane < 13) {
    float q[4] = {sh.qpos[9], sh.qpos[10], sh.qpos[11], sh.qpos[12]};
    float w[3] = {sh.vec[9], sh.vec[10], sh.vec[11]};
    float nw = sqrtf(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (nw > kMinVal) {
      float s, c;
      sincosf(0.5f * h * nw, &s, &c);
      const float rn = __builtin_amdgcn_rcpf(nw);
      float qr[4] = {c, w[0] * rn * s, w[1] * rn * s, w[2] * rn * s};
      quat_mul(q, q, qr);
    }
    quat_normalize(q);
    qpos_r = q[lane - 9];
  }
  __syncthreads();
}

// write one box-box pair's contacts into slots base, base+1, ... (slots >= kMaxCon are dropped, as the
// oracle's add_contact drops contacts beyond SO100_MAXCON)
DEV void put_box_contacts(EnvShared& sh, const PairContacts& pc, int base, int p) {
  // one frame per pair (every contact of a box pair shares its normal)
  float fr[9] = {pc.normal[0], pc.normal[1], pc.normal[2], 0, 0, 0, 0, 0, 0};
  if (pc.n > 0) make_frame(fr);
#pragma unroll
  for (int c = 0; c < SO100_MAXCONPAIR; c++) {
    const int slot = base + c;
    if (c < pc.n && slot < kMaxCon) {
#pragma unroll
      for (int t = 0; t < 9; t++) sh.con[slot].g.frame[t] = fr[t];
      sh.con[slot].g.pos[0] = pc.pos[c][0]; sh.con[slot].g.pos[1] = pc.pos[c][1];
      sh.con[slot].g.pos[2] = pc.pos[c][2]; sh.con[slot].g.pos[3] = pc.dist[c];
      sh.con_dist[slot] = pc.dist[c];
      sh.con_pair[slot] = p;
    }
  }
}

// Finger pads vs the table and the bin boxes (oracle collision(): pad_table, collide_box_pair).
//   pairs 98..105 (pad i, table), lane i: the hull-table rule on the pad's 8 corners — the corners inside
//     the top face's footprint and below the top count; one contact at the deepest corner's distance, at
//     the counted corners' x-y centroid, midway in z between the deepest corner and the top; normal -z;
//   pairs 106..145 (pad i, bin box j): a conservative test (the pad's bounding sphere against the static
//     box, 3 pairs per lane), the candidates compacted in pair order and run through the box-box
//     collider 16 at a time (a wave runs as many rounds as its busiest env needs; usually none).
// Contacts are appended after `tot` in pair order; returns the new total.
DEV int pad_contacts(const DevModel* __restrict__ m, EnvShared& sh, int lane, int grp, bool valid, int tot) {
#ifdef SO100_NO_PADS
  return tot;                             // A/B diagnostic builds only (tests/_build_variant.sh)
#endif
  // ---- pad-table (lanes 0..7)
  bool tfound = false, nearbin = false;
  float tx = 0.f, ty = 0.f, tz = 0.f;
  if (valid && lane < SO100_NPAD) {
    const int p = SO100_PAIR_PAD0 + lane, g = m->pair_g1[p];
    const int b = m->pair_b1[p];                  // = geom_body[g] (so100_create), loaded beside g
    const float* bm = sh.jaw_mat[b - 6];
    const float* gm = m->geom_mat[g];
    const float top = m->table_top, margin = m->pair_margin[p];
    float pc[3];
    mulmv3(pc, bm, m->geom_pos[g]);
#pragma unroll
    for (int k = 0; k < 3; k++) pc[k] += sh.jaw_pos[b - 6][k];
    // pad-bin prefilter: the pad's bounding sphere against the bin's AABB
    float bmarg = 0.f;
#pragma unroll
    for (int j = 0; j < SO100_NBINBOX; j++) bmarg = fmaxf(bmarg, m->pair_margin[SO100_PAIR_PADBIN0 + SO100_NBINBOX * lane + j]);
    float ex2 = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float u = fmaxf(m->bin_lo[k] - pc[k], pc[k] - m->bin_hi[k]);
      ex2 += u > 0.f ? u * u : 0.f;
    }
    const float rb = m->geom_rbound[g] + bmarg;
    nearbin = ex2 <= rb * rb;
    // table broadphase: the pad's lowest point (centre z minus its half-extent along world z)
    const float cz = pc[2];
    float ext = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) ext += fabsf(bm[6] * gm[k] + bm[7] * gm[3 + k] + bm[8] * gm[6 + k]) * m->geom_size[g][k];
    float sx = 0.f, sy = 0.f, zmin = 0.f;
    int cnt = 0;
    if (cz - ext - top < margin + 1e-4f) {
    float c[3], R[9];
    geom_pose_b(m, sh, g, b, c, R);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const float l0 = (k & 1 ? 1.f : -1.f) * m->geom_size[g][0];
      const float l1 = (k & 2 ? 1.f : -1.f) * m->geom_size[g][1];
      const float l2 = (k & 4 ? 1.f : -1.f) * m->geom_size[g][2];
      const float w0 = R[0] * l0 + R[1] * l1 + R[2] * l2 + c[0];
      const float w1 = R[3] * l0 + R[4] * l1 + R[5] * l2 + c[1];
      const float w2 = R[6] * l0 + R[7] * l1 + R[8] * l2 + c[2];
      const bool in = !(w0 < m->table_lo[0] || w0 > m->table_hi[0] || w1 < m->table_lo[1] || w1 > m->table_hi[1]) &&
                      (w2 - top < margin);
      if (in) {
        sx += w0; sy += w1;
        zmin = (cnt == 0 || w2 < zmin) ? w2 : zmin;
        cnt++;
      }
    }
    }
    tfound = cnt > 0;
    if (tfound) { tx = sx / (float)cnt; ty = sy / (float)cnt; tz = zmin; }
  }
  const uint32_t trow = (uint32_t)((__ballot(tfound) >> (grp * 16)) & 0xFFull);
  {
    const int slot = tot + __popc(trow & ((1u << lane) - 1u));
    if (tfound && slot < kMaxCon) {
      float fr[9] = {0.f, 0.f, -1.f, 0, 0, 0, 0, 0, 0};
      opaque(fr[2]);              // a constant frame: built here, not hoisted out of the fused substep loop
      make_frame(fr);
#pragma unroll
      for (int t = 0; t < 9; t++) sh.con[slot].g.frame[t] = fr[t];
      const float top = m->table_top;
      sh.con[slot].g.pos[0] = tx; sh.con[slot].g.pos[1] = ty;
      sh.con[slot].g.pos[2] = 0.5f * (tz + top); sh.con[slot].g.pos[3] = tz - top;
      sh.con_dist[slot] = tz - top;
      sh.con_pair[slot] = SO100_PAIR_PAD0 + lane;
    }
  }
  tot += __popc(trow);
  // ---- pad-bin candidates (3 pairs per lane); the whole wave skips them when no pad is near the bin
  if (__ballot(nearbin) == 0ull) return tot;
  uint64_t cm = 0ull;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int q = r * kLanes + lane;
    bool cand = false;
    if (valid && q < SO100_NPAIR_PADBIN) {
      const int p = SO100_PAIR_PADBIN0 + q;
      const int g1 = m->pair_g1[p], g2 = m->pair_g2[p];   // g1: a pad on a jaw; g2: static
      const int b = m->geom_body[g1];
      const float* bp = sh.jaw_pos[b - 6];
      const float* bm = sh.jaw_mat[b - 6];
      float t[3];
      mulmv3(t, bm, m->geom_pos[g1]);
      // the pad's bounding sphere against the static box itself: the distance from the pad centre to
      // the box, in the box frame
      const float w[3] = {bp[0] + t[0] - m->geom_pos[g2][0], bp[1] + t[1] - m->geom_pos[g2][1],
                          bp[2] + t[2] - m->geom_pos[g2][2]};
      const float* R2 = m->geom_mat[g2];
      float ex2 = 0.f;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const float u = fabsf(R2[k] * w[0] + R2[3 + k] * w[1] + R2[6 + k] * w[2]) - m->geom_size[g2][k];
        ex2 += u > 0.f ? u * u : 0.f;
      }
      const float rr = m->geom_rbound[g1] + m->pair_margin[p];
      cand = ex2 <= rr * rr;
    }
    cm |= ((__ballot(cand) >> (grp * 16)) & 0xFFFFull) << (16 * r);
  }
  const int ncand = __popcll(cm);
  const int rounds = (wave_max_i(ncand) + kLanes - 1) / kLanes;
  for (int r = 0; r < rounds; r++) {
    const int idx = r * kLanes + lane;
    int p = -1;
    if (idx < ncand) {
      uint64_t x = cm;
      for (int k = 0; k < idx; k++) x &= x - 1ull;
      p = SO100_PAIR_PADBIN0 + __ffsll((unsigned long long)x) - 1;
    }
    PairContacts pc;
    pc.n = 0;
    if (p >= 0) collide_pair(m, sh, p, pc);
    sh.cnt[lane] = pc.n;
    __syncthreads();
    int off = 0, sum = 0;
#pragma unroll
    for (int k = 0; k < kLanes; k++) { const int c = sh.cnt[k]; off += (k < lane) ? c : 0; sum += c; }
    put_box_contacts(sh, pc, tot + off, p);
    tot += sum;
    __syncthreads();
  }
  return tot;
}

#ifndef SO100_STAGE_WAVES
#define SO100_STAGE_WAVES 3      // waves per SIMD the stage kernel's register budget is sized for
#endif

// prologue: the env's state -> registers (lane k: qpos[k], qvel[k], warmstart[k]), DR parameters, counters
DEV void load_state(const StageArgs& args, int lane, int e, float& qpos_r, float& qvel_r, float& warm_r, float& mscale,
                    float& fscale, float& sigma, int& elapsed0, uint32_t& episode0) {
  const so100_buffers& B = args.b;
  qpos_r = (lane < SO100_NQ) ? B.qpos[(size_t)e * SO100_NQ + lane] : 0.f;
  qvel_r = (lane < SO100_NV) ? B.qvel[(size_t)e * SO100_NV + lane] : 0.f;
  warm_r = (lane < SO100_NV) ? B.qacc_warmstart[(size_t)e * SO100_NV + lane] : 0.f;
  mscale = 1.f; fscale = 1.f; sigma = 0.f;
  if ((args.flags & SO100_FLAG_DR) && B.dr_params) {
    mscale = B.dr_params[(size_t)e * 4 + 0];
    fscale = B.dr_params[(size_t)e * 4 + 1];
    sigma = B.dr_params[(size_t)e * 4 + 2];
  }
  elapsed0 = B.elapsed ? B.elapsed[e] : 0;
  episode0 = B.episode ? B.episode[e] : 0u;
}

// control (the same every substep of the env step: elapsed/episode only change in the epilogue): the
// action (+ DR noise) un-normalised into sh.ctrl; the EE variant's mocap pose into sh.mocap
DEV void set_controls(const StageArgs& args, EnvShared& sh, int lane, int e, float sigma, int elapsed0, uint32_t episode0) {
  const DevModel* __restrict__ m = args.m;
  const so100_buffers& B = args.b;
  if (lane < 6) {
    float a = B.action[(size_t)e * 6 + lane];
    if (sigma > 0.f)
      a += sigma * hash_normal(splitmix64(args.base_seed ^ ((uint64_t)(e + args.env_offset) << 40) ^
                                          ((uint64_t)episode0 << 20) ^ (uint64_t)(elapsed0 * 8 + lane)));
    sh.ctrl[lane] = unnormalize_f32(a, m->action_lo[lane], m->action_hi[lane], m->action_span[lane]);
  }
  if (m->ee && lane < 7) sh.mocap[lane] = B.mocap ? B.mocap[(size_t)e * 7 + lane] : m->mocap0[lane];
}

// One substep's position/velocity stages and constraint assembly on the state in registers (after the
// previous substep's Euler): kinematics, CRBA/RNE, actuation, collision, the frictionloss / limit /
// contact rows.  Newton: the rows go to nr (kFused: kept in registers for newton_solve; split: stored to the
// HBM record); PGS: the solver record of so100_pgs_kernel.
template <int kSolver, bool kFused, bool kDebug = true, bool kBcastDyn = false>
DEV void assemble(const StageArgs& args, EnvShared& sh, int lane, int grp, int env, int e, bool valid, float qpos_r,
                  float qvel_r, float warm_r, float mscale, float fscale, int sub, NewtonRows& nr) {
  const DevModel* __restrict__ m = args.m;
  const so100_buffers& B = args.b;
  SSTAMP_DECL
  SSTAMP(-1);
    // ---------------- S1: stage state in LDS
    if (lane < SO100_NQ) sh.qpos[lane] = qpos_r;
    if (lane < SO100_NV) sh.qvel[lane] = qvel_r;
    __syncthreads();
    // ---------------- S2: serial kinematics / dynamics (lane 0 of each group)
    fk_par(m, sh, lane);
    __syncthreads();
    DSTAMP(1);
    dynamics_par<kBcastDyn>(m, sh, lane, mscale DSTAMP_ARGS);
    __syncthreads();
    DSTAMP(7);
    if constexpr (kSolver == SO100_SOLVER_NEWTON) {
      // the Newton solver works with M itself: arm rows from the CRBA scratch (which collision reuses),
      // the cube's diagonal masses
#pragma unroll
      for (int j = 0; j < 6; j++) nr.mrow[j] = lane < 6 ? sh.ser.M[lane][j] : 0.f;
      nr.mcd = 0.f;
      if (lane >= 6 && lane < 9) nr.mcd = m->cube_mass * mscale;
      else if (lane >= 9 && lane < SO100_NV) nr.mcd = m->cube_inertia[lane - 9] * mscale;
      if (!kFused && valid) newton_mass_store(args.w, e, lane, nr);   // split path: the record, now
    }
    SSTAMP(1);
    // ---------------- S3: collision: hulls vs the table (lane k = hull k), box-hull pairs by MPR
    // (staged in LDS), one box pair per lane; compaction in pair order (box pairs, table-hull pairs,
    // box-hull pairs)
    float hx, hy, hz;
    const bool hfound = hull_table(m, sh, lane, grp, valid, hx, hy, hz);
    const uint32_t hrow = (uint32_t)((__ballot(hfound) >> (grp * 16)) & 0xFFFFull);
    SSTAMP(6);
    const int nmpr = mpr_contacts<kFused || SO100_SPLIT_CELLS>(m, &sh - grp, lane, grp, valid);
    SSTAMP(7);
    PairContacts pc;
    pc.n = 0;
    if (lane < SO100_NPAIR_BOX) collide_pair(m, sh, lane, pc);
#ifdef SO100_STAMP_BOXBOX
    SSTAMP(0);            // stamps diagnostic: the box-box pairs alone in slot 0 (Euler's, empty in the stage kernel)
#endif
    sh.cnt[lane] = pc.n;
    __syncthreads();
    {
      int off = 0, tot = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) { int c = sh.cnt[k]; off += (k < lane) ? c : 0; tot += c; }
      put_box_contacts(sh, pc, off, lane);
      const int hslot = tot + __popc(hrow & ((1u << lane) - 1u));
      if (hfound && hslot < kMaxCon) {
        float fr[9] = {0.f, 0.f, 1.f, 0, 0, 0, 0, 0, 0};
        opaque(fr[2]);            // a constant frame: built here, not hoisted out of the fused substep loop
        make_frame(fr);
#pragma unroll
        for (int t = 0; t < 9; t++) sh.con[hslot].g.frame[t] = fr[t];
        const float top = m->table_top;
        sh.con[hslot].g.pos[0] = hx; sh.con[hslot].g.pos[1] = hy;
        sh.con[hslot].g.pos[2] = 0.5f * (hz + top); sh.con[hslot].g.pos[3] = hz - top;
        sh.con_dist[hslot] = hz - top;
        sh.con_pair[hslot] = SO100_NPAIR_BOX + lane;
      }
      tot += __popc(hrow);
      const int mslot = tot + lane;
      if (lane < nmpr && mslot < kMaxCon) {
        const MprStage st = sh.mpr[lane];
        float fr[9] = {st.nrm[0], st.nrm[1], st.nrm[2], 0, 0, 0, 0, 0, 0};
        make_frame(fr);
#pragma unroll
        for (int t = 0; t < 9; t++) sh.con[mslot].g.frame[t] = fr[t];
#pragma unroll
        for (int t = 0; t < 4; t++) sh.con[mslot].g.pos[t] = st.pos[t];
        sh.con_dist[mslot] = st.pos[3];
        sh.con_pair[mslot] = __float_as_int(st.nrm[3]);
      }
      tot += nmpr;
      __syncthreads();
      tot = pad_contacts(m, sh, lane, grp, valid, tot);
      const int drop = tot > kMaxCon ? tot - kMaxCon : 0;   // the oracle's ncon_dropped
      if (lane == 0) {
        sh.ncon = tot < kMaxCon ? tot : kMaxCon;
        if constexpr (kFused) sh.ndrop = (sub == 0 ? 0 : sh.ndrop) + drop;   // stored by the fused epilogue
      }
      if constexpr (!kFused) {
        if (valid && lane == 0 && B.ncon_dropped)
          B.ncon_dropped[env] = (sub == 0 ? 0u : B.ncon_dropped[env]) + (uint32_t)drop;
      }
    }
    __syncthreads();
    const int ncon = valid ? sh.ncon : 0;
    const int ncon_max = wave_max_i(ncon);
    SSTAMP(2);
    if (kSolver == SO100_SOLVER_PGS && lane == 0 && ncon > kResident) {
      // this env's solver group is heavy: list it once for first dispatch (so100_pgs.hip)
      const int g = env / kPgsEnvs, ngroups = (args.n + kPgsEnvs - 1) / kPgsEnvs;
      uint32_t* fl = args.w.gflag + args.par * ngroups + g;
      if (atomicOr(fl, 1u) == 0u) {
        const int idx = atomicAdd(args.w.hcount + args.par, 1);
        if (idx < kHeavyCap) args.w.hlist[args.par * kHeavyCap + idx] = g;
        else atomicOr(fl, 2u);
      }
    }
    float* const crec = args.w.con + (size_t)e * kMaxCon * kConRec;

    // ---------------- S4/S5: M^-1 rows, frictionloss and joint-limit rows (lane = dof)
    float minv_row[6];
#pragma unroll
    for (int j = 0; j < 6; j++) minv_row[j] = (lane < 6) ? sh.minv[lane][j] : 0.f;
    const float invmc = (lane >= 6 && lane < 12) ? sh.inv_mcube[lane - 6] : 0.f;
    const float qs_r = (lane < SO100_NV) ? sh.qacc_smooth[lane] : 0.f;
    const bool has_fr = lane < SO100_NV;
    const float fr_R = has_fr ? m->fr_R[lane] : 1.f;
    const float fr_fl = has_fr ? m->fr_floss[lane] : 0.f;
    const float fr_aref = -m->fr_B * qvel_r;
    float fr_f;
    {
      const float jar = warm_r - fr_aref;
      if (jar <= -fr_R * fr_fl) fr_f = fr_fl;
      else if (jar >= fr_R * fr_fl) fr_f = -fr_fl;
      else fr_f = -jar * __builtin_amdgcn_rcpf(fr_R);
      if (!has_fr) fr_f = 0.f;
    }
    float mdiag = invmc;
#pragma unroll
    for (int j = 0; j < 6; j++) mdiag = (lane == j) ? minv_row[j] : mdiag;
    bool lim_on = false;
    float lim_s = 0.f, lim_aref = 0.f, lim_R = 1.f, lim_f = 0.f;
    if (lane < 6) {
      const float dlo = qpos_r - m->jnt_lo[lane], dhi = m->jnt_hi[lane] - qpos_r;
      float dist = 0.f;
      if (dlo < 0.f) { lim_on = true; lim_s = 1.f; dist = dlo; }
      else if (dhi < 0.f) { lim_on = true; lim_s = -1.f; dist = dhi; }
      if (lim_on) {
        const float imp = getimpedance(m->lim_solimp, dist, 0.f);
        lim_R = fmaxf(kMinVal, (1.f - imp) * __builtin_amdgcn_rcpf(imp) * m->lim_invw[lane]);
        lim_aref = -m->lim_B * (lim_s * qvel_r) - m->lim_K * imp * dist;
        const float jar = lim_s * warm_r - lim_aref;
        lim_f = jar < 0.f ? -jar * __builtin_amdgcn_rcpf(lim_R) : 0.f;
      }
    }
    const uint64_t lim_mask = __ballot(lim_on && valid);
    float cost_part = 0.f;
    float phi = has_fr ? fr_f + (lim_on ? lim_s * lim_f : 0.f) : 0.f;
    if (has_fr) cost_part += 0.5f * fr_R * fr_f * fr_f + fr_f * (qs_r - fr_aref);
    if (lim_on) cost_part += 0.5f * lim_R * lim_f * lim_f + lim_f * (lim_s * qs_r - lim_aref);

    if constexpr (kSolver == SO100_SOLVER_NEWTON) {
      // ---------------- Newton rows (so100_newton.h): J (lane = dof) and J qvel (lane c keeps contact c's),
      // per contact aref, R and the cone coefficients, qacc_smooth, the warmstart, the frictionloss and
      // limit rows.  Fused: handed to newton_solve in registers; split: stored to the HBM record.
      float cVn[4] = {0.f, 0.f, 0.f, 0.f};
      float4 jhi[kJLds];          // fused: J of contacts kJReg.., to LDS once every contact_jac has run
#pragma unroll
      for (int c = 0; c < kMaxCon; c++) {
        if (c < kJReg) nr.J[c] = make_float4(0.f, 0.f, 0.f, 0.f);
        else jhi[c - kJReg] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c < ncon_max) {
          float4 J = make_float4(0.f, 0.f, 0.f, 0.f);
          if (c < ncon && lane < SO100_NV) {
            J = contact_jac(m, sh, c, lane);
            if constexpr (!kFused) reinterpret_cast<float4*>(crec + c * kConRec + kJOff)[lane] = J;
          }
          if constexpr (kFused) {
            if (c < kJReg) nr.J[c] = J;
            else jhi[c - kJReg] = J;
          }
          const bool mine = lane == c;
          const float v0 = rowsum16(J.x * qvel_r), v1 = rowsum16(J.y * qvel_r);
          const float v2 = rowsum16(J.z * qvel_r), v3 = rowsum16(J.w * qvel_r);
          cVn[0] = mine ? v0 : cVn[0]; cVn[1] = mine ? v1 : cVn[1];
          cVn[2] = mine ? v2 : cVn[2]; cVn[3] = mine ? v3 : cVn[3];
        }
      }
      if constexpr (kFused) {
        // the J rows of contacts kJReg.. go to the contact-geometry area of LDS, dead from here to the next
        // substep's collision (ConArea is exactly kJLds x 12 float4)
        static_assert(kJLds * SO100_NV * sizeof(float4) <= sizeof(ConArea), "the LDS J rows fit the contact area");
        float4* jx = reinterpret_cast<float4*>(&sh.con[0]);
        if (kJReg < ncon_max) {
          __syncthreads();
#pragma unroll
          for (int c = kJReg; c < kMaxCon; c++)
            if (c < ncon_max && lane < SO100_NV) jx[(c - kJReg) * SO100_NV + lane] = jhi[c - kJReg];
          __syncthreads();
        }
        nr.jx = jx;
      }
      SSTAMP(3);
      nr.c_aref = make_float4(0.f, 0.f, 0.f, 0.f);
      nr.c_R = make_float4(1.f, 1.f, 1.f, 1.f);
      nr.c_mu = make_float4(1.f, 1.f, 1.f, 0.f);
      if (lane < ncon) {
        const int p = sh.con_pair[lane];
        const float dist = sh.con_dist[lane];
        const float imp = getimpedance(m->pair_solimp[p], dist, m->pair_margin[p]);
        const float K = m->pair_K[p], Bd = m->pair_B[p];
        const float fs = m->pair_cube[p] ? fscale : 1.f;     // DR friction scale: cube pairs
        const float mu0 = m->pair_mu0[p] * fs, mu1 = m->pair_mu1[p] * fs;
        float R[4];
        // (reciprocals by v_rcp, the square root by v_sqrt: 1 ulp, on the contact's setup chain)
        R[0] = fmaxf(kMinVal, (1.f - imp) * __builtin_amdgcn_rcpf(imp) * m->pair_tran[p]);
        R[1] = R[0] * mu0 * mu0 * __builtin_amdgcn_rcpf(mu0 * mu0 * m->impratio);
        R[2] = R[1];
        R[3] = R[0] * mu0 * mu0 * __builtin_amdgcn_rcpf(mu1 * mu1 * m->impratio);
        nr.c_aref = make_float4(-Bd * cVn[0] - K * imp * (dist - m->pair_margin[p]), -Bd * cVn[1], -Bd * cVn[2], -Bd * cVn[3]);
        nr.c_R = make_float4(R[0], R[1], R[2], R[3]);
        nr.c_mu = make_float4(mu0 * __builtin_amdgcn_sqrtf(R[1] * __builtin_amdgcn_rcpf(R[0])), mu0, mu1, 0.f);
      }
      SSTAMP(4);
      nr.qs = lane < SO100_NV ? qs_r : 0.f;
      nr.warm = lane < SO100_NV ? warm_r : 0.f;
      nr.fr_aref = lane < SO100_NV ? fr_aref : 0.f;
      nr.lim_s = lim_on ? lim_s : 0.f;
      nr.lim_aref = lim_aref;
      nr.lim_R = lim_R;
      nr.ncon = ncon;
      if (valid) {
        if constexpr (!kFused) {
          newton_rows_store(args.w, e, lane, nr);
        } else {
          // the contact counter (so100_contact_count) reads the last substep's count from the record
          if (lane == 0 && sub == m->nsubstep - 1) args.w.hdr[(size_t)e * kHdrEnv + H_NCON] = __int_as_float(ncon);
        }
        SSTAMP(5);
#ifdef SO100_STAGE_STAMPS
        if (kDebug && B.debug && sub == m->nsubstep - 1 && lane == 0) {
#pragma unroll
          for (int k = 0; k < 8; k++) B.debug[(size_t)env * SO100_DBG_STRIDE + 88 + k] = (float)sst_acc_[k];
        }
#endif
        if (kDebug && B.debug && sub == m->nsubstep - 1) {
          float* dbg = B.debug + (size_t)env * SO100_DBG_STRIDE;
          if (lane < kMaxCon) {
            dbg[16 + lane] = lane < ncon ? sh.con_dist[lane] : 0.f;
            dbg[48 + lane] = lane < ncon ? (float)sh.con_pair[lane] : -1.f;
          }
          if (lane < SO100_NV) dbg[64 + lane] = qs_r;
          if (lane == 0) {
            dbg[0] = (float)ncon;
            dbg[3] = (float)(12 + __popcll(lim_mask & (0xFFFFull << (grp * 16))) + 4 * ncon);
          }
        }
      }
      return;
    }
    // ---------------- S6a: per-contact Jacobian rows (-> HBM) and the row reductions (lane = dof, DPP).
    // Lane c keeps contact c's reductions: the scalar setup below then runs once per contact, in parallel
    // over the contacts, instead of redundantly on all 16 lanes for every contact.
    float4 Jr[kMaxCon];
    float cA[10], cV[4], cAc[4], cW[4];     // contact `lane`: (A)_upper, J qvel, J qacc_smooth, J qacc_warmstart
#pragma unroll
    for (int k = 0; k < 10; k++) cA[k] = 0.f;
#pragma unroll
    for (int r = 0; r < 4; r++) cV[r] = cAc[r] = cW[r] = 0.f;
#pragma unroll
    for (int c = 0; c < kMaxCon; c++) {
      Jr[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c < ncon_max) {
        float4 J = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c < ncon && lane < SO100_NV) {
          J = contact_jac(m, sh, c, lane);
          reinterpret_cast<float4*>(crec + c * kConRec + kJOff)[lane] = J;
        }
        Jr[c] = J;
        const float4 M = minv_times(J, minv_row, invmc, lane);   // M^-1 J' column of this dof
        const float jv[4] = {J.x, J.y, J.z, J.w}, mv[4] = {M.x, M.y, M.z, M.w};
        const bool mine = lane == c;
        int k = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
#pragma unroll
          for (int q = r; q < 4; q++, k++) {
            const float a = rowsum16(jv[r] * mv[q]);
            cA[k] = mine ? a : cA[k];
          }
          const float v = rowsum16(jv[r] * qvel_r), ac = rowsum16(jv[r] * qs_r), w = rowsum16(jv[r] * warm_r);
          cV[r] = mine ? v : cV[r];
          cAc[r] = mine ? ac : cAc[r];
          cW[r] = mine ? w : cW[r];
        }
      }
    }
    SSTAMP(3);
    // ---------------- S6b: scalar setup of contact `lane` (impedance, regularisers, warmstart dual map,
    // eigen-decomposition for the QCQP) -> solver block in the HBM record
    float cf[4] = {0.f, 0.f, 0.f, 0.f};
    if (lane < ncon) {
      const int p = sh.con_pair[lane];
      const float dist = sh.con_dist[lane];
      const float imp = getimpedance(m->pair_solimp[p], dist, m->pair_margin[p]);
      const float K = m->pair_K[p], Bd = m->pair_B[p];
      const float fs = m->pair_cube[p] ? fscale : 1.f;     // DR friction scale: cube pairs
      const float mu0 = m->pair_mu0[p] * fs, mu1 = m->pair_mu1[p] * fs;
      float R[4];
      R[0] = fmaxf(kMinVal, (1.f - imp) / imp * m->pair_tran[p]);
      R[1] = R[0] * mu0 * mu0 / (mu0 * mu0 * m->impratio);
      R[2] = R[1];
      R[3] = R[0] * mu0 * mu0 / (mu1 * mu1 * m->impratio);
      float aref[4];
      aref[0] = -Bd * cV[0] - K * imp * (dist - m->pair_margin[p]);
      aref[1] = -Bd * cV[1]; aref[2] = -Bd * cV[2]; aref[3] = -Bd * cV[3];
      // A + R, upper triangle row-major: 00 01 02 03 11 12 13 22 23 33
      float ar[10];
#pragma unroll
      for (int k = 0; k < 10; k++) ar[k] = cA[k];
      ar[0] += R[0]; ar[4] += R[1]; ar[7] += R[2]; ar[9] += R[3];
      // warmstart force: dual map of jar = J qacc_warmstart - aref (elliptic zones)
      float jar[4];
#pragma unroll
      for (int r = 0; r < 4; r++) jar[r] = cW[r] - aref[r];
      const float mus[3] = {mu0, mu0, mu1};
      {
        const float mu = mu0 * sqrtf(R[1] / R[0]);
        float U[4], T = 0.f;
        U[0] = jar[0] * mu;
#pragma unroll
        for (int k = 1; k < 4; k++) { U[k] = jar[k] * mus[k - 1]; T += U[k] * U[k]; }
        T = sqrtf(T);
        const float N = U[0];
        if (N >= mu * T || (T <= 0.f && N >= 0.f)) {
          cf[0] = cf[1] = cf[2] = cf[3] = 0.f;
        } else if (mu * N + T <= 0.f || (T <= 0.f && N < 0.f)) {
#pragma unroll
          for (int k = 0; k < 4; k++) cf[k] = -jar[k] / R[k];
        } else {
          const float Dm = (1.f / R[0]) / (mu * mu * (1.f + mu * mu));
          const float NmT = N - mu * T;
          cf[0] = -Dm * NmT * mu;
#pragma unroll
          for (int k = 1; k < 4; k++) cf[k] = -cf[0] / T * U[k] * mus[k - 1];
        }
      }
      // QCQP data: eigen-decomposition of the cone-scaled friction block (constant over the sweeps)
      const float A11[3][3] = {{ar[4], ar[5], ar[6]}, {ar[5], ar[7], ar[8]}, {ar[6], ar[8], ar[9]}};
      float As[3][3], Qe[3][3], lam[3];
#pragma unroll
      for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b2 = 0; b2 < 3; b2++) As[a][b2] = A11[a][b2] * mus[a] * mus[b2];
      eig3_sym(As, lam, Qe);
      // solver block (layout: so100_device.h), f written after the warmstart decision
      float P[3][3];
#pragma unroll
      for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) P[i][j] = Qe[j][i] * mus[j];
      float4* cs = reinterpret_cast<float4*>(crec + lane * kConRec);
      cs[0] = make_float4(ar[0], ar[1], ar[2], ar[3]);
      cs[1] = make_float4(ar[4], ar[5], ar[6], ar[7]);
      cs[2] = make_float4(ar[8], ar[9], P[0][0], P[0][1]);
      cs[3] = make_float4(P[0][2], P[1][0], P[1][1], P[1][2]);
      cs[4] = make_float4(P[2][0], P[2][1], P[2][2], lam[0]);
      cs[5] = make_float4(lam[1], lam[2], 1.f / lam[0], 1.f / lam[1]);
      cs[6] = make_float4(1.f / lam[2], R[0], 1.f / ar[0], R[1]);
      cs[kBlkFlags] = make_float4(R[3], m->pair_arm[p] ? 1.f : 0.f, 0.f, 0.f);
      cs[kBlkAref] = make_float4(aref[0], aref[1], aref[2], aref[3]);
#pragma unroll
      for (int r = 0; r < 4; r++) cost_part += 0.5f * R[r] * cf[r] * cf[r] + cf[r] * (cAc[r] - aref[r]);
    }
    SSTAMP(4);
    // J' f of the warmstart forces: contact c's forces broadcast from lane c
#pragma unroll
    for (int c = 0; c < kMaxCon; c++) {
      if (c < ncon_max) {
        const float4 fc = bcast_row4(make_float4(cf[0], cf[1], cf[2], cf[3]), c);
        phi += Jr[c].x * fc.x + Jr[c].y * fc.y + Jr[c].z * fc.z + Jr[c].w * fc.w;
      }
    }
    // ---------------- S7: warmstart dual cost 0.5 f'ARf + f'b (keep the warmstart only if <= 0)
    float dq = 0.f;
    {
      float acc_arm = 0.f;
#pragma unroll
      for (int j = 0; j < 6; j++) acc_arm += minv_row[j] * bcast_row(phi, j);
      dq = (lane < 6) ? acc_arm : invmc * phi;
    }
    cost_part += 0.5f * phi * dq;
    const float cost = rowsum16(cost_part);
    float qacc_c = qs_r;
    if (cost > 0.f) {
      fr_f = 0.f;
      lim_f = 0.f;
#pragma unroll
      for (int r = 0; r < 4; r++) cf[r] = 0.f;
    } else {
      qacc_c += dq;
    }
    if (lane < ncon) reinterpret_cast<float4*>(crec + lane * kConRec)[kBlkF] = make_float4(cf[0], cf[1], cf[2], cf[3]);

    // ---------------- solver record -> HBM (consumed by so100_pgs_kernel)
    if (valid) {
      if (lane < SO100_NV) {
        const int q = lane / 3, k = lane - 3 * (lane / 3);
        float* hd = args.w.hdr + (size_t)e * kHdrEnv + q * kHdrLane;
        hd[H_QACC + k] = qacc_c;
        hd[H_FRAREF + k] = fr_aref;
        hd[H_FRF + k] = fr_f;
        hd[H_LIMS + k] = lim_on ? lim_s : 0.f;
        hd[H_LIMAREF + k] = lim_aref;
        hd[H_LIMR + k] = lim_R;
        hd[H_LIMF + k] = lim_f;
        float* mr = hd + H_MROW + 6 * k;
        if (lane < 6) {
          const int own = 3 * q, par = 3 - own;
#pragma unroll
          for (int i = 0; i < 3; i++) { mr[i] = sh.minv[lane][own + i]; mr[3 + i] = sh.minv[lane][par + i]; }
        } else {
#pragma unroll
          for (int i = 0; i < 6; i++) mr[i] = (i == k) ? invmc : 0.f;
        }
        if (k == 0) hd[H_NCON] = __int_as_float(ncon);
      }
      SSTAMP(5);
#ifdef SO100_STAGE_STAMPS
      if (B.debug && sub == m->nsubstep - 1 && lane == 0) {
#pragma unroll
        for (int k = 0; k < 8; k++) B.debug[(size_t)env * SO100_DBG_STRIDE + 88 + k] = (float)sst_acc_[k];
      }
#endif
      // debug: contact set of the last substep (forces / iterations come from the solver kernel)
      if (B.debug && sub == m->nsubstep - 1) {
        float* dbg = B.debug + (size_t)env * SO100_DBG_STRIDE;
        if (lane < kMaxCon) {
          dbg[16 + lane] = lane < ncon ? sh.con_dist[lane] : 0.f;
          dbg[48 + lane] = lane < ncon ? (float)sh.con_pair[lane] : -1.f;
        }
        if (lane < SO100_NV) dbg[64 + lane] = qs_r;
        if (lane == 0) {
          dbg[0] = (float)ncon;
          dbg[3] = (float)(12 + __popcll(lim_mask & (0xFFFFull << (grp * 16))) + 4 * ncon);
        }
      }
    }
}

// The env step's epilogue (kMode 2 / the fused kernel's tail): the mj_step1 position stage (sites, contact
// set), reward, obs, TimeLimit, divergence, auto-reset, and the state store.
DEV void final_stage(const StageArgs& args, EnvShared& sh, int lane, int grp, int env, int e, bool valid, float qpos_r,
                     float qvel_r, float warm_r, int elapsed0, uint32_t episode0) {
  const DevModel* __restrict__ m = args.m;
  const so100_buffers& B = args.b;
  // ---------------- final position stage (mj_step1): sites + contact set for reward / obs
  if (lane < SO100_NQ) sh.qpos[lane] = qpos_r;
  if (lane < SO100_NV) sh.qvel[lane] = qvel_r;
  __syncthreads();
  fk_par(m, sh, lane);
  __syncthreads();
  float hx, hy, hz;
  const bool hfound = hull_table(m, sh, lane, grp, valid, hx, hy, hz);
  const uint32_t hrow = (uint32_t)((__ballot(hfound) >> (grp * 16)) & 0xFFFFull);
  PairContacts pc;
  pc.n = 0;
  if (lane < SO100_NPAIR_BOX) collide_pair(m, sh, lane, pc);
  const uint64_t hit = __ballot(pc.n > 0);
  const uint32_t bits = (uint32_t)((hit >> (grp * 16)) & 0x3FFFull) | (hrow << SO100_NPAIR_BOX);

  // divergence check (dm_control PhysicsError analogue)
  bool bad = (lane < SO100_NQ) && !(fabsf(qpos_r) < 1e4f);
  bad = bad || ((lane < SO100_NV) && !(fabsf(qvel_r) < 1e6f));
  const bool diverged = ((__ballot(bad) >> (grp * 16)) & 0xFFFFull) != 0ull;

  float cube_f[3] = {sh.site_cube[0], sh.site_cube[1], sh.site_cube[2]};
  float ee_f[3] = {sh.site_ee[0], sh.site_ee[1], sh.site_ee[2]};
  double reward = 0.0;
  bool terminated = false, truncated = false, success = false;
  int elapsed = elapsed0 + 1;
  const bool goal = args.task == SO100_TASK_GOAL;
  float goal_des[3] = {0.f, 0.f, 0.f};
  if (goal) {
    // SO100GoalEnv.step (env.py:372-406): sparse reward on ||achieved - desired|| < 0.01
#pragma unroll
    for (int k = 0; k < 3; k++) goal_des[k] = B.desired_goal[(size_t)e * 3 + k];
    float d0 = cube_f[0] - goal_des[0], d1 = cube_f[1] - goal_des[1], d2 = cube_f[2] - goal_des[2];
    float dist = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
    success = dist < (float)m->goal_threshold;
    reward = success ? 0.0 : -1.0;
    terminated = success;
    truncated = elapsed >= args.max_steps;
  } else {
    reward = task_reward(m, args.task, cube_f, ee_f, bits);
    terminated = success = (reward == 4.0);              // env.py:175
    truncated = args.max_steps > 0 && elapsed >= args.max_steps;   // TimeLimit (gym_so100/__init__.py)
  }
  if (diverged) truncated = true;
  const bool doneflag = terminated || truncated;

  const float qv_obs = bcast16(qpos_r, lane >= 9 ? lane - 9 : 0);
  if (valid) {
    if (lane == 0) {
      if (B.reward) B.reward[env] = (float)reward;
      if (B.reward64) B.reward64[env] = reward;
      if (B.terminated) B.terminated[env] = terminated;
      if (B.truncated) B.truncated[env] = truncated;
      if (B.success) B.success[env] = success;
      if (B.diverged) B.diverged[env] = diverged;
      if (B.contact_bits) B.contact_bits[env] = bits;
      if (goal && B.total_steps) B.total_steps[env] = B.total_steps[env] + 1;
      if (B.ep_return) {
        // episode statistics (RecordEpisodeStatistics): the running float64 return, and at the episode's end
        // its return and length into ep_final and the env's running totals
        const double ret = B.ep_return[env] + reward;
        B.ep_return[env] = doneflag ? 0.0 : ret;
        if (doneflag && B.ep_final) {
          B.ep_final[(size_t)env * 2] = ret;
          B.ep_final[(size_t)env * 2 + 1] = (double)elapsed;
        }
        if (doneflag && B.ep_accum) {
          double* a = B.ep_accum + (size_t)env * 4;
          a[0] += 1.0;
          a[1] += success ? 1.0 : 0.0;
          a[2] += ret;
          a[3] += (double)elapsed;
        }
      }
    }
    if (goal && B.achieved_goal && lane < 3) B.achieved_goal[(size_t)env * 3 + lane] = cube_f[lane];
    if (B.obs) write_obs(m, sh, lane, qv_obs, B.obs + (size_t)env * SO100_NOBS);
  }

  const bool autoreset = (args.flags & SO100_FLAG_AUTORESET) != 0;
  const bool do_reset = autoreset && doneflag;
  const uint64_t rmask = __ballot(do_reset && valid);
  int new_elapsed = elapsed;
  uint32_t new_episode = episode0;
  if (rmask) {
    if (do_reset && valid && B.final_obs && lane < SO100_NOBS && B.obs)
      B.final_obs[(size_t)env * SO100_NOBS + lane] = B.obs[(size_t)env * SO100_NOBS + lane];
    if (do_reset && valid) {
      new_episode = episode0 + 1;
      new_elapsed = 0;
      uint32_t seed = episode_seed(args.base_seed, (uint32_t)(env + args.env_offset), new_episode);
      env_reset_state(m, sh, lane, seed, qpos_r, qvel_r, warm_r, nullptr);
    }
    __syncthreads();
    if (lane < SO100_NQ) sh.qpos[lane] = qpos_r;
    __syncthreads();
    fk_par(m, sh, lane, do_reset && valid);
    __syncthreads();
    const float qv_r = bcast16(qpos_r, lane >= 9 ? lane - 9 : 0);
    if (do_reset && valid) {
      if (B.obs) write_obs(m, sh, lane, qv_r, B.obs + (size_t)env * SO100_NOBS);
      if (goal) {
        // _sample_goal (env.py:322-334): lifted box around the spawn while total_steps < 5000, else bin box
        const int tsteps = B.total_steps ? B.total_steps[env] : 0;
        if (lane < 3) {
          float u = hash_uniform(splitmix64(args.base_seed * 31ull + ((uint64_t)(env + args.env_offset) << 24) + new_episode * 3ull + lane));
          float lo, hi;
          if (tsteps < 5000) {
            float c = lane < 2 ? sh.qpos[6 + lane] : 0.f;
            lo = lane < 2 ? c - 0.03f : 0.01f;
            hi = lane < 2 ? c + 0.03f : 0.05f;
          } else {
            lo = m->goal_bin_lo[lane];
            hi = m->goal_bin_hi[lane];
          }
          B.desired_goal[(size_t)env * 3 + lane] = lo + (hi - lo) * u;
          if (B.achieved_goal) B.achieved_goal[(size_t)env * 3 + lane] = sh.site_cube[lane];
        }
      }
    }
  }

  // ---------------- store state
  if (valid) {
    if (lane < SO100_NQ) B.qpos[(size_t)env * SO100_NQ + lane] = qpos_r;
    if (lane < SO100_NV) {
      B.qvel[(size_t)env * SO100_NV + lane] = qvel_r;
      B.qacc_warmstart[(size_t)env * SO100_NV + lane] = warm_r;
    }
    if (lane == 0) {
      if (B.elapsed) B.elapsed[env] = new_elapsed;
      if (B.episode) B.episode[env] = new_episode;
    }
  }
}


// Substep stage kernel of the split path (one wave = 4 envs x 16 lanes).
//   kMode 0: substep 0 — position/velocity stages and constraint assembly on the stored state;
//   kMode 1: Euler with the previous substep's solver output, then the same assembly;
//   kMode 2: Euler, then the mj_step1 position stage and the task epilogue (reward, obs, autoreset).
// Assembly writes the solver's per-env record (Workspace) that so100_pgs_kernel / so100_newton_kernel consume.
template <int kMode, int kSolver>
__global__ void __launch_bounds__(kThreads, SO100_STAGE_WAVES) so100_stage_kernel(StageArgs args) {
  __shared__ EnvShared shm[kEnvsPerBlock];
  const int tid = threadIdx.x;
  const int grp = tid >> 4;
  const int lane = tid & 15;
  const int env = blockIdx.x * kEnvsPerBlock + grp;
  const bool valid = env < args.n;
  const int e = valid ? env : 0;          // clamp loads for the tail group; stores are guarded
  EnvShared& sh = shm[grp];
  float qpos_r, qvel_r, warm_r, mscale, fscale, sigma;
  int elapsed0;
  uint32_t episode0;
  load_state(args, lane, e, qpos_r, qvel_r, warm_r, mscale, fscale, sigma, elapsed0, episode0);
  if (kMode != 0) euler_update(sh, lane, args.m->timestep, warm_r, qpos_r, qvel_r);
  if constexpr (kMode != 2) {
    set_controls(args, sh, lane, e, sigma, elapsed0, episode0);
    NewtonRows nr;
    assemble<kSolver, false>(args, sh, lane, grp, env, e, valid, qpos_r, qvel_r, warm_r, mscale, fscale, args.sub, nr);
    if (kMode == 1 && valid) {
      if (lane < SO100_NQ) args.b.qpos[(size_t)env * SO100_NQ + lane] = qpos_r;
      if (lane < SO100_NV) args.b.qvel[(size_t)env * SO100_NV + lane] = qvel_r;
    }
  } else {
    final_stage(args, sh, lane, grp, env, e, valid, qpos_r, qvel_r, warm_r, elapsed0, episode0);
  }
}

#ifndef SO100_LAUNDER
#define SO100_LAUNDER 2
#endif
#ifndef SO100_LAUNDER_IDS
#define SO100_LAUNDER_IDS 2
#endif
// the fused kernel's lane / env ids inside the substep loop and the epilogue, from an opaque read of the lane's
// position in its wave (one wave per workgroup) and the workgroup's group index (scalar)
static_assert(kThreads == 64, "fresh_ids: one wave per workgroup");
DEV void fresh_ids(int group, int n, int& lane, int& grp, int& env, int& e) {
  int t;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(t));
  lane = t & (kLanes - 1);
  grp = t / kLanes;
  env = group * kEnvsPerBlock + grp;
  e = env < n ? env : 0;
}
#ifndef SO100_PRIO
#define SO100_PRIO 1
#endif
#ifndef SO100_W2_NOLAUNDER
#define SO100_W2_NOLAUNDER 0
#endif
#ifndef SO100_FUSED_WAVES
#define SO100_FUSED_WAVES 3
#endif
#ifndef SO100_FUSED_RELOAD
#define SO100_FUSED_RELOAD 0
#endif
// The whole env step in one launch (Newton solver, the default): each wave runs its 4 envs through the 10
// substeps — Euler, assembly, the Newton solve with the rows handed over in registers (no HBM record) —
// and the epilogue, with the state in registers throughout.  The split path's 21 launches end every
// substep at the slowest wave of the chip; here a wave only waits for itself.
// Results are those of the split path (so100_stage_kernel + so100_newton_kernel): the same device
// functions on the same values.  kDebug: the instantiation that also fills the debug buffer (launched when
// the caller passes one); the other has no debug code, which costs registers in the substep loop.
// kWaves: the waves per SIMD the register budget is sized for.  3 (168 VGPRs, 72 B/lane of spill slots) when
// the grid exceeds 2 waves per SIMD; a grid of at most 2 waves per SIMD (8,192 envs on 256 CUs: all waves
// resident at once) takes the 2-wave build (186 VGPRs, no scratch; +0.8 % there, -7 % at 16,384 envs).
// Register allocation only: both give the same results bit for bit.
template <bool kDebug, int kWaves = SO100_FUSED_WAVES>
__global__ void __launch_bounds__(kThreads, kWaves) so100_fused_kernel(const DevModel* __restrict__ model,
                                                                       StageArgs kargs) {
  // the model as a noalias kernel argument: no store of the step can clobber it, so its uniform loads stay
  // scalar (s_load) after the substeps' global stores (through args.m they became vector loads)
  StageArgs args = kargs;
  args.m = model;
#ifdef SO100_TIMELINE
  // diagnostic build: wave start / end (s_memrealtime) and shader cycles in assembly / Newton / epilogue
  const uint64_t tl_t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t tl_acc[3] = {0, 0, 0}, tl_prev = 0;
#define TL_MARK(slot)                                                                            \
  do {                                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                                            \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    if ((slot) >= 0) tl_acc[(slot) < 0 ? 0 : (slot)] += t_ - tl_prev;                            \
    tl_prev = t_;                                                                                \
  } while (0)
#else
#define TL_MARK(slot) do {} while (0)
#endif
  __shared__ EnvShared shm[kEnvsPerBlock];
  const uint64_t cost_t0 = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x;
  const int grp0 = tid >> 4;
  const int lane0 = tid & 15;
  const int group = args.w.order ? args.w.order[blockIdx.x] : (int)blockIdx.x;   // heavy-first (so100_order_kernel)
#if SO100_PRIO
  if (args.w.order) {   // the heavier half of the waves, by launch rank, issue first on their SIMD
    const unsigned rank = blockIdx.x, ng = gridDim.x;
    if (rank < ng / 8) __builtin_amdgcn_s_setprio(3);
    else if (rank < ng / 4) __builtin_amdgcn_s_setprio(2);
    else if (rank < ng / 2) __builtin_amdgcn_s_setprio(1);
  }
#endif
  const int env0 = group * kEnvsPerBlock + grp0;
  const int e0 = env0 < args.n ? env0 : 0;
  {
  const int grp = grp0, lane = lane0, e = e0;
  EnvShared& sh = shm[grp];
  float qpos_r, qvel_r, warm_r, mscale, fscale, sigma;
  int elapsed0;
  uint32_t episode0;
  load_state(args, lane, e, qpos_r, qvel_r, warm_r, mscale, fscale, sigma, elapsed0, episode0);
  set_controls(args, sh, lane, e, sigma, elapsed0, episode0);
  const int nsub = args.m->nsubstep;
  const float h = args.m->timestep;
  for (int sub = 0; sub < nsub; sub++) {
    // the lane / env ids laundered per substep too: what derives from them (masks, addresses, per-lane
    // model values) is recomputed in each substep instead of hoisted and held live across the loop
    int lane = lane0, grp = grp0, env = env0, e = e0;
#if SO100_LAUNDER_IDS == 2
    // recomputed from the wave's lane id (an opaque v_mbcnt pair, which LICM cannot hoist) and the
    // workgroup's scalar group index: no vector value of the ids is carried across the loop
    fresh_ids(group, args.n, lane, grp, env, e);
#else
    if constexpr (SO100_LAUNDER_IDS && !(kWaves == 2 && SO100_W2_NOLAUNDER))
      asm volatile("" : "+v"(lane), "+v"(grp), "+v"(env), "+v"(e));
#endif
    const bool valid = env < args.n;
    EnvShared& sh = shm[grp];
    TL_MARK(-1);
    if (sub > 0) euler_update(sh, lane, h, warm_r, qpos_r, qvel_r);
    // the model pointer laundered per substep: the model loads (uniform, ~1 KB) must not be hoisted out of
    // the substep loop, where they would stay live across it (register spills)
    StageArgs sa = args;
#if SO100_LAUNDER == 1
    asm volatile("" : "+s"(sa.m));
#elif SO100_LAUNDER == 2
    {
      int zero;
      asm volatile("s_mov_b32 %0, 0" : "=s"(zero));
      sa.m = reinterpret_cast<const DevModel*>(reinterpret_cast<const char*>(args.m) + zero);
    }
#endif
    NewtonRows nr;
#if SO100_FUSED_RELOAD
    // the env's DR scales re-read per substep (L2-hot, 8 B) instead of carried across the loop body's register
    // peak (the 3-wave build spilled them with the other loop-carried values)
    float ms = 1.f, fs = 1.f;
    if ((args.flags & SO100_FLAG_DR) && args.b.dr_params) {
      ms = args.b.dr_params[(size_t)e * 4 + 0];
      fs = args.b.dr_params[(size_t)e * 4 + 1];
    }
    (void)mscale; (void)fscale;
#else
    const float ms = mscale, fs = fscale;
#endif
    assemble<SO100_SOLVER_NEWTON, true, kDebug, !kDebug && kWaves == 2>(sa, sh, lane, grp, env, e, valid, qpos_r, qvel_r, warm_r, ms,
                                                fs, sub, nr);
    TL_MARK(0);
    NewtonDiag diag;
    const bool dbg = kDebug && args.b.debug && sub == nsub - 1;
    const float qacc = newton_solve(sa.m, nr, lane, valid, dbg, diag);
    if (dbg) {
      int row = env;
      asm volatile("" : "+v"(row));        // not the assembly's row address (GVN would hold that across the solve)
      newton_diag_write(args.b.debug + (size_t)row * SO100_DBG_STRIDE, lane, valid, qacc, diag);
    }
    warm_r = lane < SO100_NV ? qacc : 0.f;
    TL_MARK(1);
  }
  TL_MARK(-1);
  {
    // fresh ids again: the epilogue's store addresses must not be the prologue's load addresses (CSE would
    // hold those across the substep loop)
    int lane = lane0, grp = grp0, env = env0, e = e0;
#if SO100_LAUNDER_IDS == 2
    fresh_ids(group, args.n, lane, grp, env, e);
#else
    asm volatile("" : "+v"(lane), "+v"(grp), "+v"(env), "+v"(e));
#endif
    const bool valid = env < args.n;
    EnvShared& sh = shm[grp];
    euler_update(sh, lane, h, warm_r, qpos_r, qvel_r);
#if SO100_FUSED_RELOAD
    // the step counters re-read (the prologue's values, not yet written) instead of carried across the loop
    const int el = args.b.elapsed ? args.b.elapsed[e] : 0;
    const uint32_t ep = args.b.episode ? args.b.episode[e] : 0u;
    (void)elapsed0; (void)episode0;
#else
    const int el = elapsed0;
    const uint32_t ep = episode0;
#endif
    final_stage(args, sh, lane, grp, env, e, valid, qpos_r, qvel_r, warm_r, el, ep);
    if (valid && lane == 0 && args.b.ncon_dropped) args.b.ncon_dropped[env] = (uint32_t)sh.ndrop;
  }
  TL_MARK(2);
  if (args.w.gcost && tid == 0) args.w.gcost[group] = (uint32_t)(__builtin_amdgcn_s_memtime() - cost_t0);
#ifdef SO100_TIMELINE
  if (args.b.debug && env0 < args.n && lane0 == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    float* dbg = args.b.debug + (size_t)env0 * SO100_DBG_STRIDE;
    dbg[88] = __uint_as_float((uint32_t)tl_t0); dbg[89] = __uint_as_float((uint32_t)(tl_t0 >> 32));
    dbg[90] = __uint_as_float((uint32_t)t1); dbg[91] = __uint_as_float((uint32_t)(t1 >> 32));
    dbg[92] = (float)tl_acc[0];
    dbg[93] = (float)tl_acc[1];
    dbg[94] = (float)tl_acc[2];
  }
#endif
  }
}

// ------------------------------------------------------------------ reset kernel
struct ResetArgs {
  const DevModel* m;
  so100_buffers b;
  int n;
  int task;
  uint64_t base_seed;
  int env_offset;
  const uint8_t* mask;
  const uint32_t* seeds;
};

__global__ void __launch_bounds__(kThreads) so100_reset_kernel(ResetArgs args) {
  __shared__ EnvShared shm[kEnvsPerBlock];
  const DevModel* __restrict__ m = args.m;
  const int tid = threadIdx.x, grp = tid >> 4, lane = tid & 15;
  const int env = blockIdx.x * kEnvsPerBlock + grp;
  const bool valid = env < args.n;
  const int e = valid ? env : 0;
  EnvShared& sh = shm[grp];
  const so100_buffers& B = args.b;
  const bool act = valid && (args.mask == nullptr || args.mask[e] != 0);
  float qpos_r = 0.f, qvel_r = 0.f, warm_r = 0.f;
  uint32_t episode = B.episode ? B.episode[e] + (act ? 1u : 0u) : 0u;
  if (act) {
    uint32_t seed = args.seeds ? args.seeds[e] : episode_seed(args.base_seed, (uint32_t)(env + args.env_offset), episode);
    env_reset_state(m, sh, lane, seed, qpos_r, qvel_r, warm_r, nullptr);
  }
  if (lane < SO100_NQ) sh.qpos[lane] = qpos_r;
  __syncthreads();
  fk_par(m, sh, lane, act);
  __syncthreads();
  const float qv_r = bcast16(qpos_r, lane >= 9 ? lane - 9 : 0);
  if (act) {
    if (B.obs) write_obs(m, sh, lane, qv_r, B.obs + (size_t)env * SO100_NOBS);
    if (lane < SO100_NQ) B.qpos[(size_t)env * SO100_NQ + lane] = qpos_r;
    if (lane < SO100_NV) {
      B.qvel[(size_t)env * SO100_NV + lane] = 0.f;
      B.qacc_warmstart[(size_t)env * SO100_NV + lane] = 0.f;
    }
    if (lane == 0) {
      if (B.elapsed) B.elapsed[env] = 0;
      if (B.episode) B.episode[env] = episode;
      if (B.ep_return) B.ep_return[env] = 0.0;
    }
    if (args.task == SO100_TASK_GOAL && B.desired_goal && lane < 3) {
      const int tsteps = B.total_steps ? B.total_steps[env] : 0;
      float u = hash_uniform(splitmix64(args.base_seed * 31ull + ((uint64_t)(env + args.env_offset) << 24) + episode * 3ull + lane));
      float lo, hi;
      if (tsteps < 5000) {
        float c = lane < 2 ? sh.qpos[6 + lane] : 0.f;
        lo = lane < 2 ? c - 0.03f : 0.01f;
        hi = lane < 2 ? c + 0.03f : 0.05f;
      } else {
        lo = m->goal_bin_lo[lane];
        hi = m->goal_bin_hi[lane];
      }
      B.desired_goal[(size_t)env * 3 + lane] = lo + (hi - lo) * u;
      if (B.achieved_goal) B.achieved_goal[(size_t)env * 3 + lane] = sh.site_cube[lane];
    }
  }
}

// ------------------------------------------------------------------ standalone ops (parity surface)
__global__ void so100_reward_kernel(const DevModel* m, int task, int n, const float* cube, const float* ee,
                                    const uint32_t* bits, float* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float c[3] = {cube[3 * i], cube[3 * i + 1], cube[3 * i + 2]};
  float x[3] = {ee[3 * i], ee[3 * i + 1], ee[3 * i + 2]};
  out[i] = (float)task_reward(m, task, c, x, bits[i]);
}

__global__ void so100_spawn_kernel(const DevModel* m, int n, const uint32_t* seeds, double* pose) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double p[7];
  spawn_pose(m, seeds[i], p);
  for (int k = 0; k < 7; k++) pose[7 * i + k] = p[k];
}

__global__ void so100_unnormalize_kernel(const DevModel* m, int n, const float* a, float* c) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * 6) return;
  int k = i % 6;
  c[i] = unnormalize_f32(a[i], m->action_lo[k], m->action_hi[k], m->action_span[k]);
}

__global__ void so100_goal_reward_kernel(const DevModel* m, int n, const float* a, const float* d, float* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // np.linalg.norm(achieved - desired, axis=1) in float32 (env.py:347-349)
  float d0 = a[3 * i] - d[3 * i], d1 = a[3 * i + 1] - d[3 * i + 1], d2 = a[3 * i + 2] - d[3 * i + 2];
  float dist = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
  out[i] = dist < (float)m->goal_threshold ? 0.f : -1.f;
}

// ------------------------------------------------------------------ launchers (called by so100_capi.cpp)
hipError_t launch_pgs(const DevModel* m, const Workspace& w, float* qacc_out, float* debug, int n, int last, int par,
                      hipStream_t s);


// One env step = nsubstep x (stage, solve) + the final stage: 2 * nsubstep + 1 launches on one stream (split
// path), or one fused launch.  ev (optional, profiling): 2 nsubstep + 2 events (split) or 2 (fused), recorded
// before the first launch and after each.
hipError_t launch_newton(const DevModel* m, const Workspace& w, float* qacc_out, float* debug, int n, int last,
                         hipStream_t s);

// Heavy-first wave order for the fused kernel.  Its waves run a whole env step each (0.4-1.8 ms) and the
// grid exceeds the resident slots (12 per CU) above 12,288 envs: a long wave dispatched late sets the step's
// tail.  Wave costs persist from step to step (correlation 0.65-0.74, measured), so the groups are launched
// in descending order of their previous step's cost: a counting sort on a 12-bit float key (exponent + 4
// mantissa bits, 6 % buckets), one workgroup.  The order changes the schedule, never a result.
constexpr int kOrderBuckets = 4096;
#if SO100_PRIO
constexpr int kOrderMinGroups = 256;           // the order also sets the waves' issue priority
#else
constexpr int kOrderMinGroups = 3072;          // up to the resident capacity (12 waves x 256 CUs) all start at once
#endif
__global__ void __launch_bounds__(1024) so100_order_kernel(const uint32_t* __restrict__ gcost, int ng,
                                                           int* __restrict__ order) {
  __shared__ int hist[kOrderBuckets];
  __shared__ int part[1024];
  const int t = threadIdx.x;
  auto key = [](uint32_t c) { return (kOrderBuckets - 1) - (int)((__float_as_uint((float)c) >> 19) & 0xFFFu); };
  for (int b = t; b < kOrderBuckets; b += 1024) hist[b] = 0;
  __syncthreads();
  for (int g = t; g < ng; g += 1024) atomicAdd(&hist[key(gcost[g])], 1);
  __syncthreads();
  int loc[kOrderBuckets / 1024], sum = 0;
#pragma unroll
  for (int k = 0; k < kOrderBuckets / 1024; k++) { loc[k] = sum; sum += hist[(kOrderBuckets / 1024) * t + k]; }
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {           // inclusive scan of the per-thread sums
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const int base = part[t] - sum;
#pragma unroll
  for (int k = 0; k < kOrderBuckets / 1024; k++) hist[(kOrderBuckets / 1024) * t + k] = base + loc[k];
  __syncthreads();
  for (int g = t; g < ng; g += 1024) order[atomicAdd(&hist[key(gcost[g])], 1)] = g;
}

// compute units of the current device (cached per device; 0 if the query fails: the 3-wave build then)
static int device_cus() {
  static int cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cus[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) return 0;
    cus[dev] = v;
  }
  return cus[dev];
}

// The fused kernel build a launch of n envs takes: 1 = the debug build (a debug buffer is passed), else the
// product build for `waves` waves per SIMD (2 | 3; 0 = auto: 2 when the grid fits the chip at 2 waves per
// SIMD, i.e. at most 8 workgroups per CU, else 3).
int fused_build(int n, int waves, bool debug) {
  if (debug) return 1;
  if (waves == 2 || waves == 3) return waves;
  const int ng = (n + kEnvsPerBlock - 1) / kEnvsPerBlock;
  return ng <= 2 * 4 * device_cus() ? 2 : 3;
}

// fused (Newton only): the whole env step as one so100_fused_kernel launch; ev then takes 2 events.
// waves: the fused product build (fused_build).
hipError_t launch_step(const DevModel* m, int nsubstep, int solver, int fused, int waves, Workspace& w,
                       const so100_buffers& b, int n, int task, int flags, int max_steps, uint64_t base_seed,
                       int env_offset, hipStream_t s, hipEvent_t* ev) {
  StageArgs a{m, b, w, n, task, flags, max_steps, base_seed, env_offset, 0, 0};
  const dim3 grid((n + kEnvsPerBlock - 1) / kEnvsPerBlock);
  int k = 0;
  if (ev) (void)hipEventRecord(ev[k++], s);
  if (fused && solver == SO100_SOLVER_NEWTON) {
    const int ng = (int)grid.x;
    if (w.order && w.gcost && ng > kOrderMinGroups) {
      if (ev) (void)hipEventRecord(ev[0], s);   // the order kernel stays outside the timed launch
      hipLaunchKernelGGL(so100_order_kernel, dim3(1), dim3(1024), 0, s, w.gcost, ng, w.order);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      if (ev) (void)hipEventRecord(ev[0], s);
    } else {
      a.w.order = nullptr;
    }
    const int build = fused_build(n, waves, b.debug != nullptr);
    if (build == 1) hipLaunchKernelGGL(so100_fused_kernel<true>, grid, dim3(kThreads), 0, s, m, a);
    else if (build == 2) hipLaunchKernelGGL((so100_fused_kernel<false, 2>), grid, dim3(kThreads), 0, s, m, a);
    else hipLaunchKernelGGL((so100_fused_kernel<false, 3>), grid, dim3(kThreads), 0, s, m, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[k++], s);
    w.sub_count += (uint32_t)nsubstep;
    return hipSuccess;
  }
  for (int sub = 0; sub <= nsubstep; sub++) {
    a.sub = sub;
    a.par = (int)(w.sub_count & 1u);
    if (solver == SO100_SOLVER_NEWTON) {
      if (sub == 0) hipLaunchKernelGGL((so100_stage_kernel<0, SO100_SOLVER_NEWTON>), grid, dim3(kThreads), 0, s, a);
      else if (sub < nsubstep) hipLaunchKernelGGL((so100_stage_kernel<1, SO100_SOLVER_NEWTON>), grid, dim3(kThreads), 0, s, a);
      else hipLaunchKernelGGL((so100_stage_kernel<2, SO100_SOLVER_NEWTON>), grid, dim3(kThreads), 0, s, a);
    } else {
      if (sub == 0) hipLaunchKernelGGL((so100_stage_kernel<0, SO100_SOLVER_PGS>), grid, dim3(kThreads), 0, s, a);
      else if (sub < nsubstep) hipLaunchKernelGGL((so100_stage_kernel<1, SO100_SOLVER_PGS>), grid, dim3(kThreads), 0, s, a);
      else hipLaunchKernelGGL((so100_stage_kernel<2, SO100_SOLVER_PGS>), grid, dim3(kThreads), 0, s, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[k++], s);
    if (sub < nsubstep) {
      e = solver == SO100_SOLVER_NEWTON ? launch_newton(m, w, b.qacc_warmstart, b.debug, n, sub == nsubstep - 1, s)
                                        : launch_pgs(m, w, b.qacc_warmstart, b.debug, n, sub == nsubstep - 1, a.par, s);
      if (e != hipSuccess) return e;
      if (ev) (void)hipEventRecord(ev[k++], s);
      w.sub_count++;
    }
  }
  return hipSuccess;
}

// Sum of the contact counts in the solver records of the last substep (H_NCON of lane-0 records).
__global__ void so100_contact_count_kernel(const float* __restrict__ hdr, int n, unsigned long long* accum) {
  __shared__ int part[256];
  int s = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    s += __float_as_int(hdr[(size_t)i * kHdrEnv + H_NCON]);
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 128; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d) part[threadIdx.x] += part[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(accum, (unsigned long long)part[0]);
}
#ifdef SO100_EPA_STAMPS
}  // namespace so100
extern "C" int so100_dev_epa_cycles(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(so100::so100_epa_cyc), sizeof(unsigned long long) * 12) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[12] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(so100::so100_epa_cyc), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
namespace so100 {
#endif
hipError_t launch_contact_count(const Workspace& w, int n, uint64_t* accum, hipStream_t s) {
  int blocks = (n + 255) / 256;
  if (blocks > 256) blocks = 256;
  hipLaunchKernelGGL(so100_contact_count_kernel, dim3(blocks), dim3(256), 0, s, w.hdr, n,
                     reinterpret_cast<unsigned long long*>(accum));
  return hipGetLastError();
}

hipError_t free_workspace(Workspace* w);
hipError_t alloc_workspace(int n, Workspace* w) {
  *w = Workspace{};
  hipError_t e = hipMalloc(&w->hdr, (size_t)n * kHdrEnv * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&w->con, (size_t)n * kMaxCon * kConRec * sizeof(float));
  // zero once: record slots a solver lane reads but never uses are then finite, never garbage
  if (e == hipSuccess) e = hipMemset(w->hdr, 0, (size_t)n * kHdrEnv * sizeof(float));
  if (e == hipSuccess) e = hipMemset(w->con, 0, (size_t)n * kMaxCon * kConRec * sizeof(float));
  const size_t ngroups = (size_t)(n + kPgsEnvs - 1) / kPgsEnvs;
  if (e == hipSuccess) e = hipMalloc(&w->gflag, 2 * ngroups * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&w->hcount, 2 * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&w->hlist, 2 * kHeavyCap * sizeof(int));
  if (e == hipSuccess) e = hipMemset(w->gflag, 0, 2 * ngroups * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(w->hcount, 0, 2 * sizeof(int));
  if (e != hipSuccess) (void)free_workspace(w);
  return e;
}
hipError_t free_workspace(Workspace* w) {
  hipError_t r = hipSuccess;
  for (void* p : {(void*)w->hdr, (void*)w->con, (void*)w->gflag, (void*)w->hcount, (void*)w->hlist, (void*)w->gcost,
                  (void*)w->order}) {
    if (!p) continue;
    hipError_t e = hipFree(p);
    if (r == hipSuccess) r = e;
  }
  w->hdr = w->con = nullptr;
  w->gflag = w->gcost = nullptr;
  w->hcount = w->hlist = w->order = nullptr;
  return r;
}
// The fused path's workspace: the record header (only its contact counts are written) and the wave-order
// buffers.
hipError_t alloc_fused_workspace(int n, Workspace* w) {
  *w = Workspace{};
  const size_t ng = (size_t)(n + kEnvsPerBlock - 1) / kEnvsPerBlock;
  hipError_t e = hipMalloc(&w->hdr, (size_t)n * kHdrEnv * sizeof(float));
  if (e == hipSuccess) e = hipMemset(w->hdr, 0, (size_t)n * kHdrEnv * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&w->gcost, ng * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(w->gcost, 0, ng * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&w->order, ng * sizeof(int));
  if (e != hipSuccess) (void)free_workspace(w);
  return e;
}
hipError_t launch_reset(const DevModel* m, const so100_buffers& b, int n, int task, uint64_t base_seed,
                        int env_offset, const uint8_t* mask, const uint32_t* seeds, hipStream_t s) {
  ResetArgs a{m, b, n, task, base_seed, env_offset, mask, seeds};
  dim3 grid((n + kEnvsPerBlock - 1) / kEnvsPerBlock);
  hipLaunchKernelGGL(so100_reset_kernel, grid, dim3(kThreads), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_reward(const DevModel* m, int task, int n, const float* c, const float* e, const uint32_t* bits,
                         float* out, hipStream_t s) {
  hipLaunchKernelGGL(so100_reward_kernel, dim3((n + 255) / 256), dim3(256), 0, s, m, task, n, c, e, bits, out);
  return hipGetLastError();
}
hipError_t launch_spawn(const DevModel* m, int n, const uint32_t* seeds, double* pose, hipStream_t s) {
  hipLaunchKernelGGL(so100_spawn_kernel, dim3((n + 255) / 256), dim3(256), 0, s, m, n, seeds, pose);
  return hipGetLastError();
}
hipError_t launch_unnormalize(const DevModel* m, int n, const float* a, float* c, hipStream_t s) {
  hipLaunchKernelGGL(so100_unnormalize_kernel, dim3((n * 6 + 255) / 256), dim3(256), 0, s, m, n, a, c);
  return hipGetLastError();
}
hipError_t launch_goal_reward(const DevModel* m, int n, const float* a, const float* d, float* out, hipStream_t s) {
  hipLaunchKernelGGL(so100_goal_reward_kernel, dim3((n + 255) / 256), dim3(256), 0, s, m, n, a, d, out);
  return hipGetLastError();
}

}  // namespace so100
