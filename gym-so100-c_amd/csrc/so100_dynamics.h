// so100_dynamics.h — the arm's position / velocity stage on an env's 16 lanes: spatial algebra, MuJoCo's impedance, the EE
// variant's weld elimination, CRBA + Cholesky + M^-1 columns, RNE bias and the position actuators
// (MuJoCo mj_comPos / mj_crb / mj_factorM / mj_rne / mj_fwdActuation restated; oracle kinematics/dynamics).
// (internal; included by so100_step.hip, the one translation unit of the step kernels)
#pragma once
#include "so100_common.h"
#include "so100_kin.h"

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
  // solimp power 1 or 2 (so100_create admits no other: MuJoCo's default 2 is the model's everywhere; a general
  // power would inline four powf at every call site of this function, about 2,600 instructions of the fused kernel)
  float y;
  if (power == 1.0f) y = x;
  else y = x <= mid ? x * x * __builtin_amdgcn_rcpf(mid)
                    : 1.0f - (1.0f - x) * (1.0f - x) * __builtin_amdgcn_rcpf(1.0f - mid);
  return dmin + y * (dmax - dmin);
}

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
    for (int k = 0; k < 4; k++) q1[k] = sh.mocap[3 + k];      // normalised by set_controls
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

// Sums over the arm's bodies (lanes 0..5 of each 16-lane DPP row; lanes 6..15 hold zeros): inclusive prefix
// (bodies <= lane) and suffix (bodies >= lane) sums in 3 Hillis-Steele steps, row_shr / row_shl by 1, 2, 4 with
// bound_ctrl (lanes past the row's edge add 0).  Lane l's suffix is ((a_l + a_l+1) + (a_l+2 + a_l+3)) +
// (a_l+4 + a_l+5): the same sums as MuJoCo's serial order (engine_core_smooth.c mj_crb / mj_rne) up to rounding.
// The whole row must be active.
DEV float row_prefix6(float x) {
  x += dpp<0x111>(x);
  x += dpp<0x112>(x);
  return x + dpp<0x114>(x);
}
DEV float row_suffix6(float x) {
  x += dpp<0x101>(x);
  x += dpp<0x102>(x);
  return x + dpp<0x104>(x);
}

// The arm's dynamics on one env's 16-lane row (body a on lane a): comPos, CRBA, the M^-1 columns, RNE and the
// actuation.  The bodies' cinert / cdof / cdof_dot / body forces never leave registers: the tree's prefix and
// suffix sums are DPP scans (round 2 exchanged them through LDS with barriers and summed them serially; round 3
// by 6 row broadcasts per sum, in the serial order).
DEV void dynamics_par(const DevModel* __restrict__ m, EnvShared& sh, int lane, float mscale DSTAMP_PARAMS) {
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
  }
  DSTAMP(2);
  // ---- CRBA: composite inertia crb_i = cin_i + ... + cin_5 by a suffix scan, F_i = crb_i cdof_i; row i of M
  // (j <= i) from the row's cdof_j broadcasts, and its mirror
  {
    float crb[13];
#pragma unroll
    for (int k = 0; k < 13; k++) crb[k] = row_suffix6(cin_r[k]);
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
  // ---- RNE (flg_acc = 0) by prefix / suffix scans: cvel_a = sum_{k<=a} cdof_k qd_k, cdof_dot_a = cvel_a x cdof_a,
  // cacc_a = -g + sum_{k<=a} cdd_k qd_k, the body forces, bias_a = cdof_a . sum_{k>=a} cfrc_k
  const float qd_own = lane < 6 ? sh.qvel[lane] : 0.f;
  float cvel[6], cdd[6], cacc[6];
#pragma unroll
  for (int k = 0; k < 6; k++) cvel[k] = row_prefix6(cdof_r[k] * qd_own);
  cross_motion(cdd, cvel, cdof_r);
#pragma unroll
  for (int k = 0; k < 6; k++) cacc[k] = (k < 3 ? 0.f : -m->gravity[k - 3]) + row_prefix6(cdd[k] * qd_own);
  float cfrc[6];
  {
    float f1[6], Iv[6], f2[6];
    mul_inert(f1, cin_r, cacc);
    mul_inert(Iv, cin_r, cvel);
    cross_force(f2, cvel, Iv);
#pragma unroll
    for (int k = 0; k < 6; k++) cfrc[k] = f1[k] + f2[k];
  }
  float facc[6];                                  // sum_{k>=a} cfrc_k
#pragma unroll
  for (int k = 0; k < 6; k++) facc[k] = row_suffix6(cfrc[k]);
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


}  // namespace so100
