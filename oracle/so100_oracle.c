#include <float.h>
#include <stdio.h>
/* so100_oracle.c — CPU restatement of the SO-ARM100 bin-a-cube hot path (TEST INFRASTRUCTURE).
 *
 * ORACLE ONLY: loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker.  Never linked into the product (gym-so100-c_amd/csrc).  See so100_oracle.h for what is
 * pinned (task logic: golden vectors from the reference) and what is unpinned (MuJoCo physics).
 *
 * Written for clarity, not speed: generic dense matrices (12 dofs), one env per call, stage by stage
 * in MuJoCo's order.  Each stage cites the reference call site that reaches it and the MuJoCo 3.3.3
 * routine it restates ([3P] = third-party algorithm restated from its published behaviour).
 */
#include "so100_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef so100o_real real;
#define NV SO100_NV
#define NB SO100_NBODY
#define NEFC SO100_NEFC_MAX
#define MINVAL ((real)1e-15)
#define MINIMP ((real)0.0001)
#define MAXIMP ((real)0.9999)

/* ============================================================== small linear algebra */
static void cross3(real r[3], const real a[3], const real b[3]) {
  real t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static real dot3(const real a[3], const real b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static real norm3(const real a[3]) { return (real)sqrt((double)dot3(a, a)); }
/* mat: row-major 3x3, columns are the frame axes in world coordinates (MuJoCo xmat) */
static void mulmv3(real r[3], const real m[9], const real v[3]) {
  real t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  real t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  real t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static void mulmtv3(real r[3], const real m[9], const real v[3]) {  /* m' v */
  real t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  real t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  real t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static void mulmm3(real r[9], const real a[9], const real b[9]) {
  real t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  memcpy(r, t, sizeof(t));
}
static void quat_mul(real r[4], const real a[4], const real b[4]) {
  real t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
               a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
               a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
               a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof(t));
}
static void quat_normalize(real q[4]) {
  real n = (real)sqrt((double)(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]));
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
static void quat2mat(real m[9], const real q[4]) {
  real w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z);     m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z);     m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y);     m[7] = 2 * (y * z + w * x);     m[8] = 1 - 2 * (x * x + y * y);
}
static void axis_angle_quat(real q[4], const real axis[3], real ang) {
  real s = (real)sin((double)ang * 0.5);
  q[0] = (real)cos((double)ang * 0.5); q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
static void load3(real r[3], const double v[3]) { r[0] = (real)v[0]; r[1] = (real)v[1]; r[2] = (real)v[2]; }
static void load4(real r[4], const double v[4]) { for (int i = 0; i < 4; i++) r[i] = (real)v[i]; }

/* spatial algebra, MuJoCo convention (angular; linear) — [3P] mju_crossMotion / mju_crossForce */
static void cross_motion(real r[6], const real v[6], const real u[6]) {
  real a[3], b[3], c[3];
  cross3(a, v, u);
  cross3(b, v, u + 3);
  cross3(c, v + 3, u);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
static void cross_force(real r[6], const real v[6], const real f[6]) {
  real a[3], b[3], c[3];
  cross3(a, v, f);
  cross3(b, v + 3, f + 3);
  cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
/* spatial inertia (I about ref point (9), m*d (3), m) times motion vector — [3P] mju_mulInertVec */
static void mul_inert(real r[6], const real in[13], const real v[6]) {
  real Iw[3], mdv[3], mdw[3];
  mulmv3(Iw, in, v);
  cross3(mdv, in + 9, v + 3);
  cross3(mdw, in + 9, v);
  for (int k = 0; k < 3; k++) {
    r[k] = Iw[k] + mdv[k];
    r[3 + k] = in[12] * v[3 + k] - mdw[k];
  }
}

/* ============================================================== task layer (reference, double) */
/* gym_so100/constants.py:44-47 unnormalize + :78-86 unnormalize_so100, applied in
 * single_arm.py:33-38 to a float32 copy: every numpy op runs in float32 (python scalars are weak /
 * value-cast), and the result is written back into the float32 array. */
void so100o_unnormalize(const so100_model* m, const float action[6], float ctrl[6]) {
  for (int i = 0; i < 6; i++) {
    volatile float num = action[i];
    volatile float t = num - (float)(-1);
    volatile float u = t / (float)2;
    volatile float v = u * (float)(m->action_hi[i] - m->action_lo[i]);
    volatile float w = v + (float)m->action_lo[i];
    float lo = (float)m->action_lo[i], hi = (float)m->action_hi[i];
    float c = w < lo ? lo : w;
    c = c > hi ? hi : c;
    ctrl[i] = c;
  }
}

/* numpy legacy RandomState(seed): init_genrand(seed) + mt19937 + 53-bit random_sample, then
 * uniform(low, high) = low + (high-low)*u per component — utils.py:18-29 (sample_so100_box_pose). */
typedef struct { uint32_t mt[624]; int pos; } mt19937;
static void mt_seed(mt19937* s, uint32_t seed) {
  s->mt[0] = seed;
  for (int i = 1; i < 624; i++) s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
  s->pos = 624;
}
static uint32_t mt_next(mt19937* s) {
  if (s->pos >= 624) {
    for (int i = 0; i < 624; i++) {
      uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % 624] & 0x7fffffffu);
      s->mt[i] = s->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    s->pos = 0;
  }
  uint32_t y = s->mt[s->pos++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
static double mt_double(mt19937* s) {
  uint32_t a = mt_next(s) >> 5, b = mt_next(s) >> 6;
  return (a * 67108864.0 + b) / 9007199254740992.0;
}
void so100o_spawn_pose(uint32_t seed, double pose[7]) {
  static const double lo[3] = {-0.25, 0.3, 0.05}, hi[3] = {-0.15, 0.6, 0.05};   /* utils.py:19-21 */
  mt19937 s;
  mt_seed(&s, seed);
  for (int k = 0; k < 3; k++) pose[k] = lo[k] + (hi[k] - lo[k]) * mt_double(&s);
  pose[3] = 1; pose[4] = 0; pose[5] = 0; pose[6] = 0;                              /* utils.py:27 */
}

/* Reward ladders — single_arm.py:322-380 (CubeToBin), :149-215 (TouchCube), :246-285 (Sparse).
 * pair_bits: bit p set iff contact pair p has >= 1 contact (pairs 0..7 = pad-vs-red_box either
 * order -> touch_gripper; pair 8 = ("red_box","table") ordered -> touch_table). */
double so100o_reward(const so100_model* m, int task, const float cube_f32[3], const double cube[3],
                     const double ee[3], uint32_t pair_bits) {
  double bmin[3], bmax[3];
  const double hw = m->bin_hw, h = m->bin_h;                  /* single_arm.py:69-72 */
  bmin[0] = m->bin_center[0] + -hw; bmin[1] = m->bin_center[1] + -hw; bmin[2] = m->bin_center[2] + 0.0;
  bmax[0] = m->bin_center[0] + hw;  bmax[1] = m->bin_center[1] + hw;  bmax[2] = m->bin_center[2] + h;
  int touch_gripper = (pair_bits & ((1u << SO100_NPAIR_GRIPPER) - 1u)) != 0;
  int touch_table = (pair_bits >> SO100_PAIR_TABLE) & 1u;
  if (task == SO100_TASK_CUBE_TO_BIN) {
    /* cube_pos is float32 (get_cube_position :316-320); comparisons promote to float64 */
    double c[3] = {cube_f32[0], cube_f32[1], cube_f32[2]};
    int over = (bmin[0] < c[0] && c[0] < bmax[0]) && (bmin[1] < c[1] && c[1] < bmax[1]);
    int inside = 1;
    const float half = (float)m->cube_half;
    for (int k = 0; k < 3; k++) {
      volatile float lower = cube_f32[k] - half, upper = cube_f32[k] + half;   /* :78-80, float32 */
      inside &= ((double)lower > bmin[k]) && ((double)upper < bmax[k]);
    }
    int released = inside && !touch_gripper;
    double r = 0.0;
    if (touch_gripper) r = 1.0;
    if (touch_gripper && !touch_table) r = 2;
    if (over) r = 2.5;
    if (inside) r = 3;
    if (released) r = 4.0;
    return r;
  }
  double dv[3] = {ee[0] - cube[0], ee[1] - cube[1], ee[2] - cube[2]};
  double dist = sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
  int success = touch_gripper && dist < 0.05;
  if (task == SO100_TASK_TOUCH_CUBE_SPARSE) return success ? m->max_reward : -0.2;
  double r = 0.0;
  if (dist < 0.7) r = fmax(r, 0.1 * (1 - dist / 0.7));
  if (dist < 0.5) r = fmax(r, 0.2 * (1 - dist / 0.5));
  if (dist < 0.3) r = fmax(r, 0.5 * (1 - dist / 0.3));
  if (dist < 0.1) r = fmax(r, 1.0 * (1 - dist / 0.1));
  if (dist < 0.05) r = fmax(r, 2.0 * (1 - dist / 0.05));
  if (touch_gripper) r += 1.0;
  if (success) return m->max_reward;
  r -= 0.2;
  return r;
}

/* ============================================================== physics: position stage */
/* [3P] mj_kinematics: body frames down the tree, hinge rotation about the pre-joint axis,
 * free joint from qpos with normalised quaternion; geom/site frames. */
static void kinematics(const so100_model* m, so100o_data* d) {
  memset(d->xpos[0], 0, sizeof(d->xpos[0]));
  d->xquat[0][0] = 1; d->xquat[0][1] = d->xquat[0][2] = d->xquat[0][3] = 0;
  quat2mat(d->xmat[0], d->xquat[0]);
  for (int b = 1; b < NB; b++) {
    if (b == SO100_CUBE_BODY) {
      for (int k = 0; k < 3; k++) d->xpos[b][k] = d->qpos[6 + k];
      for (int k = 0; k < 4; k++) d->xquat[b][k] = d->qpos[9 + k];
      quat_normalize(d->xquat[b]);
    } else {
      int p = m->body_parent[b];
      real off[3], lq[4], t[3];
      load3(off, m->body_pos[b]);
      load4(lq, m->body_quat[b]);
      mulmv3(t, d->xmat[p], off);
      for (int k = 0; k < 3; k++) d->xpos[b][k] = d->xpos[p][k] + t[k];
      quat_mul(d->xquat[b], d->xquat[p], lq);
      for (int j = 0; j < SO100_NHINGE; j++) {
        if (m->jnt_body[j] != b) continue;
        real ax[3], R[9], qj[4];
        load3(ax, m->jnt_axis[j]);
        quat2mat(R, d->xquat[b]);
        mulmv3(d->xaxis[j], R, ax);
        memcpy(d->xanchor[j], d->xpos[b], sizeof(real) * 3);          /* jnt_pos = 0 */
        axis_angle_quat(qj, ax, d->qpos[j]);                         /* qpos0 = 0 */
        quat_mul(d->xquat[b], d->xquat[b], qj);
      }
      quat_normalize(d->xquat[b]);
    }
    quat2mat(d->xmat[b], d->xquat[b]);
    real ip[3], iq[4], iR[9], t[3];
    load3(ip, m->body_ipos[b]);
    load4(iq, m->body_iquat[b]);
    mulmv3(t, d->xmat[b], ip);
    for (int k = 0; k < 3; k++) d->xipos[b][k] = d->xpos[b][k] + t[k];
    quat2mat(iR, iq);
    mulmm3(d->ximat[b], d->xmat[b], iR);
  }
  /* the mocap body (the EE variant's marker, so_arm100_ee.xml:155): its frame is the mocap pose (mj_kinematics
   * takes mocap_pos and the normalised mocap_quat) */
  real mq[4] = {d->mocap_quat[0], d->mocap_quat[1], d->mocap_quat[2], d->mocap_quat[3]}, mR[9];
  quat_normalize(mq);
  quat2mat(mR, mq);
  for (int g = 0; g < SO100_NGEOM; g++) {
    const int b = m->geom_body[g];
    const real* bp = b == SO100_MOCAP_BODY ? d->mocap_pos : d->xpos[b];
    const real* bR = b == SO100_MOCAP_BODY ? mR : d->xmat[b];
    real gp[3], gq[4], gR[9], t[3];
    load3(gp, m->geom_pos[g]);
    load4(gq, m->geom_quat[g]);
    mulmv3(t, bR, gp);
    for (int k = 0; k < 3; k++) d->geom_xpos[g][k] = bp[k] + t[k];
    quat2mat(gR, gq);
    mulmm3(d->geom_xmat[g], bR, gR);
  }
  real sp[3], t[3];
  load3(sp, m->site_cube_pos);
  mulmv3(t, d->xmat[m->site_cube_body], sp);
  for (int k = 0; k < 3; k++) d->site_cube[k] = d->xpos[m->site_cube_body][k] + t[k];
  load3(sp, m->site_ee_pos);
  mulmv3(t, d->xmat[m->site_ee_body], sp);
  for (int k = 0; k < 3; k++) d->site_ee[k] = d->xpos[m->site_ee_body][k] + t[k];
}

/* tree reference point: the xpos of the tree's root body (Base for the arm, the cube itself).
 * MuJoCo uses subtree_com of the root; M, bias and qacc are invariant to this choice. */
static const real* tree_ref(const so100o_data* d, int b) {
  return b == SO100_CUBE_BODY ? d->xpos[SO100_CUBE_BODY] : d->xpos[1];
}

/* [3P] mj_comPos: cinert (com inertia about the reference point) and cdof (motion subspaces) */
static void com_pos(const so100_model* m, so100o_data* d) {
  for (int b = 1; b < NB; b++) {
    const real* r = tree_ref(d, b);
    real mass = (real)m->body_mass[b], dd[3], Ib[9], Iw[9], diag[9] = {0};
    for (int k = 0; k < 3; k++) dd[k] = d->xipos[b][k] - r[k];
    for (int k = 0; k < 3; k++) diag[4 * k] = (real)m->body_inertia[b][k];
    real RT[9];
    for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) RT[3 * i + j] = d->ximat[b][3 * j + i];
    mulmm3(Ib, d->ximat[b], diag);
    mulmm3(Iw, Ib, RT);
    real dd2 = dot3(dd, dd);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        d->cinert[b][3 * i + j] = Iw[3 * i + j] + mass * ((i == j ? dd2 : 0) - dd[i] * dd[j]);
    for (int k = 0; k < 3; k++) d->cinert[b][9 + k] = mass * dd[k];
    d->cinert[b][12] = mass;
  }
  for (int j = 0; j < SO100_NHINGE; j++) {
    const real* r = tree_ref(d, m->jnt_body[j]);
    real off[3];
    for (int k = 0; k < 3; k++) off[k] = r[k] - d->xanchor[j][k];
    for (int k = 0; k < 3; k++) d->cdof[j][k] = d->xaxis[j][k];
    cross3(d->cdof[j] + 3, d->xaxis[j], off);
  }
  for (int k = 0; k < 3; k++) {          /* free joint: 3 translations (world), 3 rotations (body axes) */
    real* ct = d->cdof[6 + k];
    real* cr = d->cdof[9 + k];
    memset(ct, 0, sizeof(real) * 6);
    ct[3 + k] = 1;
    for (int i = 0; i < 3; i++) cr[i] = d->xmat[SO100_CUBE_BODY][3 * i + k];
    cr[3] = cr[4] = cr[5] = 0;          /* anchor == reference point */
  }
}

static int dof_body(const so100_model* m, int j) { return j < SO100_NHINGE ? m->jnt_body[j] : SO100_CUBE_BODY; }
/* dof ancestry: arm dofs form one chain 0<-1<-...<-5; the 6 free dofs form chain 6<-...<-11 */
static int dof_parent(int j) { return (j == 0 || j == 6) ? -1 : j - 1; }

/* [3P] mj_crb: composite inertias bottom-up, M(i,j) = cdof_j . (crb_i cdof_i) over ancestors */
static void crb(const so100_model* m, so100o_data* d) {
  real crbi[NB][13];
  memcpy(crbi, d->cinert, sizeof(crbi));
  for (int b = NB - 1; b > 1; b--) {
    int p = m->body_parent[b];
    if (p > 0) for (int k = 0; k < 13; k++) crbi[p][k] += crbi[b][k];
  }
  memset(d->qM, 0, sizeof(d->qM));
  for (int i = 0; i < NV; i++) {
    real F[6];
    mul_inert(F, crbi[dof_body(m, i)], d->cdof[i]);
    for (int j = i; j >= 0; j = dof_parent(j)) {
      real v = 0;
      for (int k = 0; k < 6; k++) v += d->cdof[j][k] * F[k];
      d->qM[i][j] = v;
      d->qM[j][i] = v;
    }
    d->qM[i][i] += (real)m->dof_armature[i];
  }
}

/* [3P] mj_factorM: dense Cholesky here (MuJoCo uses sparse LDL'; same solves) */
static void factor_m(so100o_data* d) {
  memset(d->qL, 0, sizeof(d->qL));
  for (int j = 0; j < NV; j++) {
    real s = d->qM[j][j];
    for (int k = 0; k < j; k++) s -= d->qL[j][k] * d->qL[j][k];
    d->qL[j][j] = (real)sqrt((double)(s > MINVAL ? s : MINVAL));
    for (int i = j + 1; i < NV; i++) {
      real t = d->qM[i][j];
      for (int k = 0; k < j; k++) t -= d->qL[i][k] * d->qL[j][k];
      d->qL[i][j] = t / d->qL[j][j];
    }
  }
}
static void solve_m(const so100o_data* d, real x[NV], const real y[NV]) {
  real z[NV];
  for (int i = 0; i < NV; i++) {
    real s = y[i];
    for (int k = 0; k < i; k++) s -= d->qL[i][k] * z[k];
    z[i] = s / d->qL[i][i];
  }
  for (int i = NV - 1; i >= 0; i--) {
    real s = z[i];
    for (int k = i + 1; k < NV; k++) s -= d->qL[k][i] * x[k];
    x[i] = s / d->qL[i][i];
  }
}

/* ---------------------------------------------------------------- box-box narrowphase
 * Separating-axis test over the 15 axes, then (face case) clip the incident face against the
 * reference face and keep every clipped point within the margin, in clip order: up to 8 contacts per
 * pair, as MuJoCo's mjc_BoxBox returns them (no culling to 4: that is ODE's dBoxBox option) [3P-unverified];
 * (edge case) one contact between the closest points of the two edges.  Normal points from geom1
 * to geom2; contact position is midway between the surfaces; dist = -depth. */
static int clip_rect_quad(const real h[2], const real quad[8], real out[16]) {
  real bufa[16], bufb[16];
  real* q = bufa;
  real* r = bufb;
  int nq = 4, nr = 0;
  memcpy(q, quad, sizeof(real) * 8);
  for (int dir = 0; dir < 2; dir++) {
    for (int sign = -1; sign <= 1; sign += 2) {
      nr = 0;
      for (int i = 0; i < nq && nr < 8; i++) {
        const real* a = q + 2 * i;
        const real* b = q + 2 * ((i + 1) % nq);
        int ina = sign * a[dir] < h[dir];
        int inb = sign * b[dir] < h[dir];
        if (ina) { r[2 * nr] = a[0]; r[2 * nr + 1] = a[1]; nr++; }
        if (ina != inb && nr < 8) {
          real lim = sign * h[dir];
          r[2 * nr + 1 - dir] = a[1 - dir] + (b[1 - dir] - a[1 - dir]) / (b[dir] - a[dir]) * (lim - a[dir]);
          r[2 * nr + dir] = lim;
          nr++;
        }
      }
      real* t = q; q = r; r = t;
      nq = nr;
    }
  }
  memcpy(out, q, sizeof(real) * 2 * nq);
  return nq;
}

/* returns number of contacts written (<= SO100_MAXCONPAIR) */
static int box_box(const real p1[3], const real R1[9], const real A[3], const real p2[3], const real R2[9],
                   const real B[3], real margin, real ebias, so100o_contact out[SO100_MAXCONPAIR]) {
  real pd[3], pp[3], R[9], Q[9];
  for (int k = 0; k < 3; k++) pd[k] = p2[k] - p1[k];
  mulmtv3(pp, R1, pd);                               /* p in box1 frame */
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      R[3 * i + j] = R1[i] * R2[j] + R1[3 + i] * R2[3 + j] + R1[6 + i] * R2[6 + j];   /* a1_i . a2_j */
      Q[3 * i + j] = (real)fabs((double)R[3 * i + j]) + (real)1e-6;
    }
  real best = -(real)1e30, nb[3] = {0, 0, 0};       /* nb: best normal in box1 frame (unsigned) */
  int code = 0, invert = 0;
  /* box1 faces */
  for (int i = 0; i < 3; i++) {
    real s = (real)fabs((double)pp[i]) - (A[i] + B[0] * Q[3 * i] + B[1] * Q[3 * i + 1] + B[2] * Q[3 * i + 2]);
    if (s > margin) return 0;
    if (s > best) { best = s; code = 1 + i; invert = pp[i] < 0; nb[0] = nb[1] = nb[2] = 0; nb[i] = 1; }
  }
  /* box2 faces */
  for (int j = 0; j < 3; j++) {
    real e = pp[0] * R[j] + pp[1] * R[3 + j] + pp[2] * R[6 + j];
    real s = (real)fabs((double)e) - (A[0] * Q[j] + A[1] * Q[3 + j] + A[2] * Q[6 + j] + B[j]);
    if (s > margin) return 0;
    if (s > best) { best = s; code = 4 + j; invert = e < 0; nb[0] = R[j]; nb[1] = R[3 + j]; nb[2] = R[6 + j]; }
  }
  /* edge x edge: n = e_i x (R col j), in box1 frame; mjc_BoxBox prefers faces unless an edge axis is clearly better
   * (ebias 1.05); against the table mesh (the convex collider's exact minimum penetration) ebias is 1 */
  for (int i = 0; i < 3; i++) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
    for (int j = 0; j < 3; j++) {
      int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      real n[3] = {0, 0, 0};
      n[i1] = -R[3 * i2 + j];
      n[i2] = R[3 * i1 + j];
      real l = (real)sqrt((double)(n[i1] * n[i1] + n[i2] * n[i2]));
      if (l < (real)1e-5) continue;
      real e = pp[i2] * R[3 * i1 + j] - pp[i1] * R[3 * i2 + j];
      real ex = A[i1] * Q[3 * i2 + j] + A[i2] * Q[3 * i1 + j] + B[j1] * Q[3 * i + j2] + B[j2] * Q[3 * i + j1];
      real s = ((real)fabs((double)e) - ex) / l;
      if (s > margin) return 0;
      if (s * ebias > best) {
        best = s; code = 7 + 3 * i + j; invert = e < 0;
        nb[0] = n[0] / l; nb[1] = n[1] / l; nb[2] = n[2] / l;
      }
    }
  }
  if (code == 0) return 0;
  real normal[3];
  mulmv3(normal, R1, nb);
  if (invert) { normal[0] = -normal[0]; normal[1] = -normal[1]; normal[2] = -normal[2]; }
  const real depth0 = -best;

  if (code > 6) {                                     /* edge-edge: single contact */
    int i = (code - 7) / 3, j = (code - 7) % 3;
    real pa[3], pb[3];
    for (int k = 0; k < 3; k++) { pa[k] = p1[k]; pb[k] = p2[k]; }
    for (int k = 0; k < 3; k++) {
      if (k != i) {
        real ax[3] = {R1[k], R1[3 + k], R1[6 + k]};
        real sgn = dot3(normal, ax) > 0 ? (real)1 : (real)-1;
        for (int t = 0; t < 3; t++) pa[t] += sgn * A[k] * ax[t];
      }
      if (k != j) {
        real ax[3] = {R2[k], R2[3 + k], R2[6 + k]};
        real sgn = dot3(normal, ax) > 0 ? (real)-1 : (real)1;
        for (int t = 0; t < 3; t++) pb[t] += sgn * B[k] * ax[t];
      }
    }
    real ua[3] = {R1[i], R1[3 + i], R1[6 + i]}, ub[3] = {R2[j], R2[3 + j], R2[6 + j]};
    real pq[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
    real uaub = dot3(ua, ub), q1 = dot3(ua, pq), q2 = -dot3(ub, pq);
    real den = 1 - uaub * uaub, al = 0, be = 0;
    if (den > (real)1e-4) { den = 1 / den; al = (q1 + uaub * q2) * den; be = (uaub * q1 + q2) * den; }
    for (int t = 0; t < 3; t++) {
      pa[t] += ua[t] * al;
      pb[t] += ub[t] * be;
      out[0].pos[t] = (real)0.5 * (pa[t] + pb[t]);
      out[0].frame[t] = normal[t];
    }
    out[0].dist = -depth0;
    return 1;
  }

  /* face case: reference box (face axis codeN), incident box */
  const real *pR, *RR, *SR, *pI, *RI, *SI;
  real nref[3];
  int codeN;
  if (code <= 3) { pR = p1; RR = R1; SR = A; pI = p2; RI = R2; SI = B; codeN = code - 1;
                   for (int t = 0; t < 3; t++) nref[t] = normal[t]; }
  else { pR = p2; RR = R2; SR = B; pI = p1; RI = R1; SI = A; codeN = code - 4;
         for (int t = 0; t < 3; t++) nref[t] = -normal[t]; }
  /* incident face: the face of the incident box most anti-parallel to nref */
  real nr[3], anr[3];
  for (int k = 0; k < 3; k++) { real ax[3] = {RI[k], RI[3 + k], RI[6 + k]}; nr[k] = dot3(nref, ax); anr[k] = (real)fabs((double)nr[k]); }
  int lanr = (anr[1] > anr[0]) ? ((anr[1] > anr[2]) ? 1 : 2) : ((anr[0] > anr[2]) ? 0 : 2);
  real center[3];
  for (int t = 0; t < 3; t++) {
    real ax = RI[3 * t + lanr];
    center[t] = pI[t] - pR[t] + (nr[lanr] < 0 ? SI[lanr] : -SI[lanr]) * ax;
  }
  int c1 = (codeN == 0) ? 1 : 0, c2 = (codeN == 2) ? 1 : 2;
  int a1 = (lanr == 0) ? 1 : 0, a2 = (lanr == 2) ? 1 : 2;
  real u1[3] = {RR[c1], RR[3 + c1], RR[6 + c1]}, u2[3] = {RR[c2], RR[3 + c2], RR[6 + c2]};
  real v1[3] = {RI[a1], RI[3 + a1], RI[6 + a1]}, v2[3] = {RI[a2], RI[3 + a2], RI[6 + a2]};
  real cc1 = dot3(center, u1), cc2 = dot3(center, u2);
  real m11 = dot3(u1, v1), m12 = dot3(u1, v2), m21 = dot3(u2, v1), m22 = dot3(u2, v2);
  real k1 = m11 * SI[a1], k2 = m21 * SI[a1], k3 = m12 * SI[a2], k4 = m22 * SI[a2];
  real quad[8] = {cc1 - k1 - k3, cc2 - k2 - k4, cc1 - k1 + k3, cc2 - k2 + k4,
                  cc1 + k1 + k3, cc2 + k2 + k4, cc1 + k1 - k3, cc2 + k2 - k4};
  real rect[2] = {SR[c1], SR[c2]};
  real pts[16];
  int n = clip_rect_quad(rect, quad, pts);
  if (n < 1) return 0;
  real det = m11 * m22 - m12 * m21;
  if (fabs((double)det) < 1e-12) return 0;
  det = 1 / det;
  real i11 = m22 * det, i12 = -m12 * det, i21 = -m21 * det, i22 = m11 * det;
  real P3[8][3], dep[8];
  int cnum = 0;
  for (int k = 0; k < n; k++) {
    real x = pts[2 * k] - cc1, y = pts[2 * k + 1] - cc2;
    real s1 = i11 * x + i12 * y, s2 = i21 * x + i22 * y;
    real pt[3];
    for (int t = 0; t < 3; t++) pt[t] = center[t] + s1 * v1[t] + s2 * v2[t];
    real dp = SR[codeN] - dot3(nref, pt);
    if (dp > -margin) {
      for (int t = 0; t < 3; t++) P3[cnum][t] = pt[t] + pR[t];
      dep[cnum] = dp;
      cnum++;
    }
  }
  if (cnum < 1) return 0;
  for (int c = 0; c < cnum; c++) {
    for (int t = 0; t < 3; t++) {
      out[c].pos[t] = P3[c][t] + (real)0.5 * dep[c] * nref[t];
      out[c].frame[t] = normal[t];
    }
    out[c].dist = -dep[c];
  }
  return cnum;
}

/* test hook (tests/test_oracle_physics.py): the box-box collider on two boxes given by centre, row-major
 * rotation and half sizes; returns the contact count, contacts in out[0..n) (frames: the normal only) */
int so100o_box_box(const so100o_real p1[3], const so100o_real R1[9], const so100o_real A[3], const so100o_real p2[3],
                   const so100o_real R2[9], const so100o_real B[3], so100o_real margin, so100o_contact out[SO100_MAXCONPAIR]) {
  return box_box(p1, R1, A, p2, R2, B, margin, (real)1.05, out);
}

/* [3P] mju_makeFrame: tangents from the normal (y-axis candidate (0,1,0) unless near-parallel) */
static void make_frame(real f[9]) {
  real* n = f;
  real* t1 = f + 3;
  real nn = norm3(n);
  for (int k = 0; k < 3; k++) n[k] /= nn;
  if (fabs((double)n[1]) < 0.5) { t1[0] = 0; t1[1] = 1; t1[2] = 0; }
  else { t1[0] = 0; t1[1] = 0; t1[2] = 1; }
  real pr = dot3(n, t1);
  for (int k = 0; k < 3; k++) t1[k] -= pr * n[k];
  real tn = norm3(t1);
  for (int k = 0; k < 3; k++) t1[k] /= tn;
  cross3(f + 6, n, t1);
}

/* [3P] mj_collision restricted to the in-scope pair table (mj_collideGeoms order: pair order, then
 * contact order within the pair); bounding-sphere broadphase.
 *   pairs 0..13   box-box (box_box above);
 *   pairs 14..22  (table, hull k): an arm/jaw convex hull against the table top.  The
 *     table is a box far larger than any hull, so where a hull dips through the top face inside its
 *     footprint the convex-convex penetration (MuJoCo mjc_Convex, one contact per pair without
 *     multiccd) has the face normal +z, depth = -(lowest vertex z - top), and witness points at that
 *     vertex and its projection on the face: pos = their midpoint.  The lowest vertex is the first in
 *     hull order among ties; vertices outside the top face's x-y footprint are not counted;
 *   pairs 23..97  (box | hull, hull k) through MPR (below);
 *   pairs 98..105 (finger pad i, table): pad_table below, one contact per pair;
 *   pairs 106..145 (finger pad i, bin box j) box-box, like the cube's pairs.  The kernel appends the pad
 *     contacts after the MPR contacts in the same pair order. */
static void add_contact(so100o_data* d, const so100o_contact* c, int p) {
  /* the list has room for every pair at its collider's maximum (SO100_NCON_MAX): nothing is dropped */
  if (d->ncon >= SO100_NCON_MAX) { d->ncon_dropped++; return; }
  so100o_contact* con = &d->con[d->ncon++];
  *con = *c;
  con->pair = p;
  make_frame(con->frame);
}

/* ---------------------------------------------------------------- box vs convex hull (MPR)
 * [3P] MuJoCo mjc_Convex -> libccd ccdMPRPenetration (libccd mpr.c: discoverPortal, refinePortal,
 * findPenetr, findPenetrTouch, findPenetrSegment, findPos, expandPortal, portalDir,
 * portalEncapsulesOrigin, portalReachTolerance, portalCanEncapsuleOrigin; vec3.c
 * ccdVec3PointTriDist2), restated.  MuJoCo 3.3.3 defaults to its native GJK/EPA; this is the libccd
 * path it keeps behind mjDSBL_NATIVECCD (deviation 7).  One contact per pair (no
 * multiccd).  obj1 = the box (geom1), obj2 = hull k (geom2): Minkowski difference obj1 - obj2, centres
 * = geom_xpos (box centre; the mesh's volume centroid).  Supports as mjccd_support: box corner by the
 * sign (>= 0 -> +size) of the direction in the box frame; hull = first vertex of maximal (-d).v.
 * Everything runs in hull k's body frame H, where the vertices are stored; the contact is rotated to
 * the world at the end.  ccd_tolerance 1e-6, ccd_iterations 50 (MuJoCo defaults).  The loops libccd
 * leaves unbounded (discoverPortal's, refinePortal's) stop after the same 50 iterations: no contact. */
#define MPR_TOL ((real)1e-6)
#define EPA_VISTOL ((real)1e-6)
/* the separating-direction cache's certificate: a cached direction must clear the pair by 1 um (kernel kSepTol) */
#define SEP_TOL ((real)1e-6)
#define MPR_ITERS 50
/* libccd's zero/equality tests use MuJoCo's double-precision CCD_EPS (DBL_EPSILON) in both builds: the
 * tests are absolute, and FLT_EPSILON would misclassify mm-scale geometry (e.g. |v0 x v1|^2 ~ 1e-10 read
 * as collinear), sending the fp32 build down different branches than MuJoCo's double libccd */
#define CCD_EPS ((real)2.220446049250313e-16)
typedef struct { real v[3], v1[3], v2[3]; } mpr_sup;
typedef struct {
  int hull1;                     /* obj1: -1 = a box, else a hull (self-collision pairs) */
  real c[3], ax[9], h[3];        /* obj1 frame in H: origin (box centre / hull body origin), axes (columns
                                    of ax); box half sizes */
  const double (*vert1)[3];      /* obj1 hull vertices (its body frame) */
  int nvert1;
  real c1[3];                    /* obj1 centre in H: box centre / hull centroid */
  real bc[3], bh[3];             /* obj1 bounding box in H (axes ax): centre, half extents */
  const double (*vert)[3];       /* obj2 = hull vertices (H) */
  int nvert;
  real hc[3];                    /* hull centroid (H) */
} mpr_obj;

static int ccd_zero(real x) { return (real)fabs((double)x) < CCD_EPS; }
static int ccd_eq(real a, real b) {
  real ab = (real)fabs((double)(a - b));
  if (ab < CCD_EPS) return 1;
  real fa = (real)fabs((double)a), fb = (real)fabs((double)b);
  return fb > fa ? ab < CCD_EPS * fb : ab < CCD_EPS * fa;
}
static void sub3(real r[3], const real a[3], const real b[3]) { for (int t = 0; t < 3; t++) r[t] = a[t] - b[t]; }
static void normalize3(real v[3]) {
  real k = 1 / (real)sqrt((double)dot3(v, v));
  for (int t = 0; t < 3; t++) v[t] *= k;
}
static void mpr_support(const mpr_obj* o, const real d[3], mpr_sup* s) {
  for (int t = 0; t < 3; t++) s->v1[t] = o->c[t];
  if (o->hull1 < 0) {
    for (int i = 0; i < 3; i++) {
      real l = o->ax[i] * d[0] + o->ax[3 + i] * d[1] + o->ax[6 + i] * d[2];
      real sz = l >= 0 ? o->h[i] : -o->h[i];
      for (int t = 0; t < 3; t++) s->v1[t] += sz * o->ax[3 * t + i];
    }
  } else {                       /* obj1 hull: the first vertex maximising (ax' d) . v, back into H */
    real dl[3], best1 = 0, v1[3];
    mulmtv3(dl, o->ax, d);
    int b1 = -1;
    for (int v = 0; v < o->nvert1; v++) {
      real hv[3];
      load3(hv, o->vert1[v]);
      real sc = dot3(dl, hv);
      if (b1 < 0 || sc > best1) { best1 = sc; b1 = v; }
    }
    real hv[3];
    load3(hv, o->vert1[b1]);
    mulmv3(v1, o->ax, hv);
    for (int t = 0; t < 3; t++) s->v1[t] += v1[t];
  }
  real nd[3] = {-d[0], -d[1], -d[2]}, best = 0;
  int bi = -1;
  for (int v = 0; v < o->nvert; v++) {
    real hv[3];
    load3(hv, o->vert[v]);
    real sc = dot3(nd, hv);
    if (bi < 0 || sc > best) { best = sc; bi = v; }
  }
  load3(s->v2, o->vert[bi]);
  sub3(s->v, s->v1, s->v2);
}
static void portal_dir(const mpr_sup P[4], real dir[3]) {
  real a[3], b[3];
  sub3(a, P[2].v, P[1].v);
  sub3(b, P[3].v, P[1].v);
  cross3(dir, a, b);
  normalize3(dir);
}
static int portal_reach_tol(const mpr_sup P[4], const mpr_sup* v4, const real dir[3]) {
  real d4 = dot3(v4->v, dir);
  real d1 = d4 - dot3(P[1].v, dir), d2 = d4 - dot3(P[2].v, dir), d3 = d4 - dot3(P[3].v, dir);
  d1 = d1 < d2 ? d1 : d2;
  d1 = d1 < d3 ? d1 : d3;
  return ccd_eq(d1, MPR_TOL) || d1 < MPR_TOL;
}
static void portal_expand(mpr_sup P[4], const mpr_sup* v4) {
  real v4v0[3];
  cross3(v4v0, v4->v, P[0].v);
  if (dot3(P[1].v, v4v0) > 0) {
    if (dot3(P[2].v, v4v0) > 0) P[1] = *v4; else P[3] = *v4;
  } else {
    if (dot3(P[3].v, v4v0) > 0) P[2] = *v4; else P[1] = *v4;
  }
}
/* -1: no intersection, 0: portal, 1: touching on v1, 2: origin on the segment v0-v1 */
static int mpr_discover(const mpr_obj* o, mpr_sup P[4]) {
  for (int t = 0; t < 3; t++) { P[0].v1[t] = o->c1[t]; P[0].v2[t] = o->hc[t]; }
  sub3(P[0].v, P[0].v1, P[0].v2);
  if (ccd_zero(P[0].v[0]) && ccd_zero(P[0].v[1]) && ccd_zero(P[0].v[2])) P[0].v[0] += CCD_EPS * 10;
  real dir[3] = {-P[0].v[0], -P[0].v[1], -P[0].v[2]}, va[3], vb[3];
  normalize3(dir);
  mpr_support(o, dir, &P[1]);
  real dt = dot3(P[1].v, dir);
  if (ccd_zero(dt) || dt < 0) return -1;
  cross3(dir, P[0].v, P[1].v);
  if (ccd_zero(dot3(dir, dir))) return (ccd_zero(P[1].v[0]) && ccd_zero(P[1].v[1]) && ccd_zero(P[1].v[2])) ? 1 : 2;
  normalize3(dir);
  mpr_support(o, dir, &P[2]);
  dt = dot3(P[2].v, dir);
  if (ccd_zero(dt) || dt < 0) return -1;
  sub3(va, P[1].v, P[0].v);
  sub3(vb, P[2].v, P[0].v);
  cross3(dir, va, vb);
  normalize3(dir);
  if (dot3(dir, P[0].v) > 0) {
    mpr_sup t = P[1]; P[1] = P[2]; P[2] = t;
    for (int k = 0; k < 3; k++) dir[k] = -dir[k];
  }
  for (int it = 0; it < MPR_ITERS; it++) {
    mpr_support(o, dir, &P[3]);
    dt = dot3(P[3].v, dir);
    if (ccd_zero(dt) || dt < 0) return -1;
    int cont = 0;
    cross3(va, P[1].v, P[3].v);
    dt = dot3(va, P[0].v);
    if (dt < 0 && !ccd_zero(dt)) { P[2] = P[3]; cont = 1; }
    if (!cont) {
      cross3(va, P[3].v, P[2].v);
      dt = dot3(va, P[0].v);
      if (dt < 0 && !ccd_zero(dt)) { P[1] = P[3]; cont = 1; }
    }
    if (!cont) return 0;
    sub3(va, P[1].v, P[0].v);
    sub3(vb, P[2].v, P[0].v);
    cross3(dir, va, vb);
    normalize3(dir);
  }
  return -1;
}
static int mpr_refine(const mpr_obj* o, mpr_sup P[4]) {
  for (int it = 0; it < MPR_ITERS; it++) {
    real dir[3];
    portal_dir(P, dir);
    real dt = dot3(dir, P[1].v);
    if (ccd_zero(dt) || dt > 0) return 0;                  /* portal encapsulates the origin */
    mpr_sup v4;
    mpr_support(o, dir, &v4);
    dt = dot3(v4.v, dir);
    if (!(ccd_zero(dt) || dt > 0) || portal_reach_tol(P, &v4, dir)) return -1;
    portal_expand(P, &v4);
  }
  return -1;
}
/* ccdVec3PointTriDist2 / __ccdVec3PointSegmentDist2 with P = origin and a witness point */
static real seg_dist2(const real x0[3], const real b[3], real w[3]) {
  real dd[3], a[3];
  sub3(dd, b, x0);
  for (int t = 0; t < 3; t++) a[t] = x0[t];
  real t = -dot3(a, dd);
  t /= dot3(dd, dd);
  if (t < 0 || ccd_zero(t)) { for (int k = 0; k < 3; k++) w[k] = x0[k]; }
  else if (t > 1 || ccd_eq(t, 1)) { for (int k = 0; k < 3; k++) w[k] = b[k]; }
  else { for (int k = 0; k < 3; k++) w[k] = dd[k] * t + x0[k]; }
  return dot3(w, w);
}
static real tri_dist2(const real x0[3], const real B[3], const real C[3], real w[3]) {
  real d1[3], d2[3], a[3];
  sub3(d1, B, x0);
  sub3(d2, C, x0);
  for (int t = 0; t < 3; t++) a[t] = x0[t];
  real v = dot3(d1, d1), ww = dot3(d2, d2), p = dot3(a, d1), q = dot3(a, d2), r = dot3(d1, d2);
  real det = ww * v - r * r, s, t;
  if (ccd_zero(det)) { s = -1; t = -1; }
  else { s = (q * r - ww * p) / det; t = (-s * r - q) / ww; }
  if ((ccd_zero(s) || s > 0) && (ccd_eq(s, 1) || s < 1) && (ccd_zero(t) || t > 0) && (ccd_eq(t, 1) || t < 1) &&
      (ccd_eq(t + s, 1) || t + s < 1)) {
    for (int k = 0; k < 3; k++) w[k] = x0[k] + d1[k] * s + d2[k] * t;
    return dot3(w, w);
  }
  real w2[3];
  real dist = seg_dist2(x0, B, w);
  real d2b = seg_dist2(x0, C, w2);
  if (d2b < dist) { dist = d2b; memcpy(w, w2, sizeof(w2)); }
  d2b = seg_dist2(B, C, w2);
  if (d2b < dist) { dist = d2b; memcpy(w, w2, sizeof(w2)); }
  return dist;
}
static void mpr_find_pos(const mpr_sup P[4], real pos[3]) {
  real dir[3], vec[3], b[4];
  portal_dir(P, dir);
  cross3(vec, P[1].v, P[2].v); b[0] = dot3(vec, P[3].v);
  cross3(vec, P[3].v, P[2].v); b[1] = dot3(vec, P[0].v);
  cross3(vec, P[0].v, P[1].v); b[2] = dot3(vec, P[3].v);
  cross3(vec, P[2].v, P[1].v); b[3] = dot3(vec, P[0].v);
  real sum = b[0] + b[1] + b[2] + b[3];
  if (ccd_zero(sum) || sum < 0) {
    b[0] = 0;
    cross3(vec, P[2].v, P[3].v); b[1] = dot3(vec, dir);
    cross3(vec, P[3].v, P[1].v); b[2] = dot3(vec, dir);
    cross3(vec, P[1].v, P[2].v); b[3] = dot3(vec, dir);
    sum = b[1] + b[2] + b[3];
  }
  real inv = 1 / sum, p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
  for (int i = 0; i < 4; i++)
    for (int t = 0; t < 3; t++) { p1[t] += P[i].v1[t] * b[i]; p2[t] += P[i].v2[t] * b[i]; }
  for (int t = 0; t < 3; t++) pos[t] = (real)0.5 * (p1[t] * inv + p2[t] * inv);
}
/* ccdMPRPenetration: 1 and (depth, dir obj1 -> obj2, pos) on intersection with a defined normal */
static int mpr_penetration(const mpr_obj* o, real* depth, real dir[3], real pos[3]) {
  mpr_sup P[4];
  memset(P, 0, sizeof(P));
  int res = mpr_discover(o, P);
  if (res < 0) return 0;
  if (res == 1) return 0;                                   /* touching: zero depth, no normal */
  if (res == 2) {                                           /* origin on the segment v0-v1 */
    for (int t = 0; t < 3; t++) { pos[t] = (real)0.5 * (P[1].v1[t] + P[1].v2[t]); dir[t] = P[1].v[t]; }
    *depth = (real)sqrt((double)dot3(dir, dir));
    if (ccd_zero(*depth)) return 0;
    normalize3(dir);
    return 1;
  }
  if (mpr_refine(o, P) < 0) return 0;
  for (int it = 0;; it++) {
    real pd[3];
    portal_dir(P, pd);
    mpr_sup v4;
    mpr_support(o, pd, &v4);
    if (portal_reach_tol(P, &v4, pd) || it > MPR_ITERS) {
      *depth = (real)sqrt((double)tri_dist2(P[1].v, P[2].v, P[3].v, dir));
      if (ccd_zero(*depth)) return 0;                       /* MuJoCo drops a contact without a normal */
      normalize3(dir);
      mpr_find_pos(P, pos);
      return 1;
    }
    portal_expand(P, &v4);
  }
}
/* ---------------------------------------------------------------- convex pairs: GJK + EPA
 * [3P] MuJoCo 3.3.3's default convex collider: mjc_Convex -> the native mjc_ccd (engine_collision_gjk.c), on by
 * default since 3.3.0 (libccd's MPR, above, stays behind mjDSBL_NATIVECCD) [3P-unverified].  GJK decides the
 * overlap and leaves a tetrahedron of Minkowski-difference (A - B) support points enclosing the origin; EPA
 * expands it towards the facet of A - B nearest the origin, which gives the minimum penetration: depth = the
 * facet's distance, normal = its outward normal (geom1 -> geom2), and the witness points from the barycentric
 * coordinates of the origin's projection on the facet; one contact per pair (no multiccd) at the witnesses'
 * midpoint.  Restated from the published algorithms (GJK: Gilbert, Johnson, Keerthi 1988, simplex cases as in
 * van den Bergen 2003; EPA: van den Bergen 2001), with MuJoCo's ccd_tolerance 1e-6 and ccd_iterations 50 for
 * each loop.  MuJoCo's own sub-distance routine (signed volumes) and polytope bookkeeping change the path, not
 * the converged facet.  Supports: mpr_support (box corner by sign, first maximal hull vertex). */
/* polytope bounds: 24 vertices (20 EPA iterations), so at most 2 * 24 - 4 = 44 live faces; the horizon's
 * edge list holds 48 edges.  EPA stops at the current nearest facet when a bound would be passed (the kernel
 * keeps the polytope of a pair in 1 KB of LDS; measured: <= 13 iterations in random-action rollouts, 23 in
 * random folded arm poses, tools/dev/mpr_vs_epa.py) */
#define EPA_MAXV 24
#define EPA_MAXF 44
#define EPA_MAXE 48
typedef struct { int v[3]; real n[3]; real dist; int alive; } epa_face;


/* the simplex's sub-simplex nearest the origin, and the next search direction (towards the origin);
 * returns 1 when the origin is enclosed by the tetrahedron */
static int gjk_simplex(mpr_sup S[4], int* n, real d[3]) {
  real ao[3], ab[3], ac[3], ad[3], t[3], abc[3];
  if (*n == 2) {                                  /* line: A = S[1] (newest), B = S[0] */
    for (int k = 0; k < 3; k++) { ao[k] = -S[1].v[k]; ab[k] = S[0].v[k] - S[1].v[k]; }
    if (dot3(ab, ao) > 0) { cross3(t, ab, ao); cross3(d, t, ab); }
    else { S[0] = S[1]; *n = 1; for (int k = 0; k < 3; k++) d[k] = ao[k]; }
    return 0;
  }
  if (*n == 3) {                                  /* triangle: A = S[2], B = S[1], C = S[0] */
    for (int k = 0; k < 3; k++) { ao[k] = -S[2].v[k]; ab[k] = S[1].v[k] - S[2].v[k]; ac[k] = S[0].v[k] - S[2].v[k]; }
    cross3(abc, ab, ac);
    real e[3];
    cross3(e, abc, ac);                           /* edge AC's outward normal in the plane */
    if (dot3(e, ao) > 0) {
      if (dot3(ac, ao) > 0) { S[1] = S[2]; *n = 2; cross3(t, ac, ao); cross3(d, t, ac); return 0; }
      goto edge_ab;
    }
    cross3(e, ab, abc);                           /* edge AB's outward normal */
    if (dot3(e, ao) > 0) {
    edge_ab:
      if (dot3(ab, ao) > 0) { S[0] = S[1]; S[1] = S[2]; *n = 2; cross3(t, ab, ao); cross3(d, t, ab); return 0; }
      S[0] = S[2]; *n = 1; for (int k = 0; k < 3; k++) d[k] = ao[k];
      return 0;
    }
    if (dot3(abc, ao) > 0) { for (int k = 0; k < 3; k++) d[k] = abc[k]; }
    else {                                        /* below: flip the winding so that abc faces the origin */
      mpr_sup tmp = S[0]; S[0] = S[1]; S[1] = tmp;
      for (int k = 0; k < 3; k++) d[k] = -abc[k];
    }
    return 0;
  }
  /* tetrahedron: A = S[3] (newest), B = S[2], C = S[1], D = S[0]; BCD's winding faces away from A */
  for (int k = 0; k < 3; k++) {
    ao[k] = -S[3].v[k]; ab[k] = S[2].v[k] - S[3].v[k]; ac[k] = S[1].v[k] - S[3].v[k]; ad[k] = S[0].v[k] - S[3].v[k];
  }
  real nabc[3], nacd[3], nadb[3];
  cross3(nabc, ab, ac);
  cross3(nacd, ac, ad);
  cross3(nadb, ad, ab);
  /* orient each face normal away from the fourth vertex */
  if (dot3(nabc, ad) > 0) for (int k = 0; k < 3; k++) nabc[k] = -nabc[k];
  if (dot3(nacd, ab) > 0) for (int k = 0; k < 3; k++) nacd[k] = -nacd[k];
  if (dot3(nadb, ac) > 0) for (int k = 0; k < 3; k++) nadb[k] = -nadb[k];
  if (dot3(nabc, ao) > 0) { S[0] = S[1]; S[1] = S[2]; S[2] = S[3]; *n = 3; return gjk_simplex(S, n, d); }
  if (dot3(nacd, ao) > 0) { S[2] = S[3]; *n = 3; /* D, C, A */ return gjk_simplex(S, n, d); }
  if (dot3(nadb, ao) > 0) { S[1] = S[0]; S[0] = S[2]; S[2] = S[3]; *n = 3; return gjk_simplex(S, n, d); }
  return 1;
}

#ifdef SO100O_STATS
/* dev probe (tools/dev/narrowphase_stats.py): per position stage (candidates, GJK overlaps, contacts, GJK
 * iterations, EPA iterations); single-threaded runs only */
#define SO100O_NSTAT 5
static long so100o_stat_cur[SO100O_NSTAT];
static long* so100o_stat_buf;
static long so100o_stat_n, so100o_stat_cap;
static long *so100o_item_buf, so100o_item_n, so100o_item_cap, so100o_item_mark[2];
void so100o_stats_reset(long* buf, long cap) { so100o_stat_buf = buf; so100o_stat_cap = cap; so100o_stat_n = 0; }
long so100o_stats_count(void) { return so100o_stat_n; }
/* per narrowphase item: GJK iterations, EPA iterations, overlap, contact */
void so100o_items_reset(long* buf, long cap) { so100o_item_buf = buf; so100o_item_cap = cap; so100o_item_n = 0; }
long so100o_items_count(void) { return so100o_item_n; }
static void so100o_item_push(int hit, int sep) {
  if (so100o_item_buf && so100o_item_n < so100o_item_cap) {
    long* r = so100o_item_buf + 4 * so100o_item_n;
    r[0] = so100o_stat_cur[3] - so100o_item_mark[0];
    r[1] = so100o_stat_cur[4] - so100o_item_mark[1];
    r[2] = sep; r[3] = hit;
  }
  so100o_item_n++;
}
#define STAT(k, v) (so100o_stat_cur[k] += (v))
#else
#define STAT(k, v) ((void)0)
#endif

/* GJK: 1 when A - B encloses the origin (S holds the enclosing tetrahedron), 0 otherwise; dsep: (the direction, 1)
 * when the support test proved the pair separated, else w = 0 (the kernels' separating-direction cache) */
static int gjk(const mpr_obj* o, mpr_sup S[4], real dsep[4]) {
  dsep[0] = dsep[1] = dsep[2] = dsep[3] = 0;
  real d[3];
  for (int k = 0; k < 3; k++) d[k] = o->hc[k] - o->c1[k];   /* from the interior point c1 - hc towards the origin */
  if (ccd_zero(dot3(d, d))) d[0] = 1;
  int n = 0;
  for (int it = 0; it < MPR_ITERS; it++) {
    STAT(3, 1);
    real nd = (real)sqrt((double)dot3(d, d));
    if (ccd_zero(nd)) return 0;                    /* the origin on the simplex: touching */
    const real ind = 1 / nd;                       /* one division (the kernel's arithmetic) */
    real du[3] = {d[0] * ind, d[1] * ind, d[2] * ind};
    mpr_sup a;
    mpr_support(o, du, &a);
    if (dot3(a.v, du) <= 0) {                      /* the support does not pass the origin: separated or touching */
      dsep[0] = du[0]; dsep[1] = du[1]; dsep[2] = du[2]; dsep[3] = 1;
      return 0;
    }
    S[n++] = a;
    if (n > 1 && gjk_simplex(S, &n, d)) return 1;
    if (n == 1) for (int k = 0; k < 3; k++) d[k] = -a.v[k];
  }
  return 0;
}

int so100o_epa_debug = 0;     /* tools/dev: print each EPA's final facet */
static int epa_face_set(epa_face* f, const mpr_sup* V, int a, int b, int c) {
  real ab[3], ac[3], n[3];
  sub3(ab, V[b].v, V[a].v);
  sub3(ac, V[c].v, V[a].v);
  cross3(n, ab, ac);
  real l = (real)sqrt((double)dot3(n, n));
  if (ccd_zero(l)) return 0;
  const real il = 1 / l;                                   /* one division (the kernel's arithmetic) */
  for (int k = 0; k < 3; k++) f->n[k] = n[k] * il;
  f->v[0] = a; f->v[1] = b; f->v[2] = c;
  f->dist = dot3(f->n, V[a].v);
  f->alive = 1;
  return 1;
}

/* The contact of EPA's final facet from the features it spans (round 6).  A facet of the Minkowski difference
 * obj1 - obj2 lies on one of its faces: obj1's vertex against obj2's face (one distinct obj1 support, three of obj2),
 * obj1's face against obj2's vertex (three, one), or an edge of each (two, two).  Its witness points, normal and depth
 * are then those features' exact contact — the vertex and its projection on the face plane, or the two edges' closest
 * points with the normal along their cross product — computed from the supports' own coordinates (short edges from
 * the hull's cm-sized vertices; obj1's are its own).  The barycentric interpolation over the facet (the fallback for
 * any other facet) depends on which triangle of the face EPA stopped on, and on a sliver facet (a 1.2 m table edge
 * beside a mm-long hull edge) its fp32 solve lost 1e-2 of the weight along the long edge: the contact moved by
 * centimetres between the fp32 and fp64 restatements (tools/dev/collision_precision.py).  Returns 0 to fall back. */
static int same3(const real a[3], const real b[3]) { return a[0] == b[0] && a[1] == b[1] && a[2] == b[2]; }
static int epa_feature_witness(const mpr_sup* V, const epa_face* f, real* depth, real dir[3], real pos[3]) {
  const mpr_sup* P[3] = {&V[f->v[0]], &V[f->v[1]], &V[f->v[2]]};
  /* distinct supports of each object, in facet order */
  const real* u1[3]; const real* u2[3];
  int n1 = 0, n2 = 0;
  for (int k = 0; k < 3; k++) {
    int seen = 0;
    for (int j = 0; j < n1; j++) seen |= same3(u1[j], P[k]->v1);
    if (!seen) u1[n1++] = P[k]->v1;
    seen = 0;
    for (int j = 0; j < n2; j++) seen |= same3(u2[j], P[k]->v2);
    if (!seen) u2[n2++] = P[k]->v2;
  }
  real nn[3], p1[3], p2[3], e1[3], e2[3];
  if (n1 == 2 && n2 == 2) {                    /* edge (u1[0], u1[1]) of obj1 against edge (u2[0], u2[1]) of obj2 */
    sub3(e1, u1[1], u1[0]);
    sub3(e2, u2[1], u2[0]);
    cross3(nn, e1, e2);
    real w0[3];
    sub3(w0, u1[0], u2[0]);
    const real a = dot3(e1, e1), b = dot3(e1, e2), c = dot3(e2, e2), dd = dot3(e1, w0), e = dot3(e2, w0);
    const real den = a * c - b * b;
    if (!(den > (real)1e-6 * a * c)) return 0;  /* (nearly) parallel edges: no single closest pair */
    const real t = (b * e - c * dd) / den, u = (a * e - b * dd) / den;
    for (int q = 0; q < 3; q++) { p1[q] = u1[0][q] + t * e1[q]; p2[q] = u2[0][q] + u * e2[q]; }
  } else if (n1 == 1 && n2 == 3) {             /* obj1's vertex against obj2's face */
    sub3(e1, u2[1], u2[0]);
    sub3(e2, u2[2], u2[0]);
    cross3(nn, e1, e2);
  } else if (n1 == 3 && n2 == 1) {             /* obj1's face against obj2's vertex */
    sub3(e1, u1[1], u1[0]);
    sub3(e2, u1[2], u1[0]);
    cross3(nn, e1, e2);
  } else {
    return 0;
  }
  const real l = (real)sqrt((double)dot3(nn, nn));
  if (ccd_zero(l)) return 0;
  const real il = (dot3(nn, f->n) < 0 ? -1 : 1) / l;   /* oriented as the facet's outward normal */
  for (int q = 0; q < 3; q++) nn[q] *= il;
  real dep;
  if (n1 == 2) {
    real w[3];
    sub3(w, p1, p2);
    dep = dot3(nn, w);
  } else if (n1 == 1) {
    real w[3];
    sub3(w, u1[0], u2[0]);
    dep = dot3(nn, w);
    for (int q = 0; q < 3; q++) { p1[q] = u1[0][q]; p2[q] = u1[0][q] - dep * nn[q]; }
  } else {
    real w[3];
    sub3(w, u1[0], u2[0]);
    dep = dot3(nn, w);
    for (int q = 0; q < 3; q++) { p2[q] = u2[0][q]; p1[q] = u2[0][q] + dep * nn[q]; }
  }
  if (!(dep > 0) || ccd_zero(dep)) return 0;
  *depth = dep;
  for (int q = 0; q < 3; q++) { dir[q] = nn[q]; pos[q] = (real)0.5 * (p1[q] + p2[q]); }
  return 1;
}

/* EPA from GJK's tetrahedron: 1 and (depth, dir geom1 -> geom2, pos) on the facet reached.  Bookkeeping in
 * the kernel's order (so100_step.hip epa_penetration): faces in slots, the nearest the first alive slot of least
 * distance; a face is visible from w when n . w - dist > 0; the horizon is the visible faces' edges whose twin
 * lies on no visible face, in (slot, edge) order; each horizon edge (a, b) in turn gets the face (a, b, w) in the
 * lowest free slot (a degenerate face takes none). */
static int epa_penetration(const mpr_obj* o, mpr_sup S[4], real* depth, real dir[3], real pos[3], real fn[3]) {
  mpr_sup V[EPA_MAXV];
  epa_face F[EPA_MAXF];
  int nv = 4;
  for (int i = 0; i < EPA_MAXF; i++) F[i].alive = 0;
  for (int i = 0; i < 4; i++) V[i] = S[i];
  static const int tet[4][3] = {{0, 1, 2}, {0, 3, 1}, {0, 2, 3}, {1, 3, 2}};
  for (int i = 0; i < 4; i++) {
    int a = tet[i][0], b = tet[i][1], c = tet[i][2], e = 6 - a - b - c;
    real ab[3], ac[3], n[3], ae[3];
    sub3(ab, V[b].v, V[a].v);
    sub3(ac, V[c].v, V[a].v);
    sub3(ae, V[e].v, V[a].v);
    cross3(n, ab, ac);
    if (dot3(n, ae) > 0) { int t = b; b = c; c = t; }   /* outward: away from the fourth vertex */
    if (!epa_face_set(&F[i], V, a, b, c)) return 0;
  }
  int best = -1;
  for (int it = 0; it < MPR_ITERS; it++) {
    STAT(4, 1);
    best = -1;
    for (int i = 0; i < EPA_MAXF; i++)
      if (F[i].alive && (best < 0 || F[i].dist < F[best].dist)) best = i;
    if (best < 0) return 0;
    mpr_sup w;
    mpr_support(o, F[best].n, &w);
    const real gain = dot3(w.v, F[best].n) - F[best].dist;
    if (gain < MPR_TOL || nv >= EPA_MAXV) break;
    /* the horizon: the edges (a, b) of the visible faces whose twin (b, a) is on no visible face, in (slot, edge)
     * order (the kernel finds them lane-parallel: each lane its slots' edges, the twin test by row ballots) */
    int vis[EPA_MAXF], edges[EPA_MAXE][2], ne = 0, over = 0;
    /* visible only when w clears the facet's plane by more than the ccd_tolerance (a point on the plane within
     * rounding is not visible: no facet folds back over a coplanar one; the kernel's kEpaVisTol) */
    for (int i = 0; i < EPA_MAXF; i++) vis[i] = F[i].alive && dot3(F[i].n, w.v) - F[i].dist > EPA_VISTOL;
    for (int i = 0; i < EPA_MAXF && !over; i++) {
      if (!vis[i]) continue;
      for (int k = 0; k < 3; k++) {
        const int a = F[i].v[k], b = F[i].v[(k + 1) % 3];
        int twin = 0;
        for (int j = 0; j < EPA_MAXF && !twin; j++)
          if (vis[j])
            for (int q = 0; q < 3; q++) twin |= F[j].v[q] == b && F[j].v[(q + 1) % 3] == a;
        if (twin) continue;
        if (ne < EPA_MAXE) { edges[ne][0] = a; edges[ne][1] = b; ne++; }
        else { over = 1; break; }
      }
    }
    if (over) break;                                      /* the horizon does not fit: stop at the nearest facet */
    for (int i = 0; i < EPA_MAXF; i++)
      if (vis[i]) F[i].alive = 0;
    const int iw = nv;
    V[nv++] = w;
    for (int j = 0; j < ne; j++) {
      int slot = -1;
      for (int i = 0; i < EPA_MAXF; i++) if (!F[i].alive) { slot = i; break; }
      if (slot < 0) break;
      epa_face_set(&F[slot], V, edges[j][0], edges[j][1], iw);
    }
  }
  if (best < 0) return 0;
  const epa_face* f = &F[best];
  *depth = f->dist;
  if (ccd_zero(*depth) || *depth < 0) return 0;           /* touching: no normal (as MPR) */
  for (int t = 0; t < 3; t++) fn[t] = f->n[t];             /* the facet's normal (table_face_snap tests it) */
  /* barycentric coordinates of the origin's projection p = n dist on the facet */
  real p[3] = {f->n[0] * f->dist, f->n[1] * f->dist, f->n[2] * f->dist}, l[3];
  {
    const real* a = V[f->v[0]].v; const real* b = V[f->v[1]].v; const real* c = V[f->v[2]].v;
    real v0[3], v1[3], v2[3];
    sub3(v0, b, a); sub3(v1, c, a); sub3(v2, p, a);
    real d00 = dot3(v0, v0), d01 = dot3(v0, v1), d11 = dot3(v1, v1), d20 = dot3(v2, v0), d21 = dot3(v2, v1);
    real den = d00 * d11 - d01 * d01;
    if (ccd_zero(den)) { l[0] = 1; l[1] = 0; l[2] = 0; }
    else { l[1] = (d11 * d20 - d01 * d21) / den; l[2] = (d00 * d21 - d01 * d20) / den; l[0] = 1 - l[1] - l[2]; }
  }
  if (epa_feature_witness(V, f, depth, dir, pos)) return 1;
  if (so100o_epa_debug) {
    fprintf(stderr, "EPA%d facet n %.9g %.9g %.9g dist %.9g l %.6g %.6g %.6g\n", (int)sizeof(real), (double)f->n[0],
            (double)f->n[1], (double)f->n[2], (double)f->dist, (double)l[0], (double)l[1], (double)l[2]);
    for (int k = 0; k < 3; k++)
      fprintf(stderr, "   v1 %.9g %.9g %.9g  v2 %.9g %.9g %.9g\n", (double)V[f->v[k]].v1[0], (double)V[f->v[k]].v1[1],
              (double)V[f->v[k]].v1[2], (double)V[f->v[k]].v2[0], (double)V[f->v[k]].v2[1], (double)V[f->v[k]].v2[2]);
  }
  for (int t = 0; t < 3; t++) {
    real w1 = 0, w2 = 0;
    for (int k = 0; k < 3; k++) { w1 += l[k] * V[f->v[k]].v1[t]; w2 += l[k] * V[f->v[k]].v2[t]; }
    pos[t] = (real)0.5 * (w1 + w2);
    dir[t] = f->n[t];
  }
  return 1;
}

#ifdef SO100O_STATS
/* A filter studied with tools/dev/narrowphase_stats.py (not used by the collider): a box against a hull, separated
 * along one of the box's 3 face axes (the hull's exact projection).  It rejects 60 % of the pairs GJK separates on
 * the bench workload, but in the kernel it cost more than the GJK iterations it saved. */
#define SAT_MARGIN 1e-6
static int box_axes_separate(const mpr_obj* o) {
  if (o->hull1 >= 0) return 0;
  for (int j = 0; j < 3; j++) {
    const real a[3] = {o->ax[j], o->ax[3 + j], o->ax[6 + j]};
    real lo = (real)1e30, hi = (real)-1e30;
    for (int i = 0; i < o->nvert; i++) {
      const real s = (real)o->vert[i][0] * a[0] + (real)o->vert[i][1] * a[1] + (real)o->vert[i][2] * a[2];
      lo = s < lo ? s : lo;
      hi = s > hi ? s : hi;
    }
    const real c = o->c[0] * a[0] + o->c[1] * a[1] + o->c[2] * a[2];
    if (hi < c - o->h[j] - (real)SAT_MARGIN || lo > c + o->h[j] + (real)SAT_MARGIN) return 1;
  }
  return 0;
}
#endif

static int convex_penetration(const so100_model* m, const mpr_obj* o, real* depth, real dir[3], real pos[3],
                              real dsep[4], real fn[3]) {
  dsep[0] = dsep[1] = dsep[2] = dsep[3] = 0;
  if (m->convex == SO100_CONVEX_MPR) {
    const int r = mpr_penetration(o, depth, dir, pos);
    for (int t = 0; t < 3; t++) fn[t] = dir[t];
    return r;
  }
  mpr_sup S[4];
  if (!gjk(o, S, dsep)) return 0;
  STAT(1, 1);
  return epa_penetration(o, S, depth, dir, pos, fn);
}

/* conservative broadphase for (box, hull k) in H: bounding spheres, then OBB-OBB separating axes
 * (the hull's H-aligned bounding box vs the box; |R| padded by 1e-5) */
static int mpr_broadphase(const mpr_obj* o, const real hb[3], const real hh[3]) {
  real T[3];
  sub3(T, o->bc, hb);
  real rs = (real)sqrt((double)dot3(hh, hh)) + (real)sqrt((double)dot3(o->bh, o->bh));
  if (dot3(T, T) > rs * rs) return 0;
  real R[3][3], A[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) { R[i][j] = o->ax[3 * i + j]; A[i][j] = (real)fabs((double)R[i][j]) + (real)1e-5; }
  for (int i = 0; i < 3; i++)
    if ((real)fabs((double)T[i]) > hh[i] + o->bh[0] * A[i][0] + o->bh[1] * A[i][1] + o->bh[2] * A[i][2]) return 0;
  for (int j = 0; j < 3; j++) {
    real s = T[0] * R[0][j] + T[1] * R[1][j] + T[2] * R[2][j];
    if ((real)fabs((double)s) > hh[0] * A[0][j] + hh[1] * A[1][j] + hh[2] * A[2][j] + o->bh[j]) return 0;
  }
  for (int i = 0; i < 3; i++) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
    for (int j = 0; j < 3; j++) {
      const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      real ra = hh[i1] * A[i2][j] + hh[i2] * A[i1][j];
      real rb = o->bh[j1] * A[i][j2] + o->bh[j2] * A[i][j1];
      real s = T[i2] * R[i1][j] - T[i1] * R[i2][j];
      if ((real)fabs((double)s) > ra + rb) return 0;
    }
  }
  return 1;
}

/* one box-box pair (bounding-sphere broadphase, then box_box); pairs 0..13 and the pad-bin pairs.
 * The cube against the table (pair 8, geom2 = the table's mesh, scene_so100.xml:3,20): MuJoCo routes
 * box-mesh through its convex collider (mjc_Convex: native GJK/EPA in 3.3.3), one contact per pair without
 * multiccd (so_arm100.xml:4 sets none) [3P-unverified].  The table mesh is an exact box, so the minimum
 * penetration (normal, depth) is the separating-axis result over all 15 axes (no face preference: ebias 1); the
 * finger pads against the table (pairs 152..159) take the same rule.  The one contact takes the SAT normal, the
 * deepest point's distance, and the mean of the clipped contact positions (the contact patch's centre: the
 * face centre for a cube resting flat).  EPA's own witness point depends on its polytope triangulation and
 * is not restated (DESIGN.md §4 deviation 1). */
static void collide_box_pair(const so100_model* m, so100o_data* d, int p) {
  int g1 = m->pair_geom1[p], g2 = m->pair_geom2[p];
  real A[3], B[3];
  load3(A, m->geom_size[g1]);
  load3(B, m->geom_size[g2]);
  real dp[3] = {d->geom_xpos[g2][0] - d->geom_xpos[g1][0], d->geom_xpos[g2][1] - d->geom_xpos[g1][1],
                d->geom_xpos[g2][2] - d->geom_xpos[g1][2]};
  real margin = (real)m->pair_margin[p];
  if (norm3(dp) > norm3(A) + norm3(B) + margin) return;
  so100o_contact tmp[SO100_MAXCONPAIR];
  /* the table mesh (geom2 = 0): the exact separating-axis minimum (no face preference) */
  int n = box_box(d->geom_xpos[g1], d->geom_xmat[g1], A, d->geom_xpos[g2], d->geom_xmat[g2], B, margin,
                  g2 == 0 ? (real)1 : (real)1.05, tmp);
  if (g2 == 0 && n > 1) {                  /* the table mesh: the convex collider's one contact */
    real sp[3] = {0, 0, 0}, dmin = tmp[0].dist;
    for (int c = 0; c < n; c++) {
      for (int t = 0; t < 3; t++) sp[t] += tmp[c].pos[t];
      if (tmp[c].dist < dmin) dmin = tmp[c].dist;
    }
    for (int t = 0; t < 3; t++) tmp[0].pos[t] = sp[t] / (real)n;
    tmp[0].dist = dmin;
    n = 1;
  }
  for (int c = 0; c < n; c++) add_contact(d, &tmp[c], p);
}

/* A hull-table contact from GJK + EPA whose final facet's normal (wn, world) lies within TABLE_SNAP of one of the table
 * box's face normals
 * (world axes: the table is axis-aligned) is that face's contact: EPA stops within its tolerance of the face normal
 * (1e-6 of the facet distance: normals off by up to ~1e-6 rad), and the witness it interpolates on a Minkowski facet
 * then depends on that residual tilt (a hull corner a centimetre away wins under a 1e-7 rad tilt when the hull lies
 * flat on the face): fp32 and fp64 took different corners (tools/dev/collision_precision.py).  The face's contact is
 * restated exactly: normal the face's axis u (table -> hull), depth the face plane's distance past the hull's extreme
 * vertex along -u, the witness that vertex (the first in hull order among ties, compared in hull-relative
 * coordinates) and its projection on the face: pos their midpoint.  The top-face rule (table_hull_fast) is this on the
 * top face where it is provably the minimum penetration; here EPA has established that the face is. */
#define TABLE_SNAP ((real)1e-5)
static void table_face_snap(const so100_model* m, so100o_data* d, int k, const real wn[3], so100o_contact* con) {
  int ax = 0;
  for (int i = 1; i < 3; i++)
    if ((real)fabs((double)wn[i]) > (real)fabs((double)wn[ax])) ax = i;
  const real off = (real)sqrt((double)(wn[(ax + 1) % 3] * wn[(ax + 1) % 3] + wn[(ax + 2) % 3] * wn[(ax + 2) % 3]));
  if (!(off < TABLE_SNAP)) return;
  const real sgn = wn[ax] > 0 ? (real)1 : (real)-1;
  const int p = SO100_NPAIR_BOX + k, b = m->hull_body[k], g = m->pair_geom1[p];
  const real top = (real)m->table_top, bottom = top - 2 * (real)m->geom_size[g][2];
  const real lo = ax == 2 ? bottom : (real)m->table_lo[ax], hi = ax == 2 ? top : (real)m->table_hi[ax];
  const real face = sgn > 0 ? hi : lo;                     /* the face's coordinate on axis ax */
  const real* R = d->xmat[b];
  /* the hull's support in the body-frame direction -sgn R' e_ax (its first maximal vertex, as mpr_support scans) */
  const real nd[3] = {-sgn * R[3 * ax], -sgn * R[3 * ax + 1], -sgn * R[3 * ax + 2]};
  real best = 0, wb[3] = {0, 0, 0};
  int bi = 0;
  for (int v = 0; v < m->hull_count[k]; v++) {
    real hv[3];
    load3(hv, m->hull_vert[m->hull_start[k] + v]);
    const real sc = dot3(nd, hv);
    if (v == 0 || sc > best) { best = sc; bi = v; }
  }
  {
    real hv[3];
    load3(hv, m->hull_vert[m->hull_start[k] + bi]);
    mulmv3(wb, R, hv);
  }
  for (int t = 0; t < 3; t++) wb[t] += d->xpos[b][t];
  const real dist = sgn * wb[ax] - sgn * face;            /* < 0: the vertex lies past the face, inside the table */
  memset(con->frame, 0, sizeof(con->frame));
  con->frame[ax] = sgn;
  for (int t = 0; t < 3; t++) con->pos[t] = wb[t];
  con->pos[ax] = (real)0.5 * (wb[ax] + face);
  con->dist = dist;
}

/* one convex pair p through the convex collider (GJK + EPA, or MPR), in H = the body frame of hull k (geom2):
 *   23..76 (cube | bin box, hull k); 77..97 (hull k1, hull k2) self-collision of non-adjacent links;
 *   98..106 the static Base hull (the cube, then link hulls 1..8); 107..142 (finger pad, link hull k);
 *   143..151 (EE variant only) the mocap marker box against link hull k;
 *   14..22 (the table, hull k) where the top-face rule is not exact (table_hull_fast).  The table mesh is an exact
 *   box (scene_so100.xml:3,20; geom 0, obj1), so GJK + EPA on it is MuJoCo's mjc_Convex on the mesh. */
static void convex_pair(const so100_model* m, so100o_data* d, int p) {
  const int k = -1 - m->pair_geom2[p], g = m->pair_geom1[p], b = m->hull_body[k];
  const real* RH = d->xmat[b];
  mpr_obj o;
  memset(&o, 0, sizeof(o));
  real dp[3], hb[3], hh[3];
  const real* Rb = g >= 0 ? d->geom_xmat[g] : d->xmat[m->hull_body[-1 - g]];
  sub3(dp, g >= 0 ? d->geom_xpos[g] : d->xpos[m->hull_body[-1 - g]], d->xpos[b]);
  mulmtv3(o.c, RH, dp);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) o.ax[3 * i + j] = RH[i] * Rb[j] + RH[3 + i] * Rb[3 + j] + RH[6 + i] * Rb[6 + j];
  o.hull1 = g >= 0 ? -1 : -1 - g;
  if (g >= 0) {
    load3(o.h, m->geom_size[g]);
    memcpy(o.c1, o.c, sizeof(o.c1));
    memcpy(o.bc, o.c, sizeof(o.bc));
    memcpy(o.bh, o.h, sizeof(o.bh));
  } else {
    const int k1 = o.hull1;
    real t[3], l[3];
    o.vert1 = (const double (*)[3])m->hull_vert[m->hull_start[k1]];
    o.nvert1 = m->hull_count[k1];
    load3(l, m->hull_centroid[k1]);
    mulmv3(t, o.ax, l);
    for (int q = 0; q < 3; q++) o.c1[q] = t[q] + o.c[q];
    load3(l, m->hull_center[k1]);
    mulmv3(t, o.ax, l);
    for (int q = 0; q < 3; q++) o.bc[q] = t[q] + o.c[q];
    load3(o.bh, m->hull_half[k1]);
  }
  o.vert = (const double (*)[3])m->hull_vert[m->hull_start[k]];
  o.nvert = m->hull_count[k];
  load3(o.hc, m->hull_centroid[k]);
  load3(hb, m->hull_center[k]);
  load3(hh, m->hull_half[k]);
  if (!mpr_broadphase(&o, hb, hh)) return;
  STAT(0, 1);
#ifdef SO100O_STATS
  so100o_item_mark[0] = so100o_stat_cur[3]; so100o_item_mark[1] = so100o_stat_cur[4];
#endif
  real depth, dir[3], pos[3];
  /* the kernels' separating-direction cache (so100_convex.h mpr_contacts), when d->sep_on: a direction that proved
   * the pair separated in an earlier substep, re-checked with one support, skips GJK when it still clears the pair
   * by 1e-6; results are unchanged (tests/test_oracle_epa.py::test_separation_cache_changes_nothing) */
  if (d->sep_on && d->sep[p][3] != 0) {
    real du[3] = {d->sep[p][0], d->sep[p][1], d->sep[p][2]};
    mpr_sup a;
    mpr_support(&o, du, &a);
    if (dot3(a.v, du) < -SEP_TOL) { d->sep_hits++; return; }
  }
  real dsep[4], fn[3];
  const int hit_ = convex_penetration(m, &o, &depth, dir, pos, dsep, fn);
  for (int k = 0; k < 4; k++) d->sep[p][k] = dsep[k];
  d->sep_sep += dsep[3] != 0;
#ifdef SO100O_STATS
  so100o_item_push(hit_, box_axes_separate(&o));
#endif
  if (!hit_) return;
  STAT(2, 1);
  so100o_contact con;
  memset(&con, 0, sizeof(con));
  mulmv3(con.frame, RH, dir);
  mulmv3(con.pos, RH, pos);
  for (int t = 0; t < 3; t++) con.pos[t] += d->xpos[b][t];
  con.dist = -depth;
  if (g == 0 && m->convex != SO100_CONVEX_MPR) {
    real wfn[3];
    mulmv3(wfn, RH, fn);
    table_face_snap(m, d, k, wfn, &con);
  }
  add_contact(d, &con, p);
}

/* (table, hull k), pair 14 + k [3P: mjc_Convex on the table mesh, one contact]: the top-face rule where it is provably
 * the exact minimum penetration, else the convex collider.  From the hull's body-frame bounding box (centre c, world
 * extents ex, ey, ez): a candidate when its lowest point zb = c.z - ez is below top + margin.  With D = top - zb, an
 * upper bound of the hull's depth d below the top, the rule applies when every vertex lies inside the top face's x-y
 * footprint shrunk by D (c.x - ex >= lo.x + D, c.x + ex <= hi.x - D, and in y) and the hull's centroid (inside the
 * hull) is at least D above the table's bottom.  Then lifting the hull by d separates it, and any shorter translation
 * t leaves a point of the hull inside the table box (the hull's x-y stays inside the footprint; its z range still
 * reaches below the top and above the bottom, so by convexity some point lies between them): the minimum penetration
 * is d along +z.  The contact is EPA's vertex-face witness pair, the lowest vertex (the first in hull order among
 * ties) and its projection on the top: pos = their midpoint, normal +z (table, geom1 -> hull, geom2).  Otherwise (a
 * hull at the table's edges or side faces, or deep in it) the pair goes through the convex collider after pairs
 * 23..151 (the kernels' order).  Returns 1: contact added, 0: no contact, -1: the convex collider. */
/* test hook (tests/test_oracle_epa.py): nonzero sends every candidate hull-table pair through the convex collider (GJK
 * + EPA + the table face snap) instead of the top-face rule, to check that both give the same contact where the rule
 * applies (the kernel classifies in fp32, the fp64 oracle in fp64, near the rule's bounds) */
int so100o_table_force_slow = 0;
static int table_hull_fast(const so100_model* m, so100o_data* d, int k) {
  const int p = SO100_NPAIR_BOX + k, b = m->hull_body[k], g = m->pair_geom1[p];
  const real top = (real)m->table_top, margin = (real)m->pair_margin[p];
  const real bottom = top - 2 * (real)m->geom_size[g][2];
  const real* R = d->xmat[b];
  real c[3], wc[3], cg[3], wg[3];
  load3(c, m->hull_center[k]);
  mulmv3(wc, R, c);
  real e[3];
  for (int i = 0; i < 3; i++)
    e[i] = (real)fabs((double)R[3 * i]) * (real)m->hull_half[k][0] + (real)fabs((double)R[3 * i + 1]) * (real)m->hull_half[k][1] +
           (real)fabs((double)R[3 * i + 2]) * (real)m->hull_half[k][2];
  const real zb = d->xpos[b][2] + wc[2] - e[2];
  if (!(zb < top + margin)) return 0;
  if (so100o_table_force_slow) return -1;
  load3(cg, m->hull_centroid[k]);
  mulmv3(wg, R, cg);
  const real D = top - zb, cx = d->xpos[b][0] + wc[0], cy = d->xpos[b][1] + wc[1], gz = d->xpos[b][2] + wg[2];
  if (!(cx - e[0] >= (real)m->table_lo[0] + D && cx + e[0] <= (real)m->table_hi[0] - D &&
        cy - e[1] >= (real)m->table_lo[1] + D && cy + e[1] <= (real)m->table_hi[1] - D && gz - bottom >= D)) return -1;
  /* the lowest vertex as the hull's support along world -z in its body frame (its first maximal vertex: hull-relative
   * heights, cm-sized, rounding ~1e-9 m), the body's world position added once after: compared in world z (~0.5 m,
   * rounding 3e-8 m) a hull face lying nearly flat tied its corners, and fp32 rounding picked another lowest corner
   * than fp64, centimetres away (tools/dev/collision_precision.py) */
  const real nd[3] = {-R[6], -R[7], -R[8]};         /* world -z in the body frame: the hull's support along it */
  real sbest = 0;
  int bi = 0;
  for (int v = 0; v < m->hull_count[k]; v++) {
    real hv[3];
    load3(hv, m->hull_vert[m->hull_start[k] + v]);
    const real sc = dot3(nd, hv);
    if (v == 0 || sc > sbest) { sbest = sc; bi = v; }
  }
  real hv[3], w[3];
  load3(hv, m->hull_vert[m->hull_start[k] + bi]);
  mulmv3(w, R, hv);
  const real best = w[2] + d->xpos[b][2], bx = w[0] + d->xpos[b][0], by = w[1] + d->xpos[b][1];
  if (!(best - top < margin)) return 0;
  so100o_contact con;
  memset(&con, 0, sizeof(con));
  con.pos[0] = bx; con.pos[1] = by; con.pos[2] = (real)0.5 * (best + top);
  con.frame[0] = 0; con.frame[1] = 0; con.frame[2] = 1;
  con.dist = best - top;
  add_contact(d, &con, p);
  return 1;
}

static void collision(const so100_model* m, so100o_data* d) {
  d->ncon = 0;
  d->ncon_dropped = 0;
  for (int p = 0; p < SO100_NPAIR_BOX; p++) collide_box_pair(m, d, p);
  /* pairs 14..22 (table, hull k): the top-face rule where it is the exact minimum penetration, else the convex
   * collider (table_hull_fast below) */
  int slow = 0;
  for (int k = 0; k < SO100_NHULL; k++) {
    const int r = table_hull_fast(m, d, k);
    if (r < 0) slow |= 1 << k;
  }
  /* pairs 23..151 through the convex collider, then the table-hull pairs the top-face rule does not cover */
  for (int p = SO100_PAIR_MPR0; p < SO100_PAIR_PAD0; p++) {
    if (p >= SO100_PAIR_MOCAPHULL0 && !m->ee) break;
    convex_pair(m, d, p);
  }
  for (int k = 0; k < SO100_NHULL; k++)
    if ((slow >> k) & 1) convex_pair(m, d, SO100_NPAIR_BOX + k);
  /* pairs 152..199: the finger pads vs the table (152..159: a box against the table mesh, the cube-table rule of
   * collide_box_pair: the separating-axis minimum penetration, one contact), then vs the bin boxes (box-box) */
  for (int p = SO100_PAIR_PAD0; p < SO100_PAIR_PADBIN0; p++) collide_box_pair(m, d, p);
  for (int p = SO100_PAIR_PADBIN0; p < SO100_PAIR_MOCAPBOX0; p++) collide_box_pair(m, d, p);
  /* pairs 200..208 (EE variant only): the cube and the pads against the mocap marker box (box-box) */
  if (m->ee)
    for (int p = SO100_PAIR_MOCAPBOX0; p < SO100_NPAIR; p++) collide_box_pair(m, d, p);
#ifdef SO100O_STATS
  if (so100o_stat_buf && so100o_stat_n < so100o_stat_cap)
    for (int k = 0; k < SO100O_NSTAT; k++) so100o_stat_buf[so100o_stat_n * SO100O_NSTAT + k] = so100o_stat_cur[k];
  so100o_stat_n++;
  memset(so100o_stat_cur, 0, sizeof(so100o_stat_cur));
#endif
}

uint32_t so100o_contact_bits(const so100o_data* d) {
  uint32_t bits = 0;
  for (int c = 0; c < d->ncon; c++)
    if (d->con[c].pair < SO100_NPAIR_BITS) bits |= 1u << d->con[c].pair;
  return bits;
}

/* [3P] engine_core_constraint.c getimpedance: sigmoid between dmin and dmax over |pos-margin|/width */
static real getimpedance(const double solimp[5], real pos, real margin) {
  real dmin = (real)solimp[0], dmax = (real)solimp[1], width = (real)solimp[2];
  real mid = (real)solimp[3], power = (real)solimp[4];
  dmin = dmin < MINIMP ? MINIMP : (dmin > MAXIMP ? MAXIMP : dmin);
  dmax = dmax < MINIMP ? MINIMP : (dmax > MAXIMP ? MAXIMP : dmax);
  mid = mid < MINIMP ? MINIMP : (mid > MAXIMP ? MAXIMP : mid);
  if (power < 1) power = 1;
  if (dmin == dmax || width <= MINVAL) return (real)0.5 * (dmin + dmax);
  real x = (real)fabs((double)((pos - margin) / width));
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  real y;
  if (power == 1) y = x;
  else if (x <= mid) y = (real)(pow((double)x, (double)power) / pow((double)mid, (double)(power - 1)));
  else y = 1 - (real)(pow((double)(1 - x), (double)power) / pow((double)(1 - mid), (double)(power - 1)));
  return dmin + y * (dmax - dmin);
}
static void solref_kb(const double solref[2], const double solimp[5], real timestep, real* K, real* B) {
  real dmax = (real)solimp[1];
  dmax = dmax < MINIMP ? MINIMP : (dmax > MAXIMP ? MAXIMP : dmax);
  real tc = (real)solref[0], dr = (real)solref[1];
  if (tc > 0) {
    if (tc < 2 * timestep) tc = 2 * timestep;                          /* refsafe */
    real den = dmax * dmax * tc * tc * dr * dr;
    *K = 1 / (den > MINVAL ? den : MINVAL);
    real db = dmax * tc;
    *B = 2 / (db > MINVAL ? db : MINVAL);
  } else {
    *K = -tc / (dmax * dmax);
    *B = -dr / dmax;
  }
}

/* [3P] mj_makeConstraint + mj_makeImpedance: rows in MuJoCo order friction | limits | contacts */
static void make_constraint(const so100_model* m, so100o_data* d) {
  int r = 0;
  const real h = (real)m->timestep;
  memset(d->efc_J, 0, sizeof(d->efc_J));
  /* dof frictionloss */
  for (int k = 0; k < NV; k++) {
    if (m->dof_frictionloss[k] <= 0) continue;
    d->efc_type[r] = SO100O_EFC_FRICTION; d->efc_id[r] = k; d->efc_dim[r] = 1;
    d->efc_J[r][k] = 1;
    d->efc_pos[r] = 0; d->efc_margin[r] = 0;
    d->efc_frictionloss[r] = (real)m->dof_frictionloss[k];
    d->efc_diagApprox[r] = (real)m->dof_invweight0[k];
    d->efc_imp[r] = getimpedance(m->dof_solimp, 0, 0);
    solref_kb(m->dof_solref, m->dof_solimp, h, &d->efc_K[r], &d->efc_B[r]);
    r++;
  }
  /* joint limits (hinges; margin 0: active iff dist < 0) */
  for (int j = 0; j < SO100_NHINGE; j++) {
    for (int side = 0; side < 2; side++) {
      real dist = side == 0 ? d->qpos[j] - (real)m->jnt_range[j][0] : (real)m->jnt_range[j][1] - d->qpos[j];
      if (!(dist < 0)) continue;
      d->efc_type[r] = SO100O_EFC_LIMIT; d->efc_id[r] = j; d->efc_dim[r] = 1;
      d->efc_J[r][j] = side == 0 ? 1 : -1;
      d->efc_pos[r] = dist; d->efc_margin[r] = 0; d->efc_frictionloss[r] = 0;
      d->efc_diagApprox[r] = (real)m->dof_invweight0[j];
      d->efc_imp[r] = getimpedance(m->jnt_solimp, dist, 0);
      solref_kb(m->jnt_solref, m->jnt_solimp, h, &d->efc_K[r], &d->efc_B[r]);
      r++;
    }
  }
  /* contacts: elliptic (condim 4 for cube pairs, 3 for hull-table pairs), J rows = frame .
   * (jac(body2) - jac(body1)) at the contact point */
  for (int c = 0; c < d->ncon; c++) {
    const so100o_contact* con = &d->con[c];
    int p = con->pair;
    int b1 = m->pair_body1[p], b2 = m->pair_body2[p];
    real jp[3][NV], jr[3][NV];                     /* jac difference body2 - body1 */
    memset(jp, 0, sizeof(jp)); memset(jr, 0, sizeof(jr));
    for (int side = 0; side < 2; side++) {
      int b = side ? b2 : b1;
      real sg = side ? (real)1 : (real)-1;
      if (b == 0 || b == 1 || b == SO100_MOCAP_BODY) continue;   /* world / static Base / mocap: no dofs */
      if (b == SO100_CUBE_BODY) {
        real off[3];
        for (int t = 0; t < 3; t++) off[t] = con->pos[t] - d->xpos[b][t];
        for (int k = 0; k < 3; k++) {
          jp[k][6 + k] += sg;
          real ax[3] = {d->xmat[b][k], d->xmat[b][3 + k], d->xmat[b][6 + k]}, v[3];
          cross3(v, ax, off);
          for (int t = 0; t < 3; t++) { jp[t][9 + k] += sg * v[t]; jr[t][9 + k] += sg * ax[t]; }
        }
      } else {
        for (int j = 0; j < SO100_NHINGE; j++) {
          int a = b;                                 /* is hinge j an ancestor-or-self of b ? */
          while (a > 1 && a != m->jnt_body[j]) a = m->body_parent[a];
          if (a != m->jnt_body[j]) continue;
          real off[3], v[3];
          for (int t = 0; t < 3; t++) off[t] = con->pos[t] - d->xanchor[j][t];
          cross3(v, d->xaxis[j], off);
          for (int t = 0; t < 3; t++) { jp[t][j] += sg * v[t]; jr[t][j] += sg * d->xaxis[j][t]; }
        }
      }
    }
    const int dim = m->pair_condim[p];
    /* the mocap body is welded to the world for the dynamics: invweight0 = 0 */
    real tran = (real)((b1 == SO100_MOCAP_BODY ? 0 : m->body_invweight0[b1][0]) +
                       (b2 == SO100_MOCAP_BODY ? 0 : m->body_invweight0[b2][0]));
    real rot = (real)((b1 == SO100_MOCAP_BODY ? 0 : m->body_invweight0[b1][1]) +
                      (b2 == SO100_MOCAP_BODY ? 0 : m->body_invweight0[b2][1]));
    real imp = getimpedance(m->pair_solimp[p], con->dist, (real)m->pair_margin[p]);
    real K, B;
    solref_kb(m->pair_solref[p], m->pair_solimp[p], h, &K, &B);
    real mu[3] = {(real)m->pair_friction[p][0], (real)m->pair_friction[p][0], (real)m->pair_friction[p][1]};
    for (int k = 0; k < dim; k++) {
      int row = r + k;
      d->efc_type[row] = SO100O_EFC_CONTACT; d->efc_id[row] = c; d->efc_dim[row] = k == 0 ? dim : 0;
      for (int v = 0; v < NV; v++) {
        if (k < 3) {
          const real* ax = con->frame + 3 * k;
          d->efc_J[row][v] = ax[0] * jp[0][v] + ax[1] * jp[1][v] + ax[2] * jp[2][v];
        } else {
          d->efc_J[row][v] = con->frame[0] * jr[0][v] + con->frame[1] * jr[1][v] + con->frame[2] * jr[2][v];
        }
      }
      d->efc_pos[row] = k == 0 ? con->dist : 0;
      d->efc_margin[row] = k == 0 ? (real)m->pair_margin[p] : 0;
      d->efc_frictionloss[row] = 0;
      d->efc_diagApprox[row] = k < 3 ? tran : rot;
      d->efc_imp[row] = imp;
      d->efc_K[row] = K; d->efc_B[row] = B;
      d->efc_mu[row][0] = mu[0]; d->efc_mu[row][1] = mu[1]; d->efc_mu[row][2] = mu[2];
    }
    r += dim;
  }
  d->nefc = r;
  /* impedance -> regulariser R = (1-imp)/imp * diagApprox; elliptic friction rows:
   * R_j = R_normal * mu_0^2 / (mu_j^2 * impratio) */
  for (int i = 0; i < r; i++) {
    real imp = d->efc_imp[i];
    real Ri = (1 - imp) / imp * d->efc_diagApprox[i];
    d->efc_R[i] = Ri > MINVAL ? Ri : MINVAL;
  }
  for (int i = 0; i < r; i++) {
    if (d->efc_type[i] != SO100O_EFC_CONTACT || d->efc_dim[i] < 2) continue;
    const int dim = d->efc_dim[i];
    for (int k = 1; k < dim; k++) {
      real mk = d->efc_mu[i][k - 1];
      d->efc_R[i + k] = d->efc_R[i] * d->efc_mu[i][0] * d->efc_mu[i][0] / (mk * mk * (real)m->impratio);
    }
  }
  for (int i = 0; i < r; i++) d->efc_D[i] = 1 / d->efc_R[i];
}

/* ============================================================== EE / mocap variant: weld equality */
/* [3P] mju_mat2Quat, then the sign with w >= 0 (the shortest rotation) */
static void mat2quat_pos(real q[4], const real r[9]) {
  const real tr = r[0] + r[4] + r[8];
  if (tr > 0) {
    q[0] = (real)0.5 * (real)sqrt((double)(tr + 1));
    q[1] = (r[7] - r[5]) / (4 * q[0]); q[2] = (r[2] - r[6]) / (4 * q[0]); q[3] = (r[3] - r[1]) / (4 * q[0]);
  } else if (r[0] > r[4] && r[0] > r[8]) {
    q[1] = (real)0.5 * (real)sqrt((double)(1 + r[0] - r[4] - r[8]));
    q[0] = (r[7] - r[5]) / (4 * q[1]); q[2] = (r[1] + r[3]) / (4 * q[1]); q[3] = (r[2] + r[6]) / (4 * q[1]);
  } else if (r[4] > r[8]) {
    q[2] = (real)0.5 * (real)sqrt((double)(1 - r[0] + r[4] - r[8]));
    q[0] = (r[2] - r[6]) / (4 * q[2]); q[1] = (r[1] + r[3]) / (4 * q[2]); q[3] = (r[5] + r[7]) / (4 * q[2]);
  } else {
    q[3] = (real)0.5 * (real)sqrt((double)(1 - r[0] - r[4] + r[8]));
    q[0] = (r[3] - r[1]) / (4 * q[3]); q[1] = (r[2] + r[6]) / (4 * q[3]); q[2] = (r[5] + r[7]) / (4 * q[3]);
  }
  quat_normalize(q);
  if (q[0] < 0) for (int k = 0; k < 4; k++) q[k] = -q[k];
}

/* [3P] mj_makeEquality, mjEQ_WELD (engine_core_constraint.c), for so_arm100_ee.xml:171-173: site1 =
 * mocap_target_site (the mocap body: no dofs), site2 = ee_site (welded to Fixed_Jaw, body 6).
 *   residual  r = (p1 - p2, torquescale * imag(e)),  e = conj(q2) q1 = quat(R2' R1), w >= 0;
 *   Jacobian  J_pos = jacp(mocap, p1) - jacp(ee, p2) = -jacp(ee, p2);
 *             J_rot col j = 0.5 torquescale imag(conj(q2) (0, a_j) q1) = 0.5 ts imag((0, R2' a_j) e),
 *             a_j = jacr(mocap) - jacr(ee) = -axis_j (hinges on the ee body's chain);
 *   impedance of |r_i| (getimpedance), R = (1-imp)/imp * (invweight0(mocap) = 0 + invweight0(ee body)),
 *   aref = -B (J qvel) - K imp r.
 * MuJoCo takes e from the bodies' quaternions as they come (no sign choice); the two agree whenever
 * their product has w >= 0, i.e. for relative rotations below 180 degrees of the tracked branch.
 * The six rows are always active and quadratic (mjCNSTR_EQUALITY), so they are eliminated from the
 * constrained problem exactly: M <- M + J'DJ here and qfrc += J'D aref in the acceleration stage
 * (DESIGN.md §4 deviation 10); the solvers then see the frictionloss, limit and contact rows only. */
static void weld_fold(const so100_model* m, so100o_data* d) {
  const int b = 6;                                                 /* Fixed_Jaw */
  real pos2[3], q2l[4], R2l[9], R2[9], p2[3], t[3];
  load3(pos2, m->weld_pos2);
  load4(q2l, m->weld_quat2);
  quat_normalize(q2l);
  quat2mat(R2l, q2l);
  mulmm3(R2, d->xmat[b], R2l);
  mulmv3(t, d->xmat[b], pos2);
  for (int k = 0; k < 3; k++) p2[k] = d->xpos[b][k] + t[k];
  real q1[4] = {d->mocap_quat[0], d->mocap_quat[1], d->mocap_quat[2], d->mocap_quat[3]}, R1[9], Rr[9], e[4];
  quat_normalize(q1);
  quat2mat(R1, q1);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) Rr[3 * i + j] = R2[i] * R1[j] + R2[3 + i] * R1[3 + j] + R2[6 + i] * R1[6 + j];
  mat2quat_pos(e, Rr);
  const real ts = (real)m->weld_torquescale;
  for (int k = 0; k < 3; k++) { d->weld_pos[k] = d->mocap_pos[k] - p2[k]; d->weld_pos[3 + k] = ts * e[1 + k]; }
  memset(d->weld_J, 0, sizeof(d->weld_J));
  for (int j = 0; j < SO100_NHINGE; j++) {
    if (m->jnt_body[j] > b) continue;                              /* the Jaw hinge is not on the chain */
    const real* ax = d->xaxis[j];
    real dp[3] = {p2[0] - d->xanchor[j][0], p2[1] - d->xanchor[j][1], p2[2] - d->xanchor[j][2]}, c[3];
    cross3(c, ax, dp);
    real a[3] = {-ax[0], -ax[1], -ax[2]}, v[3], vc[3];
    mulmtv3(v, R2, a);
    cross3(vc, v, e + 1);
    for (int k = 0; k < 3; k++) {
      d->weld_J[k][j] = -c[k];
      d->weld_J[3 + k][j] = (real)0.5 * ts * (e[0] * v[k] + vc[k]);
    }
  }
  real K, B;
  solref_kb(m->weld_solref, m->weld_solimp, (real)m->timestep, &K, &B);
  for (int i = 0; i < 6; i++) {
    real vel = 0;
    for (int j = 0; j < SO100_NV; j++) vel += d->weld_J[i][j] * d->qvel[j];
    const real imp = getimpedance(m->weld_solimp, d->weld_pos[i], 0);
    real R = (1 - imp) / imp * (real)m->weld_invweight0[i < 3 ? 0 : 1];
    R = R > MINVAL ? R : MINVAL;
    d->weld_D[i] = 1 / R;
    d->weld_aref[i] = -B * vel - K * imp * d->weld_pos[i];
  }
  for (int i = 0; i < SO100_NV; i++) {
    real f = 0;
    for (int r = 0; r < 6; r++) f += d->weld_J[r][i] * d->weld_D[r] * d->weld_aref[r];
    d->weld_f[i] = f;
    for (int j = 0; j <= i; j++) {
      real v = 0;
      for (int r = 0; r < 6; r++) v += d->weld_J[r][i] * d->weld_D[r] * d->weld_J[r][j];
      d->qM[i][j] += v;
      if (j != i) d->qM[j][i] += v;
    }
  }
}

void so100o_fwd_position(const so100_model* m, so100o_data* d) {
  kinematics(m, d);
  com_pos(m, d);
  crb(m, d);
  if (m->ee) weld_fold(m, d);
  else memset(d->weld_f, 0, sizeof(d->weld_f));
  factor_m(d);
  collision(m, d);
  make_constraint(m, d);
}

/* ============================================================== physics: velocity stage */
/* [3P] mj_comVel (incl. the free-joint cdof_dot special case) + mj_rne(flg_acc=0) */
void so100o_fwd_velocity(const so100_model* m, so100o_data* d) {
  memset(d->cvel, 0, sizeof(d->cvel));
  for (int b = 1; b < NB; b++) {
    int p = m->body_parent[b];
    for (int k = 0; k < 6; k++) d->cvel[b][k] = d->cvel[p][k];
    if (b == SO100_CUBE_BODY) {
      for (int j = 6; j < 9; j++) {
        memset(d->cdof_dot[j], 0, sizeof(real) * 6);
        for (int k = 0; k < 6; k++) d->cvel[b][k] += d->cdof[j][k] * d->qvel[j];
      }
      for (int j = 9; j < 12; j++) cross_motion(d->cdof_dot[j], d->cvel[b], d->cdof[j]);
      for (int j = 9; j < 12; j++) for (int k = 0; k < 6; k++) d->cvel[b][k] += d->cdof[j][k] * d->qvel[j];
    } else {
      for (int j = 0; j < SO100_NHINGE; j++) {
        if (m->jnt_body[j] != b) continue;
        for (int k = 0; k < 6; k++) d->cvel[b][k] += d->cdof[j][k] * d->qvel[j];
        cross_motion(d->cdof_dot[j], d->cvel[b], d->cdof[j]);
      }
    }
  }
  /* RNE */
  real cacc[NB][6], cfrc[NB][6];
  memset(cacc, 0, sizeof(cacc));
  for (int k = 0; k < 3; k++) cacc[0][3 + k] = -(real)m->gravity[k];
  for (int b = 1; b < NB; b++) {
    int p = m->body_parent[b];
    for (int k = 0; k < 6; k++) cacc[b][k] = cacc[p][k];
    for (int j = 0; j < NV; j++)
      if (dof_body(m, j) == b) for (int k = 0; k < 6; k++) cacc[b][k] += d->cdof_dot[j][k] * d->qvel[j];
    real f1[6], Iv[6], f2[6];
    mul_inert(f1, d->cinert[b], cacc[b]);
    mul_inert(Iv, d->cinert[b], d->cvel[b]);
    cross_force(f2, d->cvel[b], Iv);
    for (int k = 0; k < 6; k++) cfrc[b][k] = f1[k] + f2[k];
  }
  for (int b = NB - 1; b > 0; b--) {
    int p = m->body_parent[b];
    if (p > 0) for (int k = 0; k < 6; k++) cfrc[p][k] += cfrc[b][k];
  }
  for (int j = 0; j < NV; j++) {
    real v = 0;
    for (int k = 0; k < 6; k++) v += d->cdof[j][k] * cfrc[dof_body(m, j)][k];
    d->qfrc_bias[j] = v;
  }
  for (int i = 0; i < d->nefc; i++) {
    real v = 0;
    for (int k = 0; k < NV; k++) v += d->efc_J[i][k] * d->qvel[k];
    d->efc_vel[i] = v;
  }
}

/* ============================================================== physics: acceleration stage */
/* [3P] mj_QCQP2/3: min 0.5 x'Ax + x'b  s.t. sum (x_i/d_i)^2 <= r^2, Newton on the multiplier */
static int qcqp(int n, real x[3], const real Ain[3][3], const real bin[3], const real dd[3], real r) {
  real A[3][3], b[3], y[3], la = 0;
  for (int i = 0; i < n; i++) {
    b[i] = bin[i] * dd[i];
    for (int j = 0; j < n; j++) A[i][j] = Ain[i][j] * dd[i] * dd[j];
  }
  for (int it = 0; it < 20; it++) {
    real P[3][3], Pi[3][3];
    for (int i = 0; i < n; i++) for (int j = 0; j < n; j++) P[i][j] = A[i][j] + (i == j ? la : 0);
    real det;
    if (n == 2) {
      det = P[0][0] * P[1][1] - P[0][1] * P[1][0];
      if (det < MINVAL) { for (int i = 0; i < n; i++) x[i] = 0; return 0; }
      real id = 1 / det;
      Pi[0][0] = P[1][1] * id; Pi[1][1] = P[0][0] * id; Pi[0][1] = -P[0][1] * id; Pi[1][0] = -P[1][0] * id;
    } else {
      Pi[0][0] = P[1][1] * P[2][2] - P[1][2] * P[2][1];
      Pi[0][1] = P[0][2] * P[2][1] - P[0][1] * P[2][2];
      Pi[0][2] = P[0][1] * P[1][2] - P[0][2] * P[1][1];
      Pi[1][0] = P[1][2] * P[2][0] - P[1][0] * P[2][2];
      Pi[1][1] = P[0][0] * P[2][2] - P[0][2] * P[2][0];
      Pi[1][2] = P[0][2] * P[1][0] - P[0][0] * P[1][2];
      Pi[2][0] = P[1][0] * P[2][1] - P[1][1] * P[2][0];
      Pi[2][1] = P[0][1] * P[2][0] - P[0][0] * P[2][1];
      Pi[2][2] = P[0][0] * P[1][1] - P[0][1] * P[1][0];
      det = P[0][0] * Pi[0][0] + P[0][1] * Pi[1][0] + P[0][2] * Pi[2][0];
      if (det < MINVAL) { for (int i = 0; i < n; i++) x[i] = 0; return 0; }
      real id = 1 / det;
      for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) Pi[i][j] *= id;
    }
    for (int i = 0; i < n; i++) {
      real s = 0;
      for (int j = 0; j < n; j++) s -= Pi[i][j] * b[j];
      y[i] = s;
    }
    real yy = 0;
    for (int i = 0; i < n; i++) yy += y[i] * y[i];
    real val = yy - r * r;
    if (val < (real)1e-10) break;
    real Py[3], deriv = 0;
    for (int i = 0; i < n; i++) { Py[i] = 0; for (int j = 0; j < n; j++) Py[i] += Pi[i][j] * y[j]; }
    for (int i = 0; i < n; i++) deriv += y[i] * Py[i];
    deriv *= -2;
    real delta = -val / deriv;
    if (delta < (real)1e-10) break;
    la += delta;
  }
  for (int i = 0; i < n; i++) x[i] = y[i] * dd[i];
  return la != 0;
}

/* [3P] mj_constraintUpdate (dual force from jar = J qacc - aref), used for the PGS warmstart */
static void force_from_jar(const so100_model* m, const so100o_data* d, const real* jar, real* f) {
  for (int i = 0; i < d->nefc;) {
    int t = d->efc_type[i];
    if (t == SO100O_EFC_FRICTION) {
      real fl = d->efc_frictionloss[i], R = d->efc_R[i];
      if (jar[i] <= -R * fl) f[i] = fl;
      else if (jar[i] >= R * fl) f[i] = -fl;
      else f[i] = -d->efc_D[i] * jar[i];
      i++;
    } else if (t == SO100O_EFC_LIMIT) {
      f[i] = jar[i] < 0 ? -d->efc_D[i] * jar[i] : 0;
      i++;
    } else {
      int dim = d->efc_dim[i];
      real mu = d->efc_mu[i][0] * (real)sqrt((double)(d->efc_R[i + 1] / d->efc_R[i]));
      real U[4], T = 0;
      U[0] = jar[i] * mu;
      for (int k = 1; k < dim; k++) { U[k] = jar[i + k] * d->efc_mu[i][k - 1]; T += U[k] * U[k]; }
      T = (real)sqrt((double)T);
      real N = U[0];
      if (N >= mu * T || (T <= 0 && N >= 0)) {
        for (int k = 0; k < dim; k++) f[i + k] = 0;
      } else if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
        for (int k = 0; k < dim; k++) f[i + k] = -d->efc_D[i + k] * jar[i + k];
      } else {
        real Dm = d->efc_D[i] / (mu * mu * (1 + mu * mu));
        real NmT = N - mu * T;
        f[i] = -Dm * NmT * mu;
        for (int k = 1; k < dim; k++) f[i + k] = -f[i] / T * U[k] * d->efc_mu[i][k - 1];
      }
      i += dim;
    }
  }
}

/* [3P] mj_solPGS: projected Gauss-Seidel on the dual, elliptic contact blocks (normal first, then
 * friction by QCQP), improvement-based termination scaled by 1/(meaninertia*nv). */
static void sol_pgs(const so100_model* m, so100o_data* d, const real* AR) {
  const int nefc = d->nefc;
  real* f = d->efc_force;
  const real scale = 1 / ((real)m->meaninertia * (real)NV);
  d->solver_iter = 0;
  d->solver_improvement = 0;
  for (int it = 0; it < m->iterations; it++) {
    real improvement = 0;
    for (int i = 0; i < nefc;) {
      int dim = d->efc_type[i] == SO100O_EFC_CONTACT ? d->efc_dim[i] : 1;
      real res[4], old[4];
      for (int k = 0; k < dim; k++) {
        real s = d->efc_b[i + k];
        for (int j = 0; j < nefc; j++) s += AR[(size_t)(i + k) * nefc + j] * f[j];
        res[k] = s;
        old[k] = f[i + k];
      }
      if (dim == 1) {
        f[i] -= res[0] / AR[(size_t)i * nefc + i];
        if (d->efc_type[i] == SO100O_EFC_FRICTION) {
          real fl = d->efc_frictionloss[i];
          f[i] = f[i] < -fl ? -fl : (f[i] > fl ? fl : f[i]);
        } else if (f[i] < 0) {
          f[i] = 0;
        }
      } else {
        f[i] -= res[0] / AR[(size_t)i * nefc + i];
        if (f[i] < MINVAL) {
          f[i] = 0;
          for (int k = 1; k < dim; k++) f[i + k] = 0;
        } else {
          real Af[3][3], bf[3], x[3];
          int nf = dim - 1;
          for (int a = 0; a < nf; a++) {
            bf[a] = res[1 + a] + AR[(size_t)(i + 1 + a) * nefc + i] * (f[i] - old[0]);
            for (int c = 0; c < nf; c++) {
              Af[a][c] = AR[(size_t)(i + 1 + a) * nefc + i + 1 + c];
              bf[a] -= Af[a][c] * old[1 + c];
            }
          }
          qcqp(nf, x, Af, bf, d->efc_mu[i], f[i]);
          for (int a = 0; a < nf; a++) f[i + 1 + a] = x[a];
        }
      }
      real delta[4];
      for (int k = 0; k < dim; k++) delta[k] = f[i + k] - old[k];
      for (int k = 0; k < dim; k++) {
        real q = 0;
        for (int c = 0; c < dim; c++) q += AR[(size_t)(i + k) * nefc + i + c] * delta[c];
        improvement -= delta[k] * (res[k] + (real)0.5 * q);
      }
      i += dim;
    }
    improvement *= scale;
    d->solver_iter = it + 1;
    d->solver_improvement = improvement;
    if (improvement < (real)m->tolerance) break;
  }
}

/* ---------------------------------------------------------------- primal Newton solver
 * [3P] mj_solNewton (engine_solver.c mj_solPrimal with flg_Newton), restated: minimise the convex
 *   c(a) = 1/2 (a - a_smooth)' M (a - a_smooth) + sum_b s_b(J_b a - aref_b)
 * over qacc a, where s_b is the soft-constraint cost of block b (mj_constraintUpdate, primal): dof
 * frictionloss (quadratic inside |jar| < R f, linear outside), joint limits (quadratic when jar < 0),
 * elliptic contacts (top zone 0, bottom zone quadratic, middle zone 1/2 Dm (N - mu T)^2).  Newton
 * direction from the Cholesky of H = M + sum_b J_b' H_b J_b (H_b: the block's cost Hessian in jar,
 * including the middle-zone cone Hessian), exact line search, MuJoCo's termination: scale * (old cost -
 * new cost) < tolerance or scale * |grad| < tolerance, scale = 1 / (meaninertia nv); alpha = 0 stops.
 * The start is qacc_warmstart if its cost is below qacc_smooth's (mj_fwdConstraint).  The line search
 * is ours (a safeguarded 1-D Newton on c'(alpha) to relative precision; MuJoCo brackets to ls_tolerance
 * 0.01), so the iterates differ from MuJoCo's path but converge to the same unique minimiser. */
/* Precision-dependent stops.  fp64 (the checker): the line search to |c'| <= 1e-12 |c'(0)|, MuJoCo's outer tests only.
 * fp32 (the GPU's arithmetic, mirrored by so100_newton.h): MuJoCo's ls_tolerance 0.01, a relative step stop 1e-4 (fp32
 * cannot resolve c' near the minimum: the search otherwise ran 14 evaluations), and the Newton decrement: with the
 * direction s = -H^-1 g in hand, a full step would lower the cost by -g's/2, and the solve stops when that (scaled) is
 * below MuJoCo's tolerance.  MuJoCo's own stops are below fp32's resolution there (scale |g| never reaches 1e-8 under
 * fp32 rounding of g, and the cost difference is noise at 1e-8), and rounds 3-5 stopped at a relative cost improvement
 * of 1e-6 instead, which on the EE variant (the weld folded into M: a large cost) ended solves short of the minimiser:
 * EE qvel p90 5e-4 against fp64 (tools/dev/mixed_precision.py).  The decrement resolves where fp32 can (g's noise
 * enters squared) and matches fp64's iteration counts: 1.20 line searches per substep on the bench workload
 * (fp64 1.22, the relative stop 1.88), EE qvel p90 2.5e-5.  (NEWTON_GNOISE k, measured and not kept: stop at an
 * iteration's start when every gradient component lies within k float epsilons of its terms' magnitudes, before the
 * Hessian: 2.15 -> 1.34 factorizations per substep on the bench workload at k = 16, but blind to the curvature: on
 * the GPU the deep Base folds' qvel p99 went 1.8e-3 -> 1.4e-2) */
#if defined(SO100O_FLOAT) && !defined(LS_TOL)
#define LS_TOL ((real)1e-2)
#define LS_STEP ((real)1e-4)
#define NEWTON_DECREMENT 1
#define NEWTON_GNOISE 0
#define NEWTON_QUADSTOP 1
#elif !defined(LS_TOL)
#define LS_TOL ((real)1e-12)
#define LS_STEP ((real)0)
#define NEWTON_DECREMENT 0
#define NEWTON_GNOISE 0
#define NEWTON_QUADSTOP 0
#endif

/* cost, force (= -d cost / d jar) and cost Hessian of the constraint block at row i; returns its rows */
static int block_eval(const so100o_data* d, int i, const real* jar, real* cost, real f[4], real H[4][4]) {
  memset(f, 0, sizeof(real) * 4);
  memset(H, 0, sizeof(real) * 16);
  *cost = 0;
  const int t = d->efc_type[i];
  if (t == SO100O_EFC_FRICTION) {
    const real fl = d->efc_frictionloss[i], R = d->efc_R[i], D = d->efc_D[i], x = jar[0];
    if (x >= R * fl) { f[0] = -fl; *cost = fl * x - (real)0.5 * R * fl * fl; }
    else if (x <= -R * fl) { f[0] = fl; *cost = -fl * x - (real)0.5 * R * fl * fl; }
    else { f[0] = -D * x; *cost = (real)0.5 * D * x * x; H[0][0] = D; }
    return 1;
  }
  if (t == SO100O_EFC_LIMIT) {
    const real D = d->efc_D[i], x = jar[0];
    if (x < 0) { f[0] = -D * x; *cost = (real)0.5 * D * x * x; H[0][0] = D; }
    return 1;
  }
  const int dim = d->efc_dim[i];
  const real mu = d->efc_mu[i][0] * (real)sqrt((double)(d->efc_R[i + 1] / d->efc_R[i]));
  real U[4], T = 0;
  U[0] = jar[0] * mu;
  for (int k = 1; k < dim; k++) { U[k] = jar[k] * d->efc_mu[i][k - 1]; T += U[k] * U[k]; }
  T = (real)sqrt((double)T);
  const real N = U[0];
  if (N >= mu * T || (T <= 0 && N >= 0)) return dim;                       /* top zone */
  if (mu * N + T <= 0 || (T <= 0 && N < 0)) {                              /* bottom zone */
    for (int k = 0; k < dim; k++) {
      const real D = d->efc_D[i + k];
      f[k] = -D * jar[k];
      *cost += (real)0.5 * D * jar[k] * jar[k];
      H[k][k] = D;
    }
    return dim;
  }
  /* middle zone: c = 1/2 Dm (N - mu T)^2 with g = d(N - mu T)/d jar */
  const real Dm = d->efc_D[i] / (mu * mu * (1 + mu * mu)), NmT = N - mu * T;
  real g[4];
  g[0] = mu;
  for (int k = 1; k < dim; k++) g[k] = -mu * U[k] * d->efc_mu[i][k - 1] / T;
  *cost = (real)0.5 * Dm * NmT * NmT;
  for (int k = 0; k < dim; k++) f[k] = -Dm * NmT * g[k];
  for (int k = 0; k < dim; k++)
    for (int l = 0; l < dim; l++) H[k][l] = Dm * g[k] * g[l];
  for (int k = 1; k < dim; k++)
    for (int l = 1; l < dim; l++) {
      const real fk = d->efc_mu[i][k - 1], fl = d->efc_mu[i][l - 1];
      H[k][l] -= Dm * NmT * mu * fk * fl * ((k == l ? 1 / T : 0) - U[k] * U[l] / (T * T * T));
    }
  return dim;
}

/* total cost at jar (+ Gauss term given separately); forces into f (nefc) */
static real constraint_cost(const so100o_data* d, const real* jar, real* f) {
  real c = 0;
  for (int i = 0; i < d->nefc;) {
    real cb, fb[4], Hb[4][4];
    const int n = block_eval(d, i, jar + i, &cb, fb, Hb);
    for (int k = 0; k < n; k++) f[i + k] = fb[k];
    c += cb;
    i += n;
  }
  return c;
}
static real gauss_cost(const so100o_data* d, const real a[NV]) {
  real e[NV], c = 0;
  for (int k = 0; k < NV; k++) e[k] = a[k] - d->qacc_smooth[k];
  for (int i = 0; i < NV; i++)
    for (int j = 0; j < NV; j++) c += (real)0.5 * e[i] * d->qM[i][j] * e[j];
  return c;
}
static void jar_at(const so100o_data* d, const real a[NV], real* jar) {
  for (int i = 0; i < d->nefc; i++) {
    real s = 0;
    for (int k = 0; k < NV; k++) s += d->efc_J[i][k] * a[k];
    jar[i] = s - d->efc_aref[i];
  }
}
/* dense Cholesky solve H x = b (H SPD); returns 0 if not positive definite */
static int chol_solve(real H[NV][NV], const real b[NV], real x[NV]) {
  real L[NV][NV];
  memset(L, 0, sizeof(L));
  for (int j = 0; j < NV; j++) {
    real s = H[j][j];
    for (int k = 0; k < j; k++) s -= L[j][k] * L[j][k];
    if (!(s > 0)) return 0;
    L[j][j] = (real)sqrt((double)s);
    for (int i = j + 1; i < NV; i++) {
      real t = H[i][j];
      for (int k = 0; k < j; k++) t -= L[i][k] * L[j][k];
      L[i][j] = t / L[j][j];
    }
  }
  real y[NV];
  for (int i = 0; i < NV; i++) {
    real s = b[i];
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
  for (int i = NV - 1; i >= 0; i--) {
    real s = y[i];
    for (int k = i + 1; k < NV; k++) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
  return 1;
}
/* c'(alpha), c''(alpha) along a + alpha s (e = a - a_smooth, Js = J s precomputed) */
static void line_derivs(const so100o_data* d, const real e[NV], const real s[NV], const real* jar0, const real* Js,
                        real alpha, real* d1, real* d2) {
  real Ms[NV], g1 = 0, g2 = 0;
  for (int i = 0; i < NV; i++) {
    real t = 0;
    for (int j = 0; j < NV; j++) t += d->qM[i][j] * s[j];
    Ms[i] = t;
  }
  for (int i = 0; i < NV; i++) { g1 += Ms[i] * (e[i] + alpha * s[i]); g2 += Ms[i] * s[i]; }
  for (int i = 0; i < d->nefc;) {
    real jar[4], cb, fb[4], Hb[4][4];
    const int dim = d->efc_type[i] == SO100O_EFC_CONTACT ? d->efc_dim[i] : 1;
    for (int k = 0; k < dim; k++) jar[k] = jar0[i + k] + alpha * Js[i + k];
    block_eval(d, i, jar, &cb, fb, Hb);
    for (int k = 0; k < dim; k++) {
      g1 -= fb[k] * Js[i + k];
      for (int l = 0; l < dim; l++) g2 += Js[i + k] * Hb[k][l] * Js[i + l];
    }
    i += dim;
  }
  *d1 = g1;
  *d2 = g2;
}
static real line_search(const so100o_data* d, const real a[NV], const real s[NV], const real* jar0, int* first) {
  real e[NV], Js[NEFC];
  for (int k = 0; k < NV; k++) e[k] = a[k] - d->qacc_smooth[k];
  for (int i = 0; i < d->nefc; i++) {
    real t = 0;
    for (int k = 0; k < NV; k++) t += d->efc_J[i][k] * s[k];
    Js[i] = t;
  }
  real d10, d20;
  *first = 0;
  line_derivs(d, e, s, jar0, Js, 0, &d10, &d20);
  if (!(d10 < 0)) return 0;
  const real tol = LS_TOL * -d10;
  real lo = 0, hi = -1, alpha = 1;                  /* hi < 0: no upper bracket yet */
  for (int it = 0; it < 50; it++) {
    real d1, d2;
    line_derivs(d, e, s, jar0, Js, alpha, &d1, &d2);
    if ((real)fabs((double)d1) <= tol) { *first = it == 0; break; }
    if (d1 < 0) lo = alpha; else hi = alpha;
    real nxt = d2 > 0 ? alpha - d1 / d2 : -1;
    if (hi >= 0) { if (!(nxt > lo && nxt < hi)) nxt = (real)0.5 * (lo + hi); }
    else if (!(nxt > lo)) nxt = 2 * alpha;
    if (nxt == alpha) break;
    if ((real)fabs((double)(nxt - alpha)) <= LS_STEP * (real)fabs((double)alpha)) { alpha = nxt; break; }
    alpha = nxt;
  }
  return alpha;
}

/* the zone of the row block at row i at jar (mj_constraintUpdate's cases): frictionloss 0 / 1 / 2 (linear below,
 * quadratic, linear above), joint limit 0 / 1 (inactive, quadratic), contact 0 / 1 / 2 (top: no force, bottom:
 * quadratic, middle: the cone's non-quadratic zone); its row count in *dim */
static int block_zone(const so100o_data* d, int i, const real* jar, int* dim) {
  const int t = d->efc_type[i];
  *dim = 1;
  if (t == SO100O_EFC_FRICTION) {
    const real x = jar[0], rf = d->efc_R[i] * d->efc_frictionloss[i];
    return x >= rf ? 2 : (x <= -rf ? 0 : 1);
  }
  if (t == SO100O_EFC_LIMIT) return jar[0] < 0 ? 1 : 0;
  const int n = d->efc_dim[i];
  *dim = n;
  const real mu = d->efc_mu[i][0] * (real)sqrt((double)(d->efc_R[i + 1] / d->efc_R[i]));
  real T = 0;
  for (int k = 1; k < n; k++) { const real u = jar[k] * d->efc_mu[i][k - 1]; T += u * u; }
  T = (real)sqrt((double)T);
  const real N = jar[0] * mu;
  if (N >= mu * T || (T <= 0 && N >= 0)) return 0;
  if (mu * N + T <= 0 || (T <= 0 && N < 0)) return 1;
  return 2;
}
/* the cost is exactly quadratic between two iterates when no row block changed zone and no contact is in the middle
 * zone: then a full Newton step along the exact Hessian lands on the quadratic's stationary point, the minimiser.
 * As the kernel (so100_newton.h, the quadratic-exact stop): lists longer than the kMaxCon contacts the kernel holds on
 * chip (SO100_MAXCON) keep MuJoCo's stops */
static int same_quadratic(const so100o_data* d, const real* jar0, const real* jar1) {
  if (d->ncon > SO100_MAXCON) return 0;
  for (int i = 0; i < d->nefc;) {
    int n;
    const int z0 = block_zone(d, i, jar0 + i, &n), z1 = block_zone(d, i, jar1 + i, &n);
    if (z0 != z1 || (d->efc_type[i] == SO100O_EFC_CONTACT && z0 == 2)) return 0;
    i += n;
  }
  return 1;
}

/* tools/dev: Newton work counters (gradient evaluations, Hessian + Cholesky factorizations, line searches) */
long so100o_newton_counts[3];
static void sol_newton(const so100_model* m, so100o_data* d) {
  const int nefc = d->nefc;
  const real scale = 1 / ((real)m->meaninertia * (real)NV);
  real a[NV], jar[NEFC], f[NEFC];
  /* start: the warmstart if it is cheaper than the unconstrained acceleration */
  jar_at(d, d->qacc_warmstart, jar);
  const real cw = gauss_cost(d, d->qacc_warmstart) + constraint_cost(d, jar, f);
  jar_at(d, d->qacc_smooth, jar);
  const real cs = constraint_cost(d, jar, f);
  memcpy(a, cw < cs ? d->qacc_warmstart : d->qacc_smooth, sizeof(a));
  jar_at(d, a, jar);
  real cost = gauss_cost(d, a) + constraint_cost(d, jar, f);
  d->solver_iter = 0;
  d->solver_improvement = 0;
  for (int it = 0; it < m->iterations; it++) {
    /* gradient and Hessian at a */
    /* gabs: the gradient's terms in absolute value, one per term (the Gauss row, each row block's J' f): the scale of
     * the gradient's own rounding (NEWTON_GNOISE) */
    real grad[NV], H[NV][NV], gabs[NV];
    for (int i = 0; i < NV; i++) {
      real t = 0;
      for (int j = 0; j < NV; j++) { t += d->qM[i][j] * (a[j] - d->qacc_smooth[j]); H[i][j] = d->qM[i][j]; }
      grad[i] = t;
      gabs[i] = (real)fabs((double)t);
    }
    for (int i = 0; i < nefc;) {
      real cb, fb[4], Hb[4][4];
      const int dim = block_eval(d, i, jar + i, &cb, fb, Hb);
      for (int v = 0; v < NV; v++) {
        real t = 0;
        for (int k = 0; k < dim; k++) t += d->efc_J[i + k][v] * fb[k];
        grad[v] -= t;
        gabs[v] += (real)fabs((double)t);
      }
      for (int k = 0; k < dim; k++) {
        for (int l = 0; l < dim; l++) {
          if (Hb[k][l] == 0) continue;
          for (int p = 0; p < NV; p++)
            for (int q = 0; q < NV; q++) H[p][q] += d->efc_J[i + k][p] * Hb[k][l] * d->efc_J[i + l][q];
        }
      }
      i += dim;
    }
    so100o_newton_counts[0]++;
    real gn = 0;
    int gnoise = 1;
    for (int k = 0; k < NV; k++) {
      gn += grad[k] * grad[k];
      gnoise &= (real)fabs((double)grad[k]) <= (real)NEWTON_GNOISE * (real)FLT_EPSILON * gabs[k];
    }
    if (scale * (real)sqrt((double)gn) < (real)m->tolerance) break;
    if (NEWTON_GNOISE > 0 && gnoise) break;
    real s[NV], mg[NV];
    for (int k = 0; k < NV; k++) mg[k] = -grad[k];
    so100o_newton_counts[1]++;
    if (!chol_solve(H, mg, s)) break;
    if (NEWTON_DECREMENT) {
      real gs = 0;
      for (int k = 0; k < NV; k++) gs += grad[k] * s[k];
      if (scale * (real)-0.5 * gs < (real)m->tolerance) break;
    }
    so100o_newton_counts[2]++;
    int first = 0;
    const real alpha = line_search(d, a, s, jar, &first);
    d->solver_iter = it + 1;
    if (alpha == 0) break;
    static __thread real jar_prev[NEFC];
    if (NEWTON_QUADSTOP) memcpy(jar_prev, jar, sizeof(real) * (size_t)nefc);
    for (int k = 0; k < NV; k++) a[k] += alpha * s[k];
    jar_at(d, a, jar);
    /* the quadratic-exact stop (fp32, round 6): the line search accepted alpha = 1 at its first evaluation over a
     * segment on which the cost is one quadratic (same_quadratic): the step is that quadratic's minimiser, the next
     * gradient zero up to rounding, and the decrement's confirming factorization is skipped */
    if (NEWTON_QUADSTOP && first && alpha == 1 && same_quadratic(d, jar_prev, jar)) {
      cost = gauss_cost(d, a) + constraint_cost(d, jar, f);
      break;
    }
    const real nc = gauss_cost(d, a) + constraint_cost(d, jar, f);
    const real improvement = scale * (cost - nc);
    cost = nc;
    d->solver_improvement = improvement;
    if (improvement < (real)m->tolerance) break;
  }
  constraint_cost(d, jar, d->efc_force);
  memcpy(d->qacc, a, sizeof(a));
}

/* test hook: the Newton cost (Gauss + constraint) at qacc a, on the constraint rows of the last fwd_acceleration */
double so100o_newton_cost(so100o_data* d, const so100o_real a[NV]) {
  real jar[NEFC], f[NEFC];
  jar_at(d, a, jar);
  return (double)(gauss_cost(d, a) + constraint_cost(d, jar, f));
}

/* mj_fwdActuation + the smooth acceleration + mj_referenceConstraint (the solve's inputs) */
static void acc_smooth(const so100_model* m, so100o_data* d) {
  /* [3P] mj_fwdActuation: position actuator, ctrl clamped to ctrlrange, force clamped to forcerange */
  memset(d->qfrc_actuator, 0, sizeof(d->qfrc_actuator));
  for (int i = 0; i < SO100_NU; i++) {
    real c = d->ctrl[i];
    real lo = (real)m->act_ctrlrange[i][0], hi = (real)m->act_ctrlrange[i][1];
    c = c < lo ? lo : (c > hi ? hi : c);
    real kp = (real)m->act_kp[i], kv = (real)m->act_kv[i];
    real fo = kp * c - kp * d->qpos[i] - kv * d->qvel[i];
    real flo = (real)m->act_forcerange[i][0], fhi = (real)m->act_forcerange[i][1];
    fo = fo < flo ? flo : (fo > fhi ? fhi : fo);
    d->actuator_force[i] = fo;
    d->qfrc_actuator[i] = fo;
  }
  /* [3P] mj_fwdAcceleration: qacc_smooth = M^-1 (qfrc_actuator - qfrc_bias) (no passive forces) */
  real rhs[NV];
  for (int k = 0; k < NV; k++) rhs[k] = d->qfrc_actuator[k] - d->qfrc_bias[k] + d->weld_f[k];
  solve_m(d, d->qacc_smooth, rhs);
  /* [3P] mj_referenceConstraint: aref */
  for (int i = 0; i < d->nefc; i++)
    d->efc_aref[i] = -d->efc_B[i] * d->efc_vel[i] - d->efc_K[i] * d->efc_imp[i] * (d->efc_pos[i] - d->efc_margin[i]);
}

/* the constraint solve (mj_fwdConstraint): Newton (MuJoCo's default) or PGS */
static void acc_solve(const so100_model* m, so100o_data* d) {
  const int nefc = d->nefc;
  if (nefc == 0) { memcpy(d->qacc, d->qacc_smooth, sizeof(d->qacc)); d->solver_iter = 0; return; }
  if (m->solver == SO100_SOLVER_NEWTON) { sol_newton(m, d); return; }
  /* [3P] mj_projectConstraint: b, AR = J M^-1 J' + R (nefc x nefc, on the heap: the list may be long) */
  static __thread real MJT[NEFC][NV];
  real* AR = (real*)malloc(sizeof(real) * (size_t)nefc * (size_t)nefc);
  if (!AR) abort();
  for (int i = 0; i < nefc; i++) {
    real s = 0;
    for (int k = 0; k < NV; k++) s += d->efc_J[i][k] * d->qacc_smooth[k];
    d->efc_b[i] = s - d->efc_aref[i];
    solve_m(d, MJT[i], d->efc_J[i]);
  }
  for (int i = 0; i < nefc; i++)
    for (int j = 0; j < nefc; j++) {
      real s = 0;
      for (int k = 0; k < NV; k++) s += d->efc_J[i][k] * MJT[j][k];
      AR[(size_t)i * nefc + j] = s + (i == j ? d->efc_R[i] : 0);
    }
  /* [3P] warmstart (mj_fwdConstraint, dual solver): force from jar(qacc_warmstart); keep it only if
   * its dual cost 0.5 f'ARf + f'b is not positive */
  real jar[NEFC];
  for (int i = 0; i < nefc; i++) {
    real s = 0;
    for (int k = 0; k < NV; k++) s += d->efc_J[i][k] * d->qacc_warmstart[k];
    jar[i] = s - d->efc_aref[i];
  }
  force_from_jar(m, d, jar, d->efc_force);
  real cost = 0;
  for (int i = 0; i < nefc; i++) {
    real s = 0;
    for (int j = 0; j < nefc; j++) s += AR[(size_t)i * nefc + j] * d->efc_force[j];
    cost += d->efc_force[i] * ((real)0.5 * s + d->efc_b[i]);
  }
  if (cost > 0) memset(d->efc_force, 0, sizeof(real) * nefc);
  sol_pgs(m, d, AR);
  free(AR);
  /* qacc = qacc_smooth + M^-1 J' f */
  for (int k = 0; k < NV; k++) {
    real s = 0;
    for (int i = 0; i < nefc; i++) s += MJT[i][k] * d->efc_force[i];
    d->qacc[k] = d->qacc_smooth[k] + s;
  }
}

void so100o_fwd_acceleration(const so100_model* m, so100o_data* d) {
  acc_smooth(m, d);
  acc_solve(m, d);
}

/* [3P] mj_Euler (no dof damping) -> mj_advance: qvel += h qacc; integratePos with the NEW qvel;
 * free-joint quaternion via mju_quatIntegrate (body-frame angular velocity); warmstart = qacc */
void so100o_euler(const so100_model* m, so100o_data* d) {
  const real h = (real)m->timestep;
  for (int k = 0; k < NV; k++) d->qvel[k] += h * d->qacc[k];
  for (int k = 0; k < SO100_NHINGE; k++) d->qpos[k] += h * d->qvel[k];
  for (int k = 0; k < 3; k++) d->qpos[6 + k] += h * d->qvel[6 + k];
  real w[3] = {d->qvel[9], d->qvel[10], d->qvel[11]};
  real nw = norm3(w);
  if (nw > MINVAL) {
    real ax[3] = {w[0] / nw, w[1] / nw, w[2] / nw}, qr[4];
    axis_angle_quat(qr, ax, h * nw);
    quat_mul(d->qpos + 9, d->qpos + 9, qr);
  }
  quat_normalize(d->qpos + 9);
  memcpy(d->qacc_warmstart, d->qacc, sizeof(d->qacc));
}

/* One stage of a substep (the parts of so100o_substep, in order), for the mixed-precision attribution tool
 * (tools/dev/mixed_precision.py: each stage run in fp64 or fp32 on the same state, the data converted between):
 * SO100O_STAGE_KIN kinematics + com_pos, _CRB crb (+ the weld fold) + the M factor, _COLL collision, _CONSTR the
 * constraint rows, _VEL the velocity stage, _SMOOTH actuation + qacc_smooth + aref, _SOLVE the solver, _EULER. */
void so100o_stage(const so100_model* m, so100o_data* d, int k) {
  switch (k) {
    case SO100O_STAGE_KIN: kinematics(m, d); com_pos(m, d); break;
    case SO100O_STAGE_CRB:
      crb(m, d);
      if (m->ee) weld_fold(m, d);
      else memset(d->weld_f, 0, sizeof(d->weld_f));
      factor_m(d);
      break;
    case SO100O_STAGE_COLL: collision(m, d); break;
    case SO100O_STAGE_CONSTR: make_constraint(m, d); break;
    case SO100O_STAGE_VEL: so100o_fwd_velocity(m, d); break;
    case SO100O_STAGE_SMOOTH: acc_smooth(m, d); break;
    case SO100O_STAGE_SOLVE: acc_solve(m, d); break;
    case SO100O_STAGE_EULER: so100o_euler(m, d); break;
    default: break;
  }
}

void so100o_substep(const so100_model* m, so100o_data* d) {
  so100o_fwd_position(m, d);
  so100o_fwd_velocity(m, d);
  so100o_fwd_acceleration(m, d);
  so100o_euler(m, d);
}

/* ============================================================== env layer */
/* SO100CubeToBinTask.initialize_episode (single_arm.py:299-309) inside physics.reset_context():
 * mj_resetData (qvel = 0, warmstart = 0, mocap pose = the mocap body's) then qpos[:6] = start pose, ctrl = start pose, cube pose. */
void so100o_reset(const so100_model* m, so100o_data* d, const double box_pose[7]) {
  memset(d, 0, sizeof(*d));
  load3(d->mocap_pos, m->mocap_pos0);                       /* mj_resetData: mocap = the body's pose */
  load4(d->mocap_quat, m->mocap_quat0);
  for (int k = 0; k < 6; k++) { d->qpos[k] = (real)m->start_qpos[k]; d->ctrl[k] = (real)m->start_qpos[k]; }
  for (int k = 0; k < 7; k++) d->qpos[6 + k] = (real)box_pose[k];
  so100o_fwd_position(m, d);
  so100o_fwd_velocity(m, d);
}

/* _format_raw_obs so100_state (env.py:137-145): box, bin, ee positions and qpos[:6], float32 */
void so100o_observe(const so100_model* m, const so100o_data* d, float obs[SO100_NOBS]) {
  for (int k = 0; k < 3; k++) {
    obs[k] = (float)d->site_cube[k];
    obs[3 + k] = (float)m->bin_center[k];
    obs[6 + k] = (float)d->site_ee[k];
  }
  for (int k = 0; k < 6; k++) obs[9 + k] = (float)d->qpos[k];
}

double so100o_env_step(const so100_model* m, so100o_data* d, int task, const float action[6],
                       float obs[SO100_NOBS], int* terminated) {
  float ctrl[6];
  so100o_unnormalize(m, action, ctrl);
  for (int k = 0; k < 6; k++) d->ctrl[k] = (real)ctrl[k];
  int ndrop = 0;
  for (int s = 0; s < m->nsubstep; s++) {
    so100o_substep(m, d);
    ndrop += d->ncon_dropped;
  }
  /* the last substep's solve, for the force parity tests (the final position stage replaces the contacts) */
  d->snap_ncon = d->ncon;
  d->snap_ndrop = ndrop;
  memset(d->snap_force, 0, sizeof(d->snap_force));
  memset(d->snap_frf, 0, sizeof(d->snap_frf));
  for (int c = 0; c < d->ncon; c++) d->snap_pair[c] = d->con[c].pair;
  for (int c = d->ncon; c < SO100_NCON_MAX; c++) d->snap_pair[c] = -1;
  for (int i = 0; i < d->nefc; i++) {
    if (d->efc_type[i] == SO100O_EFC_FRICTION) d->snap_frf[d->efc_id[i]] = d->efc_force[i];
    if (d->efc_type[i] != SO100O_EFC_CONTACT || d->efc_dim[i] == 0) continue;
    for (int k = 0; k < d->efc_dim[i] && k < 4; k++) d->snap_force[d->efc_id[i]][k] = d->efc_force[i + k];
  }
  memcpy(d->snap_qacc, d->qacc, sizeof(d->qacc));
  so100o_fwd_position(m, d);                         /* dm_control legacy step ends with mj_step1 */
  so100o_fwd_velocity(m, d);
  float cube_f[3] = {(float)d->site_cube[0], (float)d->site_cube[1], (float)d->site_cube[2]};
  double cube[3] = {(double)d->site_cube[0], (double)d->site_cube[1], (double)d->site_cube[2]};
  double ee[3] = {(double)d->site_ee[0], (double)d->site_ee[1], (double)d->site_ee[2]};
  double r = so100o_reward(m, task, cube_f, cube, ee, so100o_contact_bits(d));
  so100o_observe(m, d, obs);
  d->elapsed_steps++;
  if (terminated) *terminated = (r == 4);
  return r;
}

long so100o_batch_run(const so100_model* m, so100o_data* datas, int nenv, int steps, int task,
                      const float* actions, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int e = 0; e < nenv; e++) {
    float obs[SO100_NOBS];
    int term;
    for (int s = 0; s < steps; s++)
      so100o_env_step(m, &datas[e], task, actions + ((size_t)s * nenv + e) * 6, obs, &term);
  }
  return (long)nenv * steps;
}

int so100o_sizeof_data(void) { return (int)sizeof(so100o_data); }
int so100o_sizeof_model(void) { return (int)sizeof(so100_model); }
int so100o_real_bytes(void) { return (int)sizeof(real); }
