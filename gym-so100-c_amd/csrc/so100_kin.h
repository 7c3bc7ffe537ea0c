// so100_kin.h — the stage kernel's per-env LDS layout, small fp32 math and forward kinematics, shared
// with the camera rasteriser (so100_render.hip) (internal).
#pragma once
#include "so100_common.h"

namespace so100 {

struct __attribute__((aligned(16))) ConGeom {    // per-contact geometry (collision output)
  float pos[4];
  float frame[12];     // normal (geom1 -> geom2), tangent1, tangent2
};
union ConSlot {
  ConGeom g;
};
struct __attribute__((aligned(16))) MprStage {   // a box-hull (MPR) contact staged during collision
  float pos[4];        // world position, dist
  float nrm[4];        // world normal (box -> hull), pair index (int bits)
};
struct __attribute__((aligned(16))) ConArea {
  ConSlot con[kMaxCon];
  MprStage mpr[kMaxCon];
};
struct __attribute__((aligned(16))) SerialScratch {   // per-body arrays of the 6-link chain
  float cin[6][16];    // spatial inertia about the Base origin: I(9), m*d(3), m
  float cdof[6][8];    // motion subspace (angular; linear)
  float cfrc[6][8];    // RNE body forces
  float M[6][8];       // joint-space inertia of the arm (CRBA)
  float F[6][8];       // composite inertia times motion subspace, per body
  float L[6][8];       // Cholesky factor of M; L[i][6] = 1 / L[i][i]
  float X[6][8];       // M^-1 columns (X[c][i] = M^-1[i][c])
  float cdd[6][8];     // RNE: cdof_dot per body
  float tau[8];        // actuator force minus bias
  // link frames last: collision still reads them (hull scans) while it fills the contact slots and the
  // MPR staging area, which alias the dead dynamics scratch in front of them
  float xm[6][12];     // body rotation (row-major 3x3, padded)
  float xp[6][4];
};
static_assert(__builtin_offsetof(SerialScratch, xm) >= sizeof(ConArea), "link frames must outlive the contact area");
struct __attribute__((aligned(16))) EnvShared {
  float qpos[16];
  float qvel[16];
  float qacc_smooth[16];
  union {
    float vec[16];
    int cnt[16];                 // S3 compaction counts (vec is free during collision)
  };
  float ctrl[6];
  float minv[6][6];
  float inv_mcube[6];
  float anchor[6][4];
  float axis[6][4];
  float cube_pos[4];
  float cube_mat[12];
  float jaw_pos[2][4];
  float jaw_mat[2][12];
  float site_cube[4];
  float site_ee[4];
  int ncon;
  int ndrop;                     // contacts the kMaxCon cap left out, summed over the fused step's substeps
  int con_pair[kMaxCon];
  float con_dist[kMaxCon];
  float mocap[7];                // EE variant: mocap pose (pos, quat wxyz)
  int rec;                       // fused path: the env's pool contact record this substep (-1: none)
  union {
    struct {
      ConSlot con[kMaxCon];      // geometry (collision -> Jacobian)
      MprStage mpr[kMaxCon];     // MPR contacts staged before the compaction
    };
    SerialScratch ser;           // dynamics scratch (dead before collision) + link frames (live through it)
  };
};
// 3,184 B per env: 4 envs = 12,736 B per wave, under the 12,800 B that lets 12 workgroups share a CU's LDS
// (allocated in 1,280-B steps: 12,928 B held the stage and fused kernels to 11 waves per CU, measured), and
// a stride of 796 dwords (28 banks mod 64), so the 4 envs of a wave hit different LDS bank windows for the
// same field.
static_assert(sizeof(EnvShared) == 3184, "EnvShared: 4 per workgroup must stay within 12,800 B");

// ------------------------------------------------------------------ small math (same formulas as oracle)
DEV float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
DEV void cross3(float* r, const float* a, const float* b) {
  float t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
DEV void mulmv3(float* r, const float* m, const float* v) {
  float t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  float t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  float t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
DEV void mulmtv3(float* r, const float* m, const float* v) {
  float t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  float t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  float t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
DEV void mulmm3(float* r, const float* a, const float* b) {
  float t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = t[i];
}
DEV void quat_mul(float* r, const float* a, const float* b) {
  float t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
DEV void quat_normalize(float* q) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < kMinVal) { q[0] = 1.f; q[1] = q[2] = q[3] = 0.f; return; }
  float inv = 1.0f / n;
  q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
}
DEV void quat2mat(float* m, const float* q) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z);     m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z);     m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y);     m[7] = 2 * (y * z + w * x);     m[8] = 1 - 2 * (x * x + y * y);
}
// ------------------------------------------------------------------ serial position/velocity stage (lane 0)
// [3P] mj_kinematics + mj_comPos + mj_crb + factor + mj_comVel + mj_rne + actuation + qacc_smooth for
// the 6-hinge chain; cube free body in closed form (COM at the origin, principal axes): M = diag(m,m,m,I),
// bias = (-m g, w x I w).  Results to LDS.
DEV void cube_frame(const float* qp, float* pos, float* mat) {
  float q[4] = {qp[3], qp[4], qp[5], qp[6]};
  quat_normalize(q);
  quat2mat(mat, q);
  pos[0] = qp[0]; pos[1] = qp[1]; pos[2] = qp[2];
}

// the 6 hinge half-angle sines/cosines, one per lane (lanes 0..5), staged in sh.vec for fk_stage: the
// transcendentals leave the serial chain on lane 0.  A barrier must separate it from fk_stage.
DEV void joint_sincos(EnvShared& sh, int lane, bool act = true) {
  if (act && lane < 6) {
    float sn, cs;
    sincosf(0.5f * sh.qpos[lane], &sn, &cs);
    sh.vec[2 * lane] = sn;
    sh.vec[2 * lane + 1] = cs;
  }
}

// full serial stage; writes frames, M^-1, qacc_smooth, sites into sh
// Forward kinematics of the 6-link chain (lane 0 of the env's row): body frames, joint anchors/axes,
// jaw frames, sites, cube frame.  dynamics_par continues from these.
DEV void fk_stage(const DevModel* __restrict__ m, EnvShared& sh) {
  // ---- forward kinematics along the chain; frames staged in LDS to bound register pressure
  {
    float pos[3] = {m->base_pos[0], m->base_pos[1], m->base_pos[2]};
    float quat[4] = {m->base_quat[0], m->base_quat[1], m->base_quat[2], m->base_quat[3]};
    float R[9];
    quat2mat(R, quat);
    for (int a = 0; a < 6; a++) {
      float t[3];
      mulmv3(t, R, m->body_pos[a]);
      pos[0] += t[0]; pos[1] += t[1]; pos[2] += t[2];
      quat_mul(quat, quat, m->body_quat[a]);
      float R2[9], ax[3];
      quat2mat(R2, quat);
      mulmv3(ax, R2, m->jnt_axis[a]);
      const float sn = sh.vec[2 * a], cs = sh.vec[2 * a + 1];    // joint_sincos
      float qj[4] = {cs, m->jnt_axis[a][0] * sn, m->jnt_axis[a][1] * sn, m->jnt_axis[a][2] * sn};
      quat_mul(quat, quat, qj);
      quat_normalize(quat);
      quat2mat(R, quat);
#pragma unroll
      for (int k = 0; k < 3; k++) { sh.anchor[a][k] = pos[k]; sh.axis[a][k] = ax[k]; sh.ser.xp[a][k] = pos[k]; }
#pragma unroll
      for (int k = 0; k < 9; k++) sh.ser.xm[a][k] = R[k];
    }
  }
  asm volatile("" ::: "memory");
#pragma unroll
  for (int j = 0; j < 2; j++) {
#pragma unroll
    for (int t = 0; t < 3; t++) sh.jaw_pos[j][t] = sh.ser.xp[4 + j][t];
#pragma unroll
    for (int t = 0; t < 9; t++) sh.jaw_mat[j][t] = sh.ser.xm[4 + j][t];
  }
  {
    float t[3];
    mulmv3(t, sh.ser.xm[4], m->site_ee);
#pragma unroll
    for (int k = 0; k < 3; k++) sh.site_ee[k] = sh.ser.xp[4][k] + t[k];
  }
  {
    float qp[7], cpos[3], cmat[9];
#pragma unroll
    for (int k = 0; k < 7; k++) qp[k] = sh.qpos[6 + k];
    cube_frame(qp, cpos, cmat);
#pragma unroll
    for (int k = 0; k < 3; k++) sh.cube_pos[k] = cpos[k];
#pragma unroll
    for (int k = 0; k < 9; k++) sh.cube_mat[k] = cmat[k];
    float t[3];
    mulmv3(t, cmat, m->site_cube);
#pragma unroll
    for (int k = 0; k < 3; k++) sh.site_cube[k] = cpos[k] + t[k];
  }
}

// Forward kinematics with the 16 lanes of the env's row (lane a < 6: body a of the chain; lane 6: the cube):
// the same frames as fk_stage from the staged qpos (a barrier must separate the qpos stores), without its
// serial chain on one lane.  fk_stage's per-body product q_a = normalize(q_{a-1} (x) qb_a (x) qj_a) becomes
// a prefix product over the lanes of c_a = qb_a (x) qj_a (3 DPP steps), normalised once per body; the
// positions pos_a = pos_{a-1} + R_{a-1} body_pos[a] a prefix sum (3 DPP steps); the joint axis R_a
// jnt_axis[a] (the joint rotation leaves its axis fixed: fk_stage's pre-rotation frame gives the same axis).
// Equal to fk_stage up to fp32 rounding (association), which the parity tests' tolerances cover.
// row_shr:D with a fill: lane l of the row gets v of lane l - D, lanes l < D get `old` (no select, so the
// compiler cannot put the DPP under an exec mask that disables its source lanes, which then read 0)
template <int D>
DEV float fk_shr(float old, float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                                0x110 + D, 0xF, 0xF, false));
}
DEV void fk_par(const DevModel* __restrict__ m, EnvShared& sh, int lane, bool act = true) {
  const bool arm = lane < 6;
  const int a = arm ? lane : 5;
  float c[4];
  {
    float sn, cs;
    sincosf(0.5f * sh.qpos[a], &sn, &cs);
    const float qj[4] = {cs, m->jnt_axis[a][0] * sn, m->jnt_axis[a][1] * sn, m->jnt_axis[a][2] * sn};
    float t[4], u[4];
    quat_mul(t, m->body_quat[a], qj);
    quat_mul(u, m->base_quat, t);                 // lane 0 starts from the Base's frame
#pragma unroll
    for (int k = 0; k < 4; k++) c[k] = lane == 0 ? u[k] : (arm ? t[k] : (k == 0 ? 1.f : 0.f));
  }
  // inclusive prefix product over lanes 0..5 (left factor: the earlier lanes)
#define FK_SCAN_Q(D)                                                                             \
  {                                                                                              \
    float p[4];                                                                                  \
    for (int k = 0; k < 4; k++) p[k] = fk_shr<D>(k == 0 ? 1.f : 0.f, c[k]);   /* identity fill */  \
    quat_mul(c, p, c);                                                                           \
  }
  FK_SCAN_Q(1) FK_SCAN_Q(2) FK_SCAN_Q(4)
#undef FK_SCAN_Q
  quat_normalize(c);
  float R[9], Rp[9], Rb[9];
  quat2mat(R, c);
  quat2mat(Rb, m->base_quat);
#pragma unroll
  for (int k = 0; k < 9; k++) Rp[k] = fk_shr<1>(Rb[k], R[k]);   // the parent's frame (lane 0: the Base's)
  float t[3];
  mulmv3(t, Rp, m->body_pos[a]);
#define FK_SCAN_P(D)                                                                             \
  {                                                                                              \
    for (int k = 0; k < 3; k++) t[k] += fk_shr<D>(0.f, t[k]);                                    \
  }
  FK_SCAN_P(1) FK_SCAN_P(2) FK_SCAN_P(4)
#undef FK_SCAN_P
  const float pos[3] = {m->base_pos[0] + t[0], m->base_pos[1] + t[1], m->base_pos[2] + t[2]};
  float ax[3];
  mulmv3(ax, R, m->jnt_axis[a]);
  if (act && arm) {
#pragma unroll
    for (int k = 0; k < 3; k++) { sh.anchor[a][k] = pos[k]; sh.axis[a][k] = ax[k]; sh.ser.xp[a][k] = pos[k]; }
#pragma unroll
    for (int k = 0; k < 9; k++) sh.ser.xm[a][k] = R[k];
    if (a >= 4) {
#pragma unroll
      for (int k = 0; k < 3; k++) sh.jaw_pos[a - 4][k] = pos[k];
#pragma unroll
      for (int k = 0; k < 9; k++) sh.jaw_mat[a - 4][k] = R[k];
    }
    if (a == 4) {
      float w[3];
      mulmv3(w, R, m->site_ee);
#pragma unroll
      for (int k = 0; k < 3; k++) sh.site_ee[k] = pos[k] + w[k];
    }
  }
  if (act && lane == 6) {
    float qp[7], cpos[3], cmat[9];
#pragma unroll
    for (int k = 0; k < 7; k++) qp[k] = sh.qpos[6 + k];
    cube_frame(qp, cpos, cmat);
#pragma unroll
    for (int k = 0; k < 3; k++) sh.cube_pos[k] = cpos[k];
#pragma unroll
    for (int k = 0; k < 9; k++) sh.cube_mat[k] = cmat[k];
    float w[3];
    mulmv3(w, cmat, m->site_cube);
#pragma unroll
    for (int k = 0; k < 3; k++) sh.site_cube[k] = cpos[k] + w[k];
  }
}

}  // namespace so100
