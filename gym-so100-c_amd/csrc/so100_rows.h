// so100_rows.h — per-contact constraint rows: the contact frame (mju_makeFrame), the contact Jacobian column of a dof,
// M^-1 J', and the symmetric 3x3 eigen-decomposition of the PGS friction block (oracle make_frame /
// contact_jac / eig3).
// (internal; included by so100_step.hip, the one translation unit of the step kernels)
#pragma once
#include "so100_common.h"
#include "so100_kin.h"

namespace so100 {

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

// the Jacobian column for dof `lane` of the contact of pair p at point cp with frame fr (rows: normal, t1, t2
// on the point velocity; torsion on the angular velocity); J = frame . (jac(body of geom2) - jac(body of
// geom1)) at the contact point
DEV float4 contact_jac_at(const DevModel* __restrict__ m, const EnvShared& sh, int p, const float* cp, const float* fr,
                          int lane) {
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
// contact c < kMaxCon (on chip)
DEV float4 contact_jac(const DevModel* __restrict__ m, const EnvShared& sh, int c, int lane) {
  return contact_jac_at(m, sh, sh.con_pair[c], sh.con[c].g.pos, sh.con[c].g.frame, lane);
}
// contact c >= kMaxCon: its geometry from the env's HBM contact record (so100_step.hip store_contact)
DEV float4 contact_jac_ovf(const DevModel* __restrict__ m, const EnvShared& sh, const float* crec, int c, int lane) {
  const float* g = crec + (size_t)c * kConStride + kGeoOff;
  float cp[3], fr[9];
#pragma unroll
  for (int t = 0; t < 3; t++) cp[t] = g[t];
#pragma unroll
  for (int t = 0; t < 9; t++) fr[t] = g[4 + t];
  return contact_jac_at(m, sh, __float_as_int(g[16]), cp, fr, lane);
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

}  // namespace so100
