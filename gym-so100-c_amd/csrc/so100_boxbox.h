// so100_boxbox.h — box-box narrowphase (separating axes + face clipping, every clipped point: MuJoCo mjc_BoxBox; oracle
// box_box / collide_box_pair), geom poses, and the arm hulls against the table top (oracle hull_table).
// (internal; included by so100_step.hip, the one translation unit of the step kernels)
#pragma once
#include "so100_common.h"
#include "so100_kin.h"

namespace so100 {

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

// collapse: the pair is a box (the cube, a finger pad) against the table's mesh, one contact (MuJoCo's convex
// collider; the oracle's collide_box_pair): the exact separating-axis minimum over all 15 axes (no face preference
// for the edge axes: the convex collider's minimum penetration), the mean of the kept points' positions and the
// deepest distance, summed in clip order as the kept points would be, without their compaction and 8-slot output
// (bitwise the same contact)
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
  const float ebias = collapse ? 1.f : 1.05f;      // mjc_BoxBox prefers faces unless an edge axis is clearly better
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
      if (s * ebias > best) {
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
  if (b == SO100_MOCAP_BODY) {   // the EE variant's marker box: centred on the mocap body (so100_create checks)
#pragma unroll
    for (int k = 0; k < 3; k++) pos[k] = sh.mocap[k];
    quat2mat(mat, sh.mocap + 3);      // normalised by set_controls
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
  // a box (the cube, a finger pad) against the table's mesh (geom2 = geom 0): MuJoCo's convex collider, one contact
  // per pair (the oracle's collide_box_pair): the SAT normal, the deepest distance, the mean of the clipped positions
  box_box(p1, R1, A, p2, R2, B, margin, pc, g2 == 0);
}

// Arm/jaw hulls vs the table (pairs SO100_NPAIR_BOX + k; oracle table_hull_fast).  The table is a mesh, so MuJoCo
// collides it through its convex collider: the minimum penetration.  Lane k < SO100_NHULL classifies hull k from its
// body-frame bounding box (world z extent ez, x-y extents ex, ey about the box centre c):
//  * candidate: the box's lowest point zb = c.z - ez below top + margin (else separated);
//  * top-face rule (fast): with D = top - zb (>= the hull's depth below the top), every vertex lies inside the top
//    face's footprint shrunk by D (c.x - ex >= lo.x + D, ...) and the hull's centroid (model constant, inside the
//    hull) is at least D above the table's bottom.  Then the minimum penetration is exactly the depth d of the lowest
//    vertex along +z: lifting by d separates, and any shorter translation leaves a point of the hull inside the
//    table box.  The contact: the lowest vertex (first in hull order among ties) and its projection on the top;
//  * otherwise (at the table's edges and side faces, or deep): the convex collider (mpr_contacts' slow items).
// Returns the classification bits of lane k: 1 = candidate, 2 = top-face rule.
DEV int table_hull_class(const DevModel* __restrict__ m, const EnvShared& sh, int lane, bool valid) {
  if (!valid || lane >= SO100_NHULL) return 0;
  const int a = m->hull_body[lane] - 2;
  const float4 hc = reinterpret_cast<const float4*>(m->hull_center)[lane];
  const float4 hh = reinterpret_cast<const float4*>(m->hull_half)[lane];
  const float4 hg = reinterpret_cast<const float4*>(m->hull_centroid)[lane];
  const float* R = sh.ser.xm[a];
  const float* P = sh.ser.xp[a];
  const float top = m->table_top;
  const float cz = (R[6] * hc.x + R[7] * hc.y + R[8] * hc.z) + P[2];
  const float ez = fabsf(R[6]) * hh.x + fabsf(R[7]) * hh.y + fabsf(R[8]) * hh.z;
  if (!(cz - ez < top + m->pair_margin[SO100_NPAIR_BOX + lane])) return 0;
  const float cx = (R[0] * hc.x + R[1] * hc.y + R[2] * hc.z) + P[0];
  const float cy = (R[3] * hc.x + R[4] * hc.y + R[5] * hc.z) + P[1];
  const float ex = fabsf(R[0]) * hh.x + fabsf(R[1]) * hh.y + fabsf(R[2]) * hh.z;
  const float ey = fabsf(R[3]) * hh.x + fabsf(R[4]) * hh.y + fabsf(R[5]) * hh.z;
  const float gz = (R[6] * hg.x + R[7] * hg.y + R[8] * hg.z) + P[2];
  const float D = top - (cz - ez);
  const bool fast = cx - ex >= m->table_lo[0] + D && cx + ex <= m->table_hi[0] - D && cy - ey >= m->table_lo[1] + D &&
                    cy + ey <= m->table_hi[1] - D && gz - m->table_bottom >= D;
  return fast ? 3 : 1;
}

}  // namespace so100
