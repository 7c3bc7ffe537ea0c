// so100_convex.h — the mesh pairs' convex collider (MuJoCo mjc_Convex): GJK + EPA (the default, MuJoCo 3.3.3's native ccd)
// and libccd's MPR, the hull supports through the cube-map cells, the bounding-sphere / OBB broadphase and
// the wave-shared narrowphase (oracle gjk_* / epa_penetration / mpr_* / collision()).
// (internal; included by so100_step.hip, the one translation unit of the step kernels)
#pragma once
#include "so100_common.h"
#include "so100_kin.h"
#include "so100_boxbox.h"
#include "so100_pool.h"

namespace so100 {

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
};
constexpr float kCcdEps = 2.220446049250313e-16f;   // MuJoCo's double libccd CCD_EPS (absolute tests: see oracle)
constexpr float kMprTol = 1e-6f;            // MuJoCo ccd_tolerance
constexpr float kSepTol = 1e-6f;            // a cached separating direction must clear the pair by 1 um (mpr_contacts;
                                            // oracle SEP_TOL)
// EPA: a facet is visible from the new support point only when the point clears its plane by more than this (the
// ccd_tolerance; oracle EPA_VISTOL): a point on a facet's plane within fp32 rounding is not "visible", so no facet is
// built folding back over a coplanar one (an inverted facet, negative distance, that derailed fp32 EPA on face-face
// hull contacts: DESIGN.md §4 deviation 7)
constexpr float kEpaVisTol = 1e-6f;
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
    if (cells && am > 1e-30f && am < __builtin_inff()) {
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

// The top-face rule's contacts (oracle table_hull_fast): for the hulls table_hull_class puts under it in some env of
// the wave, the env's row finds the hull's lowest vertex by its support (hull_support) in the body-frame direction of
// world -z.  Needs the link frames of fk_stage (sh.ser.xm / xp).  Lane k < SO100_NHULL returns
// hull k's contact flag (its lowest vertex below top + margin) and its lowest vertex.
DEV bool hull_table(const DevModel* __restrict__ m, const EnvShared& sh, int lane, int grp, bool valid, float& hx,
                    float& hy, float& hz) {
  bool found = false;
  hx = hy = hz = 0.f;
  const float top = m->table_top;
  const bool cand = table_hull_class(m, sh, lane, valid) == 3;
  const uint64_t cm = __ballot(cand);
  const uint32_t env_cand = (uint32_t)(cm >> (grp * 16)) & 0xFFFFu;
  uint32_t wave_cand = (uint32_t)((cm | (cm >> 16) | (cm >> 32) | (cm >> 48)) & 0xFFFFull);
  while (wave_cand) {
    const int k = __builtin_ctz(wave_cand);
    wave_cand &= wave_cand - 1u;
    const bool mine = (env_cand >> k) & 1u;
    float bz = __builtin_inff(), bx = 0.f, by = 0.f;
    int bi = 0x7fffffff;
    if (mine) {
      // the lowest vertex: hull k's support in the body-frame direction -R' e_z (its first maximal vertex: a whole-hull
      // scan, 8 loads in flight per lane; the cells' lookup spilled the 3-wave build here), in hull-relative terms; the body's
      // position is added after (compared in world z, ~0.5 m with 3e-8 m rounding, a hull face lying nearly flat
      // tied its corners and fp32 picked another than fp64, centimetres away; round 6, oracle table_hull_fast)
      const float* R = sh.ser.xm[m->hull_body[k] - 2];
      const float4 v = hull_support(m, false, k, m->hull_start[k], m->hull_count[k], -R[6], -R[7], -R[8], lane);
      const float hv[3] = {v.x, v.y, v.z};
      float w[3];
      mulmv3(w, R, hv);
      bx = w[0]; by = w[1]; bz = w[2]; bi = __float_as_int(v.w);
    }
    if (lane == k) {
      const float* P = sh.ser.xp[m->hull_body[k] - 2];
      hx = bx + P[0]; hy = by + P[1]; hz = bz + P[2];
      found = mine && bi != 0x7fffffff && (hz - top < m->pair_margin[SO100_NPAIR_BOX + k]);
    }
  }
  return found;
}

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
  const float4 v = hull_support(m, o.cells, o.k, o.s0, o.n, -d[0], -d[1], -d[2], lane);
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

// GJK (oracle gjk): true when A - B encloses the origin, S then holds the enclosing tetrahedron.
// sc: the pair's entry of mpr_contacts' separating-direction cache, set to (the unit direction, 1) when the support
// test proves the pair separated (stored here: a direction returned to the caller was a value live across EPA,
// spilled in the 3-wave build)
DEV bool gjk_enclose(const DevModel* __restrict__ m, const MprObj& o, GjkPt* S, int lane, float4* sc) {
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
    if (dot3(a.v, du) <= 0.f) {
      if (lane == 0) *sc = make_float4(du[0], du[1], du[2], 1.f);
      return false;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) pt_sel(S[k], a, n == k);
    n++;
    if (n > 1 && gjk_simplex(S, n, d)) return true;
    if (n == 1) { d[0] = -a.v[0]; d[1] = -a.v[1]; d[2] = -a.v[2]; }
  }
  return false;
}

// a facet (a, b, c) of the polytope into slot f (oracle epa_face_set); false for a degenerate triangle (its slot
// is then written anyway, unused: the caller abandons the polytope; no branch, so the initial tetrahedron's 4
// facets are straight-line code)
DEV bool epa_face_set(EpaPoly& P, int f, int a, int b, int c, const float* A, const float* B, const float* C) {
  float ab[3], ac[3], n[3];
  sub3(ab, B, A);
  sub3(ac, C, A);
  cross3(n, ab, ac);
  const float l2 = dot3(n, n);
  const bool good = l2 >= kCcdEps * kCcdEps;      // !ccd_zero(|n|) (a NaN facet, from NaN points, also fails)
  const float il = __builtin_amdgcn_rsqf(l2);     // 1 / |n| (oracle epa_face_set: one division), v_rsq
  n[0] = n[0] * il; n[1] = n[1] * il; n[2] = n[2] * il;
  P.plane[f] = make_float4(n[0], n[1], n[2], dot3(n, A));
  P.fv[f] = (uint32_t)a | (uint32_t)b << 5 | (uint32_t)c << 10;
  return good;
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

// The contact of EPA's final facet from the features it spans (round 6; oracle epa_feature_witness).  The facet lies on
// a face of the Minkowski difference obj1 - obj2: obj1's vertex against obj2's face (one distinct obj1 support id,
// three of obj2), obj1's face against obj2's vertex (three, one), or an edge of each (two, two); the contact is then
// those features' exact one (the vertex and its projection on the face plane, or the edges' closest points with the
// normal along their cross product), from the supports' own coordinates.  The barycentric interpolation over the facet
// (the fallback for any other facet) depends on which triangle of the face EPA stopped on, and on a sliver facet (a
// 1.2 m table edge beside a mm-long hull edge) fp32 lost 1e-2 of the weight along the long edge: the contact moved
// centimetres between fp32 and fp64 (tools/dev/collision_precision.py).  Row-redundant; false: fall back.
// The case is decided from the support ids alone, and only the 4 points it needs are rebuilt (P0 = obj1's point of
// the facet's first vertex, P3 = obj2's; P1, P2 the features' other points): the 3 whole supports of the barycentric
// path held across it spilled the 3-wave build.
// obj1's (which = 1) or obj2's (2) point of the support with id `id`, by mpr_support's arithmetic (sup_from_id's)
DEV void sup_point(const DevModel* __restrict__ m, const MprObj& o, uint32_t id, int which, float* r) {
  float v1[3];
#pragma unroll
  for (int t = 0; t < 3; t++) v1[t] = o.c[t];
  if (o.hull1 < 0) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const float sz = (id >> i) & 1u ? o.h[i] : -o.h[i];
#pragma unroll
      for (int t = 0; t < 3; t++) v1[t] += sz * o.ax[3 * t + i];
    }
  } else {
    const float4 hv = reinterpret_cast<const float4*>(m->hull_vert)[o.s1 + (int)(id & 1023u)];
    const float vv[3] = {hv.x, hv.y, hv.z};
    float w[3];
    mulmv3(w, o.ax, vv);
#pragma unroll
    for (int t = 0; t < 3; t++) v1[t] += w[t];
  }
  const float4 v2 = reinterpret_cast<const float4*>(m->hull_vert)[o.s0 + (int)((id >> 10) & 1023u)];
  r[0] = which == 1 ? v1[0] : v2.x;
  r[1] = which == 1 ? v1[1] : v2.y;
  r[2] = which == 1 ? v1[2] : v2.z;
}
DEV bool epa_feature_witness(const DevModel* __restrict__ m, const MprObj& o, uint32_t ia, uint32_t ib, uint32_t ic,
                             const float* fn, float& depth, float4& fdir, float4& fpos) {
  const uint32_t a1 = ia & 1023u, b1 = ib & 1023u, c1 = ic & 1023u;
  const uint32_t a2 = (ia >> 10) & 1023u, b2 = (ib >> 10) & 1023u, c2 = (ic >> 10) & 1023u;
  const int n1 = 1 + (b1 != a1) + (c1 != a1 && c1 != b1);
  const int n2 = 1 + (b2 != a2) + (c2 != a2 && c2 != b2);
  const bool ee = n1 == 2 && n2 == 2, vf = n1 == 1 && n2 == 3, fvx = n1 == 3 && n2 == 1;
  if (!(ee || vf || fvx)) return false;
  // ee: P1 = obj1's other edge end, P2 = obj2's; vf: P1, P2 = obj2's face corners B2, C2; fvx: obj1's B1, C1
  float P0[3], P1[3], P2[3], P3[3];
  sup_point(m, o, ia, 1, P0);
  sup_point(m, o, ia, 2, P3);
  sup_point(m, o, ee ? (b1 != a1 ? ib : ic) : ib, vf ? 2 : 1, P1);
  sup_point(m, o, ee ? (b2 != a2 ? ib : ic) : ic, fvx ? 1 : 2, P2);
  float e1[3], e2[3], nn[3], w0[3], p1[3], p2[3];
#pragma unroll
  for (int t = 0; t < 3; t++) {
    e1[t] = P1[t] - (vf ? P3[t] : P0[t]);
    e2[t] = P2[t] - (fvx ? P0[t] : P3[t]);
    w0[t] = P0[t] - P3[t];
  }
  cross3(nn, e1, e2);
  if (ee) {
    const float a = dot3(e1, e1), b = dot3(e1, e2), c = dot3(e2, e2), dd = dot3(e1, w0), e = dot3(e2, w0);
    const float den = a * c - b * b;
    if (!(den > 1e-6f * a * c)) return false;   // (nearly) parallel edges: no single closest pair
    const float t_ = (b * e - c * dd) / den, u_ = (a * e - b * dd) / den;
#pragma unroll
    for (int t = 0; t < 3; t++) { p1[t] = P0[t] + t_ * e1[t]; p2[t] = P3[t] + u_ * e2[t]; }
  }
  const float l = sqrtf(dot3(nn, nn));
  if (ccd_zero(l)) return false;
  const float il = (dot3(nn, fn) < 0.f ? -1.f : 1.f) / l;   // oriented as the facet's outward normal
  nn[0] *= il; nn[1] *= il; nn[2] *= il;
  float dep;
  if (ee) {
    float w[3];
    sub3(w, p1, p2);
    dep = dot3(nn, w);
  } else {
    dep = dot3(nn, w0);
#pragma unroll
    for (int t = 0; t < 3; t++) {
      p1[t] = vf ? P0[t] : P3[t] + dep * nn[t];
      p2[t] = vf ? P0[t] - dep * nn[t] : P3[t];
    }
  }
  if (!(dep > 0.f) || ccd_zero(dep)) return false;
  depth = dep;
  fdir = make_float4(nn[0], nn[1], nn[2], 0.f);
  fpos = make_float4(0.5f * (p1[0] + p2[0]), 0.5f * (p1[1] + p2[1]), 0.5f * (p1[2] + p2[2]), 0.f);
  return true;
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
      ok = epa_face_set(P, i, a, bb, cc, A.v, B.v, C.v) && ok;
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
    // the lane's position in its row from an opaque v_mbcnt pair each iteration: lane-derived values (the facet slot
    // addresses, the below-lane mask) held across the iterations were spilled values reloaded inside them
    lane = row_lane();
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
        mv[s3] = (pl.x * w.v[0] + pl.y * w.v[1] + pl.z * w.v[2]) - pl.w > kEpaVisTol;
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
        const int src = row_lane_addr(vi);
        const float x0 = shfl_at(V.x[0], src), x1 = shfl_at(V.x[1], src);
        const float y0 = shfl_at(V.y[0], src), y1 = shfl_at(V.y[1], src);
        const float z0 = shfl_at(V.z[0], src), z1 = shfl_at(V.z[1], src);
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
  // the contact's witness is computed after the round's narrowphase, by one lane (epa_contact): the final facet's 3
  // support ids go out in pos (as bits), its normal in dir (round 6: computed here, inside the narrowphase's register
  // peak, the feature witness spilled the 3-wave build)
  const uint32_t fv = P.fv[best];
  pos[0] = __uint_as_float(P.vid[fv & 31u]);
  pos[1] = __uint_as_float(P.vid[(fv >> 5) & 31u]);
  pos[2] = __uint_as_float(P.vid[(fv >> 10) & 31u]);
#pragma unroll
  for (int t = 0; t < 3; t++) dir[t] = bn[t];
  return true;
}

// EPA's contact from its final facet (the support ids a, b, c and the facet's plane (n, dist)): the features' exact
// contact (epa_feature_witness), else the witness points from the barycentric coordinates of the origin's projection
// p = n dist on the facet (oracle epa_penetration).  In H: odir (normal), opos (xyz, the depth in w).
DEV void epa_contact(const DevModel* __restrict__ m, const MprObj& o, uint32_t ia, uint32_t ib, uint32_t ic,
                     const float* bn, float bd, float4& odir, float4& opos) {
#ifndef SO100_NO_FEAT   // (A/B switch: the barycentric witness alone, round 5's)
  float4 fdir, fpos;
  float fdepth = bd;
  if (epa_feature_witness(m, o, ia, ib, ic, bn, fdepth, fdir, fpos)) {
    odir = fdir;
    opos = make_float4(fpos.x, fpos.y, fpos.z, fdepth);
    return;
  }
#endif
  MprSup A, B, C;
  sup_from_id(m, o, ia, A);
  sup_from_id(m, o, ib, B);
  sup_from_id(m, o, ic, C);
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
  float q[3];
#pragma unroll
  for (int t = 0; t < 3; t++) {
    float w1 = 0.f, w2 = 0.f;
    w1 += l0 * A.v1[t]; w2 += l0 * A.v2[t];
    w1 += l1 * B.v1[t]; w2 += l1 * B.v2[t];
    w1 += l2 * C.v1[t]; w2 += l2 * C.v2[t];
    q[t] = 0.5f * (w1 + w2);
  }
  odir = make_float4(bn[0], bn[1], bn[2], 0.f);
  opos = make_float4(q[0], q[1], q[2], bd);
}

// the mesh pairs' collider of the model (so100_model.convex): GJK + EPA (MuJoCo 3.3.3's default) or MPR
DEV bool convex_penetration(const DevModel* __restrict__ m, const MprObj& o, float& depth, float* dir, float* pos,
                            EpaPoly& P, int lane, int grp, float4* sc) {
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
  const bool enc = gjk_enclose(m, o, S, lane, sc);
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

// Convex pair p (23..151; 14..22 outside the top-face rule): obj1 = box geom (cube, bin box, finger pad, the marker,
// the table: geom 0, a static box) or hull k1 (self-collision, the Base), obj2 = hull k, both in hull k's body frame H.
// Oracle convex_pair.
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
// centre; box: its centre) and radius (hull_half.w / geom_rbound), by the arithmetic mpr_sphere uses.  (The
// EE variant's marker box, the last geom, has its own pass: marker_contacts.)
static_assert(SO100_MOCAP_GEOM == SO100_NGEOM - 1, "the marker box is the last geom");
constexpr int kSphObj = SO100_NHULL_ALL + SO100_MOCAP_GEOM - 1;   // 24
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

// A table-hull contact from GJK + EPA (pair p = 14 + k) whose world normal lies within 1e-5 rad of one of the table
// box's face normals (world axes) is that face's contact (round 6; oracle table_face_snap): EPA stops within its
// tolerance of the face normal, and under that residual tilt a hull lying flat on the face tied its corners, fp32 and
// fp64 taking different ones.  Restated exactly: normal the face's axis u (table -> hull), the hull's extreme vertex
// along -u (the first in hull order among ties, compared in hull-relative coordinates: the hull's support in the body-
// frame direction, through the cube-map cells on the fused path), depth from the face plane, pos the midpoint of the
// vertex and its projection on the face.  Row-uniform; true when the contact snapped, with its WORLD-frame position and depth (wp: xyz, -depth in w)
// and normal (wn: xyz) in their own registers (written into dir / pos, the arrays went to scratch).
DEV bool table_face_snap(const DevModel* __restrict__ m, const EnvShared& sh, int p, const float* dir, int lane,
                         const MprObj& o, float4& wpo, float4& wno) {
  const int k = -1 - m->pair_g2[p];
  float RH[9], pH[3], wn[3];
  hull_frame(m, sh, m->hull_body[k], RH, pH);
  mulmv3(wn, RH, dir);
  const float a0 = fabsf(wn[0]), a1 = fabsf(wn[1]), a2 = fabsf(wn[2]);
  const int ax = a1 > a0 ? (a2 > a1 ? 2 : 1) : (a2 > a0 ? 2 : 0);
  const float o1 = ax == 0 ? wn[1] : wn[0], o2 = ax == 2 ? wn[1] : wn[2];
  if (!(sqrtf(o1 * o1 + o2 * o2) < 1e-5f)) return false;
  const float wa = ax == 0 ? wn[0] : ax == 1 ? wn[1] : wn[2];
  const float sgn = wa > 0.f ? 1.f : -1.f;
  const float lo = ax == 2 ? m->table_bottom : ax == 1 ? m->table_lo[1] : m->table_lo[0];
  const float hi = ax == 2 ? m->table_top : ax == 1 ? m->table_hi[1] : m->table_hi[0];
  const float face = sgn > 0.f ? hi : lo;
  // the row of RH that gives the world coordinate on axis ax
  const float ra = ax == 0 ? RH[0] : ax == 1 ? RH[3] : RH[6];
  const float rb = ax == 0 ? RH[1] : ax == 1 ? RH[4] : RH[7];
  const float rc = ax == 0 ? RH[2] : ax == 1 ? RH[5] : RH[8];
  // the hull's extreme vertex along -u: its support in the body-frame direction -sgn (ra, rb, rc) (the first maximal
  // vertex: the cube-map cells' candidates on the fused path, the whole hull on the split path, the same vertex)
  const float4 v = hull_support(m, o.cells, k, o.s0, o.n, -sgn * ra, -sgn * rb, -sgn * rc, lane);
  const float hv[3] = {v.x, v.y, v.z};
  float wb[3];
  mulmv3(wb, RH, hv);
  wb[0] += pH[0]; wb[1] += pH[1]; wb[2] += pH[2];
  const float wax = ax == 0 ? wb[0] : ax == 1 ? wb[1] : wb[2];
  const float mid = 0.5f * (wax + face);
  wpo = make_float4(ax == 0 ? mid : wb[0], ax == 1 ? mid : wb[1], ax == 2 ? mid : wb[2], sgn * wax - sgn * face);
  wno = make_float4(ax == 0 ? sgn : 0.f, ax == 1 ? sgn : 0.f, ax == 2 ? sgn : 0.f, 0.f);
  return true;
}

// a convex pair's contact (in hull k's body frame H; world: already in the world frame, table_face_snap) to the world,
// staged as the env's convex contact `slot`: the LDS staging area, or (rare: beyond kMaxCon) the env's HBM contact
// record crec
DEV void stage_convex_hit(const DevModel* __restrict__ m, EnvShared& sh, float* crec, int slot, int p, float depth,
                          const float* dir_in, const float* pos_in, bool world, float4 wpo, float4 wno) {
  const int k = -1 - m->pair_g2[p];
  float RH[9], pH[3], wn[3], wp[3];
  const float dir[3] = {dir_in[0], dir_in[1], dir_in[2]}, pos[3] = {pos_in[0], pos_in[1], pos_in[2]};
  hull_frame(m, sh, m->hull_body[k], RH, pH);
  mulmv3(wn, RH, dir);
  mulmv3(wp, RH, pos);
  const float4 sp = world ? wpo : make_float4(wp[0] + pH[0], wp[1] + pH[1], wp[2] + pH[2], -depth);
  const float4 sn = world ? make_float4(wno.x, wno.y, wno.z, __int_as_float(p))
                          : make_float4(wn[0], wn[1], wn[2], __int_as_float(p));
  if (slot < kMaxCon) {
    MprStage& st = sh.mpr[slot];
    st.pos[0] = sp.x; st.pos[1] = sp.y; st.pos[2] = sp.z; st.pos[3] = sp.w;
    st.nrm[0] = sn.x; st.nrm[1] = sn.y; st.nrm[2] = sn.z; st.nrm[3] = sn.w;
  } else if (crec) {               // (fused path: no record only if the pool ran out, which its sizing rules out)
    float4* stg = reinterpret_cast<float4*>(crec + (size_t)slot * kConStride + kMprStageOff);
    stg[0] = sp;
    stg[1] = sn;
  }
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
// Returns the env's number of convex contacts (uniform across its row).  Staged contacts j >= kMaxCon go to the
// env's HBM contact record (slot j, kMprStageOff; crec0: the record of the wave's first env).
template <bool kCells>
DEV int mpr_contacts(const DevModel* __restrict__ m, const Workspace& w, EnvShared* shm, float* crec0, float4* sep0, int lane,
                     int grp, bool valid) {
  constexpr int kConvex = SO100_NPAIR_CONVEX;
  constexpr int kRounds = (kConvex + kLanes - 1) / kLanes;   // 8
  static_assert(kRounds <= 8, "candidate masks hold 128 pairs");
  // each env's candidates go to its dynamics scratch (RNE cdd + tau: dead from the collision on; the contact
  // area holds the rows' EPA polytopes)
  // list items: q < kConvex the wave-shared pairs SO100_PAIR_MPR0 + q, then the EE marker's 9 (pairs 143..151), then
  // the slow table-hull pairs (kTableItem0 + k: pair SO100_NPAIR_BOX + k)
  constexpr int kTableItem0 = kConvex + SO100_NPAIR_MOCAPHULL;
  constexpr int kItems = kTableItem0 + SO100_NHULL;
  static_assert(kItems <= kSepPairs, "a separating-direction slot per item");
  static_assert(kItems <= (int)(sizeof(shm[0].ser.cdd) + sizeof(shm[0].ser.tau)), "an env's candidate list fits");
  static_assert(SO100_PAIR_MOCAPHULL0 == SO100_PAIR_MPR0 + kConvex, "the marker pairs follow the wave-shared pairs");
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
  const bool ee = m->ee;
  // the table-hull pairs outside the top-face rule (table_hull_class: at the table's edges and side faces, or deep):
  // lane k < SO100_NHULL of each env, appended to the env's list after the other convex pairs (items kTableItem0 + k)
  const bool tslow = table_hull_class(m, sh, lane, valid) == 1;
  const bool anyslow = __ballot(tslow) != 0ull;
  if (stotal == 0 && !ee && !anyslow) return 0;
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
  if (ee) {
    // EE variant: the marker box against the 9 link hulls (pairs 143..151, list items kConvex + k): both broadphase
    // stages on lanes 0..8 of the env's own row, the survivors appended to its list (they follow in pair order)
    bool cand = false;
    if (valid && lane < SO100_NPAIR_MOCAPHULL) {
      const int p = SO100_PAIR_MOCAPHULL0 + lane;
      if (mpr_sphere(m, sh, p)) {
        MprObj o;
        mpr_obj_setup(m, sh, p, o);
        cand = mpr_broadphase(m, o, -1 - m->pair_g2[p]);
      }
    }
    const uint64_t mb = __ballot(cand);
    if (cand) {
      const int base = grp == 0 ? c0 : grp == 1 ? c1 : grp == 2 ? c2 : c3;
      const uint32_t row = (uint32_t)((mb >> (grp * 16)) & 0xFFFFull);
      reinterpret_cast<uint8_t*>(&shm[grp].ser.cdd[0][0])[base + __popc(row & ((1u << lane) - 1u))] = (uint8_t)(kConvex + lane);
    }
    c0 += __popcll(mb & 0xFFFFull); c1 += __popcll(mb & (0xFFFFull << 16));
    c2 += __popcll(mb & (0xFFFFull << 32)); c3 += __popcll(mb & (0xFFFFull << 48));
  }
  if (anyslow) {
    // the slow table-hull pairs (14..22): both broadphase stages on lanes 0..8 of the env's own row (the table box
    // as obj1, as the bin boxes), the survivors appended to its list in hull order
    bool cand = false;
    if (tslow) {
      const int p = SO100_NPAIR_BOX + lane;
      if (mpr_sphere(m, sh, p)) {
        MprObj o;
        mpr_obj_setup(m, sh, p, o);
        cand = mpr_broadphase(m, o, lane);
      }
    }
    const uint64_t mb = __ballot(cand);
    if (cand) {
      const int base = grp == 0 ? c0 : grp == 1 ? c1 : grp == 2 ? c2 : c3;
      const uint32_t row = (uint32_t)((mb >> (grp * 16)) & 0xFFFFull);
      reinterpret_cast<uint8_t*>(&shm[grp].ser.cdd[0][0])[base + __popc(row & ((1u << lane) - 1u))] = (uint8_t)(kTableItem0 + lane);
    }
    c0 += __popcll(mb & 0xFFFFull); c1 += __popcll(mb & (0xFFFFull << 16));
    c2 += __popcll(mb & (0xFFFFull << 32)); c3 += __popcll(mb & (0xFFFFull << 48));
  }
  const int total = c0 + c1 + c2 + c3;
  if (total == 0) return 0;
  // the list's env offsets (pre_1..3 <= 3 x 129) and the envs' staged counts (<= 129 each) packed into one word each:
  // wave-uniform values held across the narrowphase's register peak (4 + 3 separate ones were spilled)
  static_assert(3 * kItems < 1024 && kItems < 256, "packed counts");
  const uint32_t prepk = (uint32_t)c0 | (uint32_t)(c0 + c1) << 10 | (uint32_t)(c0 + c1 + c2) << 20;
  __syncthreads();
  uint32_t fpk = 0u;                            // staged contacts of env e in byte e (wave-uniform)
  const int rounds = (total + kEnvsPerBlock - 1) / kEnvsPerBlock;
  auto pre_of = [&](int e) { return e == 0 ? 0 : (int)((prepk >> (10 * (e - 1))) & 1023u); };
  auto env_of = [&](int item) { return item >= pre_of(3) ? 3 : item >= pre_of(2) ? 2 : item >= pre_of(1) ? 1 : 0; };
  for (int rd = 0; rd < rounds; rd++) {
    const int item = kEnvsPerBlock * rd + grp;
    const bool act = item < total;
    const int ie = env_of(item);
    float depth = 0.f, dir[3] = {0.f, 0.f, 0.f}, pos[3] = {0.f, 0.f, 0.f};
    bool hit = false, world = false;
    float4 wpo = make_float4(0.f, 0.f, 0.f, 0.f), wno = wpo;    // table_face_snap's world-frame contact
    int p = SO100_PAIR_MPR0;
    if (act) {
      const int q = reinterpret_cast<const uint8_t*>(&shm[ie].ser.cdd[0][0])[item - pre_of(ie)];
      p = q < kTableItem0 ? SO100_PAIR_MPR0 + q : SO100_NPAIR_BOX + (q - kTableItem0);
      MprObj o;
      mpr_obj_setup(m, shm[ie], p, o);
      o.cells = kCells;
      // Temporal coherence: the direction that proved this pair separated in an earlier substep, re-checked on the
      // current geometry with one support evaluation: max over the Minkowski difference along it below -kSepTol
      // proves the pair separated now, which is GJK's own verdict (it returns no contact for a separated pair and
      // for a touching one), so the contact list is the same; otherwise GJK (+ EPA) runs as before, from its usual
      // start.  The cache never decides a contact: a stale entry (a reset, a far move) only fails the check.
      float4* const sc = sep0 + (size_t)ie * kSepPairs + q;
      const float4 c = *sc;
      bool proved = false;
      if (c.w != 0.f) {
        const float du[3] = {c.x, c.y, c.z};
        MprSup as;
        mpr_support(m, o, du, as, lane);
        proved = dot3(as.v, du) < -kSepTol;
      }
      if (!proved) {
        if (lane == 0 && c.w != 0.f) sc->w = 0.f;   // stale: invalidated (GJK stores a new one if it separates)
        hit = convex_penetration(m, o, depth, dir, pos, *reinterpret_cast<EpaPoly*>(&shm[grp].con[0]), lane, grp, sc);
        if (hit && m->convex != SO100_CONVEX_MPR) {
#ifndef SO100_NO_SNAP   // (A/B switch: no table-face snap, round 5's EPA contact)
          if (q >= kTableItem0) world = table_face_snap(m, shm[ie], p, dir, lane, o, wpo, wno);
#endif
          if (!world) {
            // the contact from EPA's final facet (its support ids came out in pos, its plane in dir and depth), by the
            // row, with the pair's MprObj still in hand (on the staging lane it had to be set up again: slower at
            // 8,192 envs, where the step waits for the heavy envs' convex items)
            float4 hd, hp;
            epa_contact(m, o, __float_as_uint(pos[0]), __float_as_uint(pos[1]), __float_as_uint(pos[2]), dir, depth, hd,
                        hp);
            dir[0] = hd.x; dir[1] = hd.y; dir[2] = hd.z;
            pos[0] = hp.x; pos[1] = hp.y; pos[2] = hp.z;
            depth = hp.w;
          }
        }
      }
    }
    // this round's hits, row g at bit 16 g; rows earlier in the list with the same env come first
    const uint64_t hb = __ballot(hit);
    uint32_t fnew = fpk;                        // the envs' staged counts after this round
#pragma unroll
    for (int g = 0; g < kEnvsPerBlock; g++) {
      const int it = kEnvsPerBlock * rd + g;
      if (it < total && ((hb >> (16 * g)) & 1ull)) fnew += 1u << (8 * env_of(it));
    }
    // fused path: an env whose staged contacts pass kMaxCon takes its pool record before they are staged there
    if constexpr (kCells) (void)ensure_rec<true>(w, shm, grp, lane, valid, (int)((fnew >> (8 * grp)) & 0xFFu), nullptr);
    int slot = (int)((fpk >> (8 * ie)) & 0xFFu);
#pragma unroll
    for (int g = 0; g < kEnvsPerBlock; g++) {
      const int it = kEnvsPerBlock * rd + g;
      const bool h = it < total && ((hb >> (16 * g)) & 1ull);
      if (g < grp && h && env_of(it) == ie) slot++;
    }
    if (hit && lane == 0) {
      // the env's record: the split path's per-env record (crec0: the wave's first env's), or the fused path's pool
      // record (crec0: the pool) if the env holds one (none only if the pool ran out, which its sizing rules out: the
      // contacts beyond kMaxCon are then not stored, and assemble counts them in ncon_dropped)
      float* const rb = kCells ? pool_rec(w, shm[0].rec, ie) : crec0 + (size_t)ie * kConEnv;
      stage_convex_hit(m, shm[ie], rb, slot, p, depth, dir, pos, world, wpo, wno);
    }
    fpk = fnew;
  }
  return (int)((fpk >> (8 * grp)) & 0xFFu);
}

}  // namespace so100
