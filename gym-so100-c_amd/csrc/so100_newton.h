// so100_newton.h — the constraint solve of one substep by MuJoCo's default solver: primal Newton
// (engine_solver.c mj_solNewton; the reference's model sets no solver, so_arm100.xml:4), restated as
// oracle/so100_oracle.c sol_newton (internal).
//
// Minimises c(a) = 1/2 (a - a_smooth)' M (a - a_smooth) + sum_rows s(J a - aref) over qacc a
// (frictionloss: Huber; limits: one-sided quadratic; elliptic contacts: three cone zones), with the
// Newton direction from the Cholesky factor of H = M + J' H_rows J and an exact line search.  Unlike PGS
// the result does not depend on the sweep order or an iteration cap: it is the problem's unique
// minimiser, reached in 1-7 iterations (1.2 on the bench workload).  The fp32 stops (DESIGN.md §3.3, §4 deviation
// 8): MuJoCo's gradient test, the Newton decrement after the Cholesky, and the quadratic-exact stop after a full
// step over which no row changed zone; MuJoCo's improvement test stays.
//
// Layout: one wave64 = 4 envs x 16 lanes (a DPP row per env, as the stage kernel).
//   * lane d < 12 owns dof d: qacc, qacc_smooth, the search direction, row d of H and of its Cholesky
//     factor (plus column d, collected during the factorisation for the back substitution), the
//     frictionloss row of dof d and, for d < 6, the joint-limit row;
//   * lane c owns contact c's block: jar, force, the 4x4 cone Hessian; the per-row scalar work of a
//     cost/gradient/Hessian evaluation runs once per row, in parallel over the rows;
//   * every dof lane holds J of its dof for contacts 0..kJReg-1 (one float4 per contact), so J x is a DPP
//     row reduction and J' f, J' H J come from DPP row broadcasts.  Contacts kJReg.. (rare: 0.4 % of envs
//     have more than 4) keep J in LDS (NewtonRows.jx) and take rolled loops with LDS broadcast reads and
//     ds_bpermute row shuffles: 32 fewer VGPRs, which the fused kernel needs for 3 waves per SIMD;
//   * contacts kMaxCon.. (the list holds every contact, up to kConCap; beyond 16 is rare, a jaw jammed into
//     the bin walls) live in the env's HBM contact record, in blocks of 16 (lane k owns contact kMaxCon + 16 b
//     + k): J, aref / R / cone coefficients, and the solve's per-contact state (jar, J s, force), read back
//     through L2 in rolled loops behind wave-uniform branches that the common case skips.
//
// The problem arrives as NewtonRows, one lane's share of it.  The fused step kernel (so100_step.hip
// so100_fused_kernel) hands it over in registers from the assembly of the same wave; the split path
// stores it in the HBM record (so100_device.h NewtonHdr) and so100_newton_kernel loads it back.
#pragma once
#include "so100.h"
#include "so100_common.h"

namespace so100 {

// One lane's share of a substep's Newton problem (its rows of the record).
constexpr int kJReg = 8;               // contacts whose J rows stay in VGPRs
constexpr int kJLds = kMaxCon - kJReg;  // the others' J rows: LDS [kJLds][SO100_NV] float4 per env
struct NewtonRows {
  float qs, warm, fr_aref;              // dof lanes: qacc_smooth, warmstart, frictionloss aref
  float lim_s, lim_aref, lim_R;         // lanes < 6: joint-limit side (+-1, 0 = inactive), aref, R
  float mrow[6];                        // lanes < 6: row of the arm's M (incl. armature)
  float mcd;                            // lanes 6..11: the cube's diagonal mass
  int ncon;                             // the env's contact count
  float4 J[kJReg];                      // dof lanes: J of this dof, contact c's 4 rows (0 beyond ncon)
  float4* jx;                           // LDS: J of contacts kJReg + i at jx[i * SO100_NV + dof] (0 beyond ncon)
  float4 c_aref, c_R, c_mu;             // lane c < ncon: contact c's aref, R, (cone mu, friction0, friction1)
};

// The solve's square roots and reciprocals on its serial chains: the hardware v_sqrt / v_rcp (1 ulp) instead of
// the IEEE sequences (a dozen dependent instructions each).
DEV float nsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
DEV float nrcp(float x) { return __builtin_amdgcn_rcpf(x); }

// MuJoCo mj_constraintUpdate (primal), elliptic contact block at jar: cost, force f = -dc/djar, and the
// cost Hessian (upper triangle 00 01 02 03 11 12 13 22 23 33); returns the cone zone: 0 top (no force), 1 bottom
// (quadratic), 2 middle.  Oracle block_eval.
DEV int cone_eval(const float* jar, const float* D, float Dm, float mu, float fr0, float fr1, float& cost, float* f,
                  float* h) {
  const float fr[4] = {mu, fr0, fr0, fr1};
  float U[4];
#pragma unroll
  for (int k = 0; k < 4; k++) U[k] = jar[k] * fr[k];
  const float T = nsqrt(U[1] * U[1] + U[2] * U[2] + U[3] * U[3]);
  const float N = U[0];
  cost = 0.f;
#pragma unroll
  for (int k = 0; k < 4; k++) f[k] = 0.f;
#pragma unroll
  for (int k = 0; k < 10; k++) h[k] = 0.f;
  if (N >= mu * T || (T <= 0.f && N >= 0.f)) return 0;                        // top zone: no force
  if (mu * N + T <= 0.f || (T <= 0.f && N < 0.f)) {                            // bottom zone: quadratic
#pragma unroll
    for (int k = 0; k < 4; k++) { f[k] = -D[k] * jar[k]; cost += 0.5f * D[k] * jar[k] * jar[k]; }
    h[0] = D[0]; h[4] = D[1]; h[7] = D[2]; h[9] = D[3];
    return 1;
  }
  // middle zone: c = 1/2 Dm (N - mu T)^2, g = d(N - mu T)/djar
  const float NmT = N - mu * T, invT = nrcp(T);
  float g[4];
  g[0] = mu;
#pragma unroll
  for (int k = 1; k < 4; k++) g[k] = -mu * U[k] * fr[k] * invT;
  cost = 0.5f * Dm * NmT * NmT;
#pragma unroll
  for (int k = 0; k < 4; k++) f[k] = -Dm * NmT * g[k];
  const float c2 = -Dm * NmT * mu, invT3 = invT * invT * invT;
  int q = 0;
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int l = k; l < 4; l++, q++) {
      float v = Dm * g[k] * g[l];
      if (k >= 1) v += c2 * fr[k] * fr[l] * ((k == l ? invT : 0.f) - U[k] * U[l] * invT3);
      h[q] = v;
    }
  return 2;
}
// The line search's view of a contact block: the cost's first and second derivatives at jar along v, as
// -f . v and v' H v, without forming H (in the middle zone H is rank one plus the friction rows' curvature, so
// v' H v = Dm (g.v)^2 + c2 (|fr v|^2 / T - (sum U_k fr_k v_k)^2 / T^3)): the same zones and the same values as
// cone_eval followed by f . v and v' sym4(h, v), in a third of the dependent operations; returns the zone as cone_eval.
DEV int cone_dir(const float* jar, const float* v, const float* D, float Dm, float mu, float fr0, float fr1,
                 float& fv, float& vhv) {
  const float U1 = jar[1] * fr0, U2 = jar[2] * fr0, U3 = jar[3] * fr1;
  const float T = nsqrt(U1 * U1 + U2 * U2 + U3 * U3);
  const float N = jar[0] * mu;
  fv = 0.f;
  vhv = 0.f;
  if (N >= mu * T || (T <= 0.f && N >= 0.f)) return 0;                        // top zone: no force
  if (mu * N + T <= 0.f || (T <= 0.f && N < 0.f)) {                            // bottom zone: quadratic
#pragma unroll
    for (int k = 0; k < 4; k++) { fv -= D[k] * jar[k] * v[k]; vhv += D[k] * v[k] * v[k]; }
    return 1;
  }
  const float NmT = N - mu * T, invT = nrcp(T);
  const float w1 = fr0 * v[1], w2 = fr0 * v[2], w3 = fr1 * v[3];
  const float s1 = w1 * w1 + w2 * w2 + w3 * w3, s2 = U1 * w1 + U2 * w2 + U3 * w3;
  const float gv = mu * v[0] - mu * invT * s2;                               // g . v
  fv = -Dm * NmT * gv;
  vhv = Dm * gv * gv - Dm * NmT * mu * (invT * s1 - invT * invT * invT * s2 * s2);
  return 2;
}
// frictionloss row (Huber) and joint-limit row (one-sided quadratic) at jar x; they return their zone (frictionloss:
// 2 linear above, 0 linear below, 1 quadratic; limit: 1 active)
DEV int fr_eval(float x, float fl, float R, float D, float& cost, float& f, float& h) {
  if (x >= R * fl) { f = -fl; cost = fl * x - 0.5f * R * fl * fl; h = 0.f; return 2; }
  if (x <= -R * fl) { f = fl; cost = -fl * x - 0.5f * R * fl * fl; h = 0.f; return 0; }
  f = -D * x; cost = 0.5f * D * x * x; h = D;
  return 1;
}
DEV int lim_eval(float x, bool on, float D, float& cost, float& f, float& h) {
  const bool act = on && x < 0.f;
  f = act ? -D * x : 0.f;
  cost = act ? 0.5f * D * x * x : 0.f;
  h = act ? D : 0.f;
  return act;
}
// h (upper triangle) times v
DEV float4 sym4(const float* h, float4 v) {
  return make_float4(h[0] * v.x + h[1] * v.y + h[2] * v.z + h[3] * v.w, h[1] * v.x + h[4] * v.y + h[5] * v.z + h[6] * v.w,
                     h[2] * v.x + h[5] * v.y + h[7] * v.z + h[8] * v.w, h[3] * v.x + h[6] * v.y + h[8] * v.z + h[9] * v.w);
}
DEV float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

// (M x)[dof]: the dense arm block by row broadcasts, the cube's diagonal masses
DEV float mul_m(const float* mrow, float mcd, float x) {
  float acc = mcd * x;
#pragma unroll
  for (int j = 0; j < 6; j++) acc += mrow[j] * bcast_row(x, j);
  return acc;
}
// ---------------------------------------------------------------- contacts beyond kMaxCon (the HBM record)
// slot of contact c in the env's contact record (so100_device.h: kConStride floats per contact)
DEV float* ovf_slot(float* crec, int c) { return crec + (size_t)c * kConStride; }
// J of contact c >= kMaxCon for dof `lane` (0 on the non-dof lanes and beyond the env's ncon: slots past the
// env's own contacts hold an earlier substep's rows)
DEV float4 ovf_j(const float* crec, int c, int lane, int ncon) {
  return (lane < SO100_NV && c < ncon) ? reinterpret_cast<const float4*>(crec + (size_t)c * kConStride + kJOff)[lane]
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
}
// contact c's Newton data from its record slot (as the resident contacts' NewtonRows fields: aref, D = 1 / R, the
// cone's mu, friction coefficients and middle-zone Dm; the assembly stores D and Dm, so100_step.hip)
struct OvfCon {
  float aref[4], D[4], mu, fr0, fr1, Dm;
};
DEV void ovf_load(const float* slot, OvfCon& o) {
  const float4 a = reinterpret_cast<const float4*>(slot)[0], D = reinterpret_cast<const float4*>(slot)[1];
  const float4 u = reinterpret_cast<const float4*>(slot)[2];
  o.aref[0] = a.x; o.aref[1] = a.y; o.aref[2] = a.z; o.aref[3] = a.w;
  o.D[0] = D.x; o.D[1] = D.y; o.D[2] = D.z; o.D[3] = D.w;
  o.mu = u.x; o.fr0 = u.y; o.fr1 = u.z;
  o.Dm = u.w;
}
DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
DEV void st4(float* p, const float* v) { *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]); }
// J x of the block of contacts b0 .. b0 + 15 on their owning lanes k = c - b0
DEV float4 ovf_rows(const float* crec, int b0, float x, int lane, int ncon, int ncon_max) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
  for (int k = 0; k < kLanes && b0 + k < ncon_max; k++) {
    const float4 j = ovf_j(crec, b0 + k, lane, ncon);
    const float a0 = rowsum16(j.x * x), a1 = rowsum16(j.y * x), a2 = rowsum16(j.z * x), a3 = rowsum16(j.w * x);
    if (lane == k) r = make_float4(a0, a1, a2, a3);
  }
  return r;
}
// J x (and J y) of the block of contacts b0 .. b0 + 15 on their owning lanes k = c - b0
DEV void ovf_rows2(const float* crec, int b0, float x, float y, int lane, int ncon, int ncon_max, float4& rx, float4& ry) {
  rx = make_float4(0.f, 0.f, 0.f, 0.f);
  ry = rx;
#pragma unroll 1
  for (int k = 0; k < kLanes && b0 + k < ncon_max; k++) {
    const float4 j = ovf_j(crec, b0 + k, lane, ncon);
    const float a0 = rowsum16(j.x * x), a1 = rowsum16(j.y * x), a2 = rowsum16(j.z * x), a3 = rowsum16(j.w * x);
    const float c0 = rowsum16(j.x * y), c1 = rowsum16(j.y * y), c2 = rowsum16(j.z * y), c3 = rowsum16(j.w * y);
    if (lane == k) { rx = make_float4(a0, a1, a2, a3); ry = make_float4(c0, c1, c2, c3); }
  }
}

// J of contact c >= kJReg for this lane's dof (LDS; 0 on the non-dof lanes)
DEV float4 jx_own(const NewtonRows& r, int c, int lane) {
  return lane < SO100_NV ? r.jx[(c - kJReg) * SO100_NV + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
}
// lane src of this lane's 16-lane row, src not a compile-time constant (ds_bpermute)
DEV float4 shfl_row4(float4 v, int src) {
  const int a = row_lane_addr(src);
  return make_float4(shfl_at(v.x, a), shfl_at(v.y, a), shfl_at(v.z, a), shfl_at(v.w, a));
}
// contact c's J x (4 rows) on lane c (the contacts present anywhere in the wave)
DEV float4 contact_rows(const NewtonRows& rw, float x, int lane, int ncon_max) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int c = 0; c < kJReg; c++) {
    if (c < ncon_max) {
      const float4* J = rw.J;
      const float v0 = rowsum16(J[c].x * x), v1 = rowsum16(J[c].y * x), v2 = rowsum16(J[c].z * x);
      const float v3 = rowsum16(J[c].w * x);
      if (lane == c) r = make_float4(v0, v1, v2, v3);
    }
  }
  for (int c = kJReg; c < ncon_max && c < kMaxCon; c++) {
    const float4 j = jx_own(rw, c, lane);
    const float v0 = rowsum16(j.x * x), v1 = rowsum16(j.y * x), v2 = rowsum16(j.z * x), v3 = rowsum16(j.w * x);
    if (lane == c) r = make_float4(v0, v1, v2, v3);
  }
  return r;
}
// contact_rows of two vectors in one pass: 8 independent row sums per contact instead of two chains of
// 4 behind their own uniform branches (the same sums in the same order: bitwise contact_rows twice)
DEV void contact_rows2(const NewtonRows& rw, float x, float y, int lane, int ncon_max, float4& rx, float4& ry) {
  rx = make_float4(0.f, 0.f, 0.f, 0.f);
  ry = rx;
#pragma unroll
  for (int c = 0; c < kJReg; c++) {
    if (c < ncon_max) {
      const float4 j = rw.J[c];
      const float a0 = rowsum16(j.x * x), a1 = rowsum16(j.y * x), a2 = rowsum16(j.z * x), a3 = rowsum16(j.w * x);
      const float b0 = rowsum16(j.x * y), b1 = rowsum16(j.y * y), b2 = rowsum16(j.z * y), b3 = rowsum16(j.w * y);
      if (lane == c) { rx = make_float4(a0, a1, a2, a3); ry = make_float4(b0, b1, b2, b3); }
    }
  }
  for (int c = kJReg; c < ncon_max && c < kMaxCon; c++) {
    const float4 j = jx_own(rw, c, lane);
    const float a0 = rowsum16(j.x * x), a1 = rowsum16(j.y * x), a2 = rowsum16(j.z * x), a3 = rowsum16(j.w * x);
    const float b0 = rowsum16(j.x * y), b1 = rowsum16(j.y * y), b2 = rowsum16(j.z * y), b3 = rowsum16(j.w * y);
    if (lane == c) { rx = make_float4(a0, a1, a2, a3); ry = make_float4(b0, b1, b2, b3); }
  }
}

// The split path's HBM record (so100_device.h NewtonHdr): the stage kernel stores a lane's rows, the
// Newton kernel loads them back.  J is stored by the stage as it is computed (so100_step.hip).
// (M goes first, as soon as the CRBA has it: the stage reuses its LDS for collision.)
DEV void newton_mass_store(const Workspace& w, int e, int lane, const NewtonRows& r) {
  float* hd = w.hdr + (size_t)e * kHdrEnv;
  if (lane < 6) {
#pragma unroll
    for (int j = 0; j < 6; j++) hd[N_M + 6 * lane + j] = r.mrow[j];
  } else if (lane < SO100_NV) {
    hd[N_MC + lane - 6] = r.mcd;
  }
}
DEV void newton_rows_store(const Workspace& w, int e, int lane, const NewtonRows& r) {
  float* hd = w.hdr + (size_t)e * kHdrEnv;
  float* crec = w.con + (size_t)e * kConEnv;
  if (lane < r.ncon) {
    float4* cs = reinterpret_cast<float4*>(crec + lane * kConStride);
    cs[0] = r.c_aref;
    cs[1] = r.c_R;
    cs[2] = r.c_mu;
  }
  if (lane < SO100_NV) { hd[N_QS + lane] = r.qs; hd[N_WARM + lane] = r.warm; hd[N_FRAREF + lane] = r.fr_aref; }
  if (lane < 6) { hd[N_LIMS + lane] = r.lim_s; hd[N_LIMAREF + lane] = r.lim_aref; hd[N_LIMR + lane] = r.lim_R; }
  if (lane == 0) hd[H_NCON] = __int_as_float(r.ncon);
}

// jx: the env's LDS area for the J rows of contacts kJReg.. (a barrier must follow before the solve)
DEV void newton_rows_load(const Workspace& w, int e, int lane, bool valid, float4* jx, NewtonRows& r) {
  const bool dof = lane < SO100_NV;
  const float* __restrict__ hd = w.hdr + (size_t)e * kHdrEnv;
  r.qs = dof ? hd[N_QS + lane] : 0.f;
  r.warm = dof ? hd[N_WARM + lane] : 0.f;
  r.fr_aref = dof ? hd[N_FRAREF + lane] : 0.f;
  r.lim_s = 0.f; r.lim_aref = 0.f; r.lim_R = 1.f;
  if (lane < 6) {
    r.lim_s = hd[N_LIMS + lane];
    r.lim_aref = hd[N_LIMAREF + lane];
    r.lim_R = hd[N_LIMR + lane];
  }
#pragma unroll
  for (int j = 0; j < 6; j++) r.mrow[j] = lane < 6 ? hd[N_M + 6 * lane + j] : 0.f;
  r.mcd = (lane >= 6 && dof) ? hd[N_MC + lane - 6] : 0.f;
  r.ncon = valid ? __float_as_int(hd[H_NCON]) : 0;
  const int ncon_max = wave_max_row(r.ncon);
  const float* __restrict__ crec = w.con + (size_t)e * kConEnv;
#pragma unroll
  for (int c = 0; c < kJReg; c++) {
    r.J[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < ncon_max && c < r.ncon && dof) r.J[c] = reinterpret_cast<const float4*>(crec + c * kConStride + kJOff)[lane];
  }
  for (int c = kJReg; c < ncon_max && c < kMaxCon; c++) {
    float4 j = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < r.ncon && dof) j = reinterpret_cast<const float4*>(crec + c * kConStride + kJOff)[lane];
    if (dof) jx[(c - kJReg) * SO100_NV + lane] = j;
  }
  r.jx = jx;
  r.c_aref = make_float4(0.f, 0.f, 0.f, 0.f);
  r.c_R = make_float4(1.f, 1.f, 1.f, 1.f);
  r.c_mu = make_float4(1.f, 1.f, 1.f, 0.f);
  if (lane < r.ncon) {
    const float4* cb = reinterpret_cast<const float4*>(crec + lane * kConStride);
    r.c_aref = cb[0];
    r.c_R = cb[1];
    r.c_mu = cb[2];
  }
}

// Diagnostics of a solve (debug buffer rows): the final frictionloss force of the lane's dof, contact
// `lane`'s force (normal, then its friction rows), the iteration count, the last cost improvement, and the
// phase stamps.
struct NewtonDiag {
  float f_fr, f_n, f_t[3], impr;
  int iters;
#ifdef SO100_STAMPS
  unsigned long long st[8];
#endif
};
DEV void newton_diag_write(float* dbg, int lane, bool valid, float qacc, const NewtonDiag& d) {
  if (!valid) return;
#ifdef SO100_STAMPS
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) dbg[88 + k] = (float)d.st[k];
  }
#endif
  if (lane < SO100_NV) { dbg[4 + lane] = qacc; dbg[76 + lane] = d.f_fr; }
  if (lane < kMaxCon) {
    dbg[32 + lane] = d.f_n;
#pragma unroll
    for (int k = 0; k < 3; k++) dbg[96 + 3 * lane + k] = d.f_t[k];
  }
  if (lane == 0) { dbg[1] = (float)d.iters; dbg[2] = d.impr; }
}

// The debug record's entries of the contacts beyond kMaxCon (include/so100.h SO100_DBG_STRIDE: from
// SO100_DBG_OVF, 6 floats per contact: dist, pair, normal force, 3 friction forces), from the env's contact record
// after the last solve: the forces at the final iterate's jar, as newton_diag_write's for the resident contacts.
DEV void newton_diag_write_ovf(float* dbg, const float* crec, int ncon, int lane) {
  for (int c = kMaxCon + lane; c < ncon; c += kLanes) {
    const float* sl = crec + (size_t)c * kConStride;
    OvfCon o;
    ovf_load(sl, o);
    const float4 j4 = ld4(sl + kOvfJc);
    const float x[4] = {j4.x, j4.y, j4.z, j4.w};
    float cc, fo[4], ho[10];
    cone_eval(x, o.D, o.Dm, o.mu, o.fr0, o.fr1, cc, fo, ho);
    float* d = dbg + SO100_DBG_OVF + 6 * (c - kMaxCon);
    d[0] = sl[kGeoDist];
    d[1] = (float)__float_as_int(sl[kGeoPair]);
#pragma unroll
    for (int k = 0; k < 4; k++) d[2 + k] = fo[k];
  }
}

// Solve one env's substep problem (its 16 lanes); returns qacc on the dof lanes.  want_diag: fill diag, the
// diagnostics for the debug row, written by the caller (the row's address is then not held live across
// the solve).  rec(): the env's HBM contact record (contacts >= kMaxCon), computed only where such contacts exist.
// kOvf: the contacts beyond kMaxCon are handled (the wave holds an env with more than kMaxCon); the callers
// instantiate both and choose per wave (newton_solve_any), so the common solve carries none of that code (a
// same-box A/B measured the overflow paths inside the one solve at -3.0 % env steps/s at 65,536 envs)
template <bool kOvf, class RecFn>
DEV float newton_solve(const DevModel* __restrict__ m, const NewtonRows& r, int lane, bool valid, bool want_diag,
                       NewtonDiag& diag, RecFn rec) {
  const bool dof = lane < SO100_NV;
  STAMP_DECL
  STAMP(-1);
  const float qs = r.qs, warm = r.warm, fr_aref = r.fr_aref;
  const float fr_fl = dof ? m->fr_floss[lane] : 0.f;
  const float fr_R = dof ? m->fr_R[lane] : 1.f;
  const float fr_D = 1.f / fr_R;
  const float lim_s = lane < 6 ? r.lim_s : 0.f, lim_aref = lane < 6 ? r.lim_aref : 0.f;
  const float lim_D = lane < 6 ? 1.f / r.lim_R : 0.f;
  const bool lim_on = lim_s != 0.f;
  const float* mrow = r.mrow;
  const float mcd = r.mcd;
  const int ncon = r.ncon;
  const int ncon_max = wave_max_row(ncon);
  const float4* J = r.J;                  // contacts < kJReg; the others: r.jx (LDS)
  const bool own = lane < ncon;                   // lane c owns contact c
  float c_aref[4] = {0.f, 0.f, 0.f, 0.f}, c_D[4] = {1.f, 1.f, 1.f, 1.f}, c_mu = 1.f, c_fr0 = 1.f, c_fr1 = 1.f;
  if (own) {
    c_aref[0] = r.c_aref.x; c_aref[1] = r.c_aref.y; c_aref[2] = r.c_aref.z; c_aref[3] = r.c_aref.w;
    c_D[0] = 1.f / r.c_R.x; c_D[1] = 1.f / r.c_R.y; c_D[2] = 1.f / r.c_R.z; c_D[3] = 1.f / r.c_R.w;
    c_mu = r.c_mu.x; c_fr0 = r.c_mu.y; c_fr1 = r.c_mu.z;
  }
  const float c_Dm = c_D[0] / (c_mu * c_mu * (1.f + c_mu * c_mu));   // the middle zone's Dm (oracle block_eval)

  // cost of the rows this lane owns at (frictionloss / limit jar of its dof, contact jar)
  auto rows_cost = [&](float xfr, float xlim, const float* xc) {
    float cost = 0.f, f, h, cc, fc[4], hc[10];
    if (dof) { fr_eval(xfr, fr_fl, fr_R, fr_D, cc, f, h); cost += cc; }
    lim_eval(xlim, lim_on, lim_D, cc, f, h);
    cost += cc;
    if (own) { cone_eval(xc, c_D, c_Dm, c_mu, c_fr0, c_fr1, cc, fc, hc); cost += cc; }
    return cost;
  };

  STAMP(0);
  // ---------------- start: the warmstart if its cost is below qacc_smooth's (mj_fwdConstraint)
  // The start's a - a_smooth, M(a - a_smooth), Gauss term and cost are the chosen candidate's, already
  // evaluated for the choice (at qacc_smooth: exactly 0, 0, 0 and its row cost), not evaluated again.
  float qacc, jc[4], ev, Me, gauss, cost;
  {
    float4 jw, js;
    contact_rows2(r, warm, qs, lane, ncon_max, jw, js);
    const float xw[4] = {jw.x - c_aref[0], jw.y - c_aref[1], jw.z - c_aref[2], jw.w - c_aref[3]};
    const float xs[4] = {js.x - c_aref[0], js.y - c_aref[1], js.z - c_aref[2], js.w - c_aref[3]};
    const float ew = warm - qs;
    const float mew = mul_m(mrow, mcd, ew);
    const float gw = 0.5f * rowsum16(dof ? ew * mew : 0.f);
    float cwl = rows_cost(warm - fr_aref, lim_s * warm - lim_aref, xw);
    float csl = rows_cost(qs - fr_aref, lim_s * qs - lim_aref, xs);
    if (kOvf && ncon_max > kMaxCon) {
      // contacts beyond kMaxCon: their jar at both candidates, the block's costs on the owning lanes; the
      // candidates go to the record (the chosen one becomes the iterate's jar below)
      float* crec = rec();
      for (int b0 = kMaxCon; b0 < ncon_max; b0 += kLanes) {
        float4 ow, os;
        ovf_rows2(crec, b0, warm, qs, lane, ncon, ncon_max, ow, os);
        const int c = b0 + lane;
        if (c < ncon) {
          float* sl = ovf_slot(crec, c);
          OvfCon o;
          ovf_load(sl, o);
          const float yw[4] = {ow.x - o.aref[0], ow.y - o.aref[1], ow.z - o.aref[2], ow.w - o.aref[3]};
          const float ys[4] = {os.x - o.aref[0], os.y - o.aref[1], os.z - o.aref[2], os.w - o.aref[3]};
          float cc, fc[4], hc[10];
          cone_eval(yw, o.D, o.Dm, o.mu, o.fr0, o.fr1, cc, fc, hc);
          cwl += cc;
          cone_eval(ys, o.D, o.Dm, o.mu, o.fr0, o.fr1, cc, fc, hc);
          csl += cc;
          st4(sl + kOvfJc, yw);
          st4(sl + kOvfJs, ys);
        }
      }
    }
    const float cw = gw + rowsum16(cwl);
    const float cs = rowsum16(csl);
    const bool use_w = cw < cs;
    if (kOvf && ncon_max > kMaxCon && !use_w) {
      float* crec = rec();
      for (int c = kMaxCon + lane; c < ncon; c += kLanes) {
        float* sl = ovf_slot(crec, c);
        *reinterpret_cast<float4*>(sl + kOvfJc) = ld4(sl + kOvfJs);
      }
    }
    qacc = use_w ? warm : qs;
#pragma unroll
    for (int k = 0; k < 4; k++) jc[k] = use_w ? xw[k] : xs[k];
    ev = use_w ? ew : 0.f;                                // a - a_smooth
    Me = use_w ? mew : 0.f;
    gauss = use_w ? gw : 0.f;
    cost = use_w ? cw : cs;
  }
  float jfr = qacc - fr_aref, jlim = lim_s * qacc - lim_aref;
  const float scale = m->pgs_scale, tolerance = m->tolerance;
  STAMP(1);

  bool done = !valid;
  int iters = 0;
  float last_impr = 0.f;
  for (int it = 0; it < m->iterations; it++) {
    if (__ballot(!done) == 0ull) break;
    if (!done) {
      // ---- rows at the current point: forces and Hessians
      float c0, f_fr = 0.f, h_fr = 0.f, f_lim, h_lim, fc[4], hc[10];
      int zf = 0;
      if (dof) zf = fr_eval(jfr, fr_fl, fr_R, fr_D, c0, f_fr, h_fr);
      const int zl = lim_eval(jlim, lim_on, lim_D, c0, f_lim, h_lim);
      const int zc = cone_eval(jc, c_D, c_Dm, c_mu, c_fr0, c_fr1, c0, fc, hc);
      // the rows' zones at the iterate, for the quadratic-exact stop (frictionloss rows only where they exist)
      const int z0 = (fr_fl > 0.f ? zf : 0) | zl << 2 | (own ? zc : 0) << 3;
      if (!own) {
#pragma unroll
        for (int k = 0; k < 4; k++) fc[k] = 0.f;
#pragma unroll
        for (int k = 0; k < 10; k++) hc[k] = 0.f;
      }
      // ---- gradient M (a - a_smooth) - J' f
      // gab: the gradient's terms in absolute value (the Gauss row, each row block's J' f), the scale of its rounding
      float grad = Me - f_fr - lim_s * f_lim;
      float gab = fabsf(Me) + fabsf(f_fr) + fabsf(lim_s * f_lim);
#pragma unroll
      for (int c = 0; c < kJReg; c++) {
        if (c < ncon_max) {
          const float t = dot4(J[c], bcast_row4(make_float4(fc[0], fc[1], fc[2], fc[3]), c));
          grad -= t;
          gab += fabsf(t);
        }
      }
      for (int c = kJReg; c < ncon_max && c < kMaxCon; c++) {
        const float t = dot4(jx_own(r, c, lane), shfl_row4(make_float4(fc[0], fc[1], fc[2], fc[3]), c));
        grad -= t;
        gab += fabsf(t);
      }
      if (kOvf && ncon_max > kMaxCon) {
        // contacts beyond kMaxCon: forces at the iterate's jar (kept in the record for c'(0) below), J' f
        float* crec = rec();
        for (int b0 = kMaxCon; b0 < ncon_max; b0 += kLanes) {
          const int c = b0 + lane;
          float fo[4] = {0.f, 0.f, 0.f, 0.f};
          if (c < ncon) {
            float* sl = ovf_slot(crec, c);
            OvfCon o;
            ovf_load(sl, o);
            const float4 j4 = ld4(sl + kOvfJc);
            const float x[4] = {j4.x, j4.y, j4.z, j4.w};
            float cc, hc[10];
            cone_eval(x, o.D, o.Dm, o.mu, o.fr0, o.fr1, cc, fo, hc);
            st4(sl + kOvfF, fo);
          }
#pragma unroll 1
          for (int k = 0; k < kLanes && b0 + k < ncon_max; k++) {
            const float t = dot4(ovf_j(crec, b0 + k, lane, ncon), shfl_row4(make_float4(fo[0], fo[1], fo[2], fo[3]), k));
            grad -= t;
            gab += fabsf(t);
          }
        }
      }
      grad = dof ? grad : 0.f;
      const float gn = nsqrt(rowsum16(grad * grad));
      // (A/B switch, measured and not kept: -DSO100_GNOISE_K=k stops at the gradient's own rounding, every dof's within
      // k float epsilons of its terms' magnitudes, before the Hessian and the Cholesky: 1.34 instead of 2.15
      // factorizations per substep on the bench workload and +2 % env steps/s at 65,536 envs, but blind to the
      // curvature — in the deep Base folds a gradient at the rounding of centimetre-deep contact forces still moved the
      // light dofs, and the GPU's qvel p99 there went 1.8e-3 -> 1.4e-2 against a floor of 2.7e-3)
#ifdef SO100_GNOISE_K
      const bool gquiet =
          rowsum16((dof && !(fabsf(grad) <= SO100_GNOISE_K * 1.1920929e-7f * gab)) ? 1.f : 0.f) == 0.f;
#else
      const bool gquiet = false;
      (void)gab;
#endif
      STAMP(2);
      if (scale * gn < tolerance || gquiet) {
        done = true;
      } else {
        // ---- Hessian row `lane`: M + diag(frictionloss, limit) + sum_c J_c' H_c J_c
        float H[SO100_NV];
#pragma unroll
        for (int j = 0; j < SO100_NV; j++) {
          H[j] = j < 6 ? mrow[j] : 0.f;
          if (lane == j) H[j] += mcd + h_fr + h_lim;
        }
#pragma unroll
        for (int c = 0; c < kJReg; c++) {
          // (skipping contacts whose Hessian is zero in every env of the wave, or zero J columns, measured
          // 2% slower: the uniform branches cost more than the DPP/FMA they save)
          if (c < ncon_max) {
            float hb[10];
#pragma unroll
            for (int k = 0; k < 10; k++) hb[k] = bcast_row(hc[k], c);
            const float4 w = sym4(hb, J[c]);
#pragma unroll
            for (int j = 0; j < SO100_NV; j++) H[j] += dot4(w, bcast_row4(J[c], j));
          }
        }
        for (int c = kJReg; c < ncon_max && c < kMaxCon; c++) {       // J from LDS: one broadcast read per dof
          float hb[10];
#pragma unroll
          for (int k = 0, a = row_lane_addr(c); k < 10; k++) hb[k] = shfl_at(hc[k], a);
          const float4* jc_l = r.jx + (c - kJReg) * SO100_NV;
          const float4 w = sym4(hb, jx_own(r, c, lane));
#pragma unroll
          for (int j = 0; j < SO100_NV; j++) H[j] += dot4(w, jc_l[j]);
        }
        if (kOvf && ncon_max > kMaxCon) {
          // contacts beyond kMaxCon: J' H_c J with J from the record (the Hessian re-evaluated at the iterate)
          float* crec = rec();
          for (int b0 = kMaxCon; b0 < ncon_max; b0 += kLanes) {
            const int c = b0 + lane;
            float ho[10];
#pragma unroll
            for (int k = 0; k < 10; k++) ho[k] = 0.f;
            if (c < ncon) {
              float* sl = ovf_slot(crec, c);
              OvfCon o;
              ovf_load(sl, o);
              const float4 j4 = ld4(sl + kOvfJc);
              const float x[4] = {j4.x, j4.y, j4.z, j4.w};
              float cc, fo[4];
              cone_eval(x, o.D, o.Dm, o.mu, o.fr0, o.fr1, cc, fo, ho);
            }
#pragma unroll 1
            for (int k = 0; k < kLanes && b0 + k < ncon_max; k++) {
              float hb[10];
#pragma unroll
              for (int t = 0, a = row_lane_addr(k); t < 10; t++) hb[t] = shfl_at(ho[t], a);
              const float4 w = sym4(hb, ovf_j(crec, b0 + k, lane, ncon));
              const bool live = b0 + k < ncon;          // this env's contact (else J is 0)
              const float4* jrow = reinterpret_cast<const float4*>(crec + (size_t)(b0 + k) * kConStride + kJOff);
#pragma unroll
              for (int j = 0; j < SO100_NV; j++) H[j] += live ? dot4(w, jrow[j]) : 0.f;
            }
          }
        }
        STAMP(3);
        // ---- Cholesky H = L L' (lane i: row i of L; lc: column i, gathered from the broadcasts)
        float lc[SO100_NV], dinv = 1.f;
#pragma unroll
        for (int k = 0; k < SO100_NV; k++) {
          const float dkk = bcast_row(H[k], k);
          const float inv = __builtin_amdgcn_rsqf(fmaxf(dkk, kMinVal));   // 1 / L_kk: one v_rsq (1 ulp)
          const float lik = H[k] * inv;
          if (lane >= k) H[k] = lik;
          if (lane == k) dinv = inv;
#pragma unroll
          for (int j = k + 1; j < SO100_NV; j++) {
            const float ljk = bcast_row(lik, j);
            if (lane > k) H[j] -= lik * ljk;
            if (lane == k) lc[j] = ljk;
          }
        }
        // ---- search direction s = -H^-1 grad: L y = -grad, L' s = y
        float y = -grad;
#pragma unroll
        for (int k = 0; k < SO100_NV; k++) {
          const float yk = bcast_row(y * dinv, k);
          if (lane == k) y = yk;
          else if (lane > k) y -= H[k] * yk;
        }
        float sv = y;
#pragma unroll
        for (int k = SO100_NV - 1; k >= 0; k--) {
          const float xk = bcast_row(sv * dinv, k);
          if (lane == k) sv = xk;
          else if (lane < k) sv -= lc[k] * xk;
        }
        sv = dof ? sv : 0.f;
        STAMP(4);
        // ---- exact line search on c(a + alpha s): safeguarded 1-D Newton on c'(alpha) (oracle line_search)
        const float Ms = mul_m(mrow, mcd, sv);
        const float A1 = rowsum16(dof ? Ms * ev : 0.f), A2 = rowsum16(dof ? Ms * sv : 0.f);
        const float4 js4 = contact_rows(r, sv, lane, ncon_max);
        const float jsc[4] = {js4.x, js4.y, js4.z, js4.w};
        const float sfr = sv, slim = lim_s * sv;
        float ovf_l10 = 0.f;                   // contacts beyond kMaxCon: -f . J s at alpha = 0
        if (kOvf && ncon_max > kMaxCon) {
          float* crec = rec();
          for (int b0 = kMaxCon; b0 < ncon_max; b0 += kLanes) {
            const float4 s4 = ovf_rows(crec, b0, sv, lane, ncon, ncon_max);
            const int c = b0 + lane;
            if (c < ncon) {
              float* sl = ovf_slot(crec, c);
              const float4 f4 = ld4(sl + kOvfF);
              ovf_l10 -= f4.x * s4.x + f4.y * s4.y + f4.z * s4.z + f4.w * s4.w;
              *reinterpret_cast<float4*>(sl + kOvfJs) = s4;
            }
          }
        }
        // (returns the rows' zones at alpha, as z0)
        auto derivs = [&](float al, float& d1, float& d2) -> int {
          float l1 = 0.f, l2 = 0.f, cc, f, h;
          int zf = 0, zc = 0;
          if (dof) { zf = fr_eval(jfr + al * sfr, fr_fl, fr_R, fr_D, cc, f, h); l1 -= f * sfr; l2 += h * sfr * sfr; }
          const int zl = lim_eval(jlim + al * slim, lim_on, lim_D, cc, f, h);
          l1 -= f * slim; l2 += h * slim * slim;
          if (own) {
            float x[4], fv, vhv;
#pragma unroll
            for (int k = 0; k < 4; k++) x[k] = jc[k] + al * jsc[k];
            zc = cone_dir(x, jsc, c_D, c_Dm, c_mu, c_fr0, c_fr1, fv, vhv);
            l1 -= fv;
            l2 += vhv;
          }

          if (kOvf && ncon_max > kMaxCon) {
            float* crec = rec();
            for (int c = kMaxCon + lane; c < ncon; c += kLanes) {
              float* sl = ovf_slot(crec, c);
              OvfCon o;
              ovf_load(sl, o);
              const float4 j4 = ld4(sl + kOvfJc), s4 = ld4(sl + kOvfJs);
              const float x[4] = {j4.x + al * s4.x, j4.y + al * s4.y, j4.z + al * s4.z, j4.w + al * s4.w};
              const float v[4] = {s4.x, s4.y, s4.z, s4.w};
              float fv, vhv;
              cone_dir(x, v, o.D, o.Dm, o.mu, o.fr0, o.fr1, fv, vhv);
              l1 -= fv;
              l2 += vhv;
            }
          }
          d1 = rowsum16(l1) + A1 + al * A2;
          d2 = rowsum16(l2) + A2;
          return (fr_fl > 0.f ? zf : 0) | zl << 2 | zc << 3;
        };
        // c'(0) from the forces already evaluated at the current point (= derivs(0)'s d1)
        float d10;
        {
          float l1 = 0.f;
          l1 -= f_fr * sfr;
          l1 -= f_lim * slim;
          l1 -= fc[0] * jsc[0] + fc[1] * jsc[1] + fc[2] * jsc[2] + fc[3] * jsc[3];
          if (kOvf && ncon_max > kMaxCon) l1 += ovf_l10;
          d10 = rowsum16(l1) + A1;
        }
        // the Newton decrement (fp32 stop, round 6; oracle NEWTON_DECREMENT): a full step along s = -H^-1 g would
        // lower the cost by -c'(0) / 2; below MuJoCo's tolerance (scaled) the solve is done.  It replaces the relative
        // cost-improvement stop of rounds 3-5 (1e-6 of |cost|), which ended EE solves (the weld folded into M: a large
        // cost) short of the minimiser; MuJoCo's own stops are below fp32 resolution here (DESIGN.md §4 deviation 8)
#ifdef SO100_NEWTON_RELSTOP   // (A/B switch: rounds 3-5's relative cost-improvement stop instead)
        const bool converged = false;
#else
        const bool converged = scale * (-0.5f * d10) < tolerance;
#endif
        float alpha = 0.f;
        int z1 = -1;                           // the line search took alpha = 1 at its first evaluation: the zones there
        if (!converged && d10 < 0.f) {
          // fp32 stops (oracle LS_TOL / LS_STEP): MuJoCo's ls_tolerance 0.01 on |c'|, or a relative step 1e-4
          const float tol_ls = 1e-2f * -d10;
          float lo = 0.f, hi = -1.f;
          alpha = 1.f;
          for (int ls = 0; ls < 50; ls++) {
            float d1, d2;
            const int z = derivs(alpha, d1, d2);
            if (fabsf(d1) <= tol_ls) { if (ls == 0) z1 = z; break; }
            if (d1 < 0.f) lo = alpha; else hi = alpha;
            float nxt = d2 > 0.f ? alpha - d1 * nrcp(d2) : -1.f;
            if (hi >= 0.f) { if (!(nxt > lo && nxt < hi)) nxt = 0.5f * (lo + hi); }
            else if (!(nxt > lo)) nxt = 2.f * alpha;
            if (nxt == alpha) break;
            if (fabsf(nxt - alpha) <= 1e-4f * fabsf(alpha)) { alpha = nxt; break; }
            alpha = nxt;
          }
        }
        // the quadratic-exact stop (round 6; oracle NEWTON_QUADSTOP): a full step (alpha = 1 accepted at once) along
        // which no row changed zone and no contact is in the cone's middle zone (an env with contacts beyond kMaxCon
        // keeps MuJoCo's stops: its record's zones are not tracked).  The cost is then one quadratic on the whole
        // segment and the step, along its exact Hessian, lands on that quadratic's minimiser: the next gradient is
        // zero up to rounding, and evaluating it (a Hessian and a Cholesky for the decrement to confirm) is skipped
        const bool quad = rowsum16(z1 == z0 && (z0 >> 3) != 2 && ncon <= kMaxCon ? 0.f : 1.f) == 0.f;
        if (!converged) iters = it + 1;
        STAMP(5);
        if (alpha == 0.f) {
          done = true;
        } else {
          // ---- move; the new cost gives MuJoCo's improvement test
          qacc += alpha * sv;
          ev += alpha * sv;
          Me += alpha * Ms;
          jfr += alpha * sfr;
          jlim += alpha * slim;
#pragma unroll
          for (int k = 0; k < 4; k++) jc[k] += alpha * jsc[k];
          gauss += alpha * A1 + 0.5f * alpha * alpha * A2;
          float ncl = rows_cost(jfr, jlim, jc);
          if (kOvf && ncon_max > kMaxCon) {
            // contacts beyond kMaxCon: jar += alpha J s in the record, their cost at the new iterate
            float* crec = rec();
            for (int c = kMaxCon + lane; c < ncon; c += kLanes) {
              float* sl = ovf_slot(crec, c);
              OvfCon o;
              ovf_load(sl, o);
              const float4 j4 = ld4(sl + kOvfJc), s4 = ld4(sl + kOvfJs);
              const float x[4] = {j4.x + alpha * s4.x, j4.y + alpha * s4.y, j4.z + alpha * s4.z, j4.w + alpha * s4.w};
              st4(sl + kOvfJc, x);
              float cc, fo[4], ho[10];
              cone_eval(x, o.D, o.Dm, o.mu, o.fr0, o.fr1, cc, fo, ho);
              ncl += cc;
            }
          }
          const float nc = gauss + rowsum16(ncl);
          const float improvement = scale * (cost - nc);
          cost = nc;
          last_impr = improvement;
          // MuJoCo's test (the Newton decrement above is the fp32 stop that resolves)
#ifdef SO100_NEWTON_RELSTOP
          if (improvement < tolerance || improvement < 1e-6f * scale * fabsf(cost)) done = true;
#else
          if (improvement < tolerance) done = true;
#endif
#ifndef SO100_NO_QUADSTOP
          if (quad) done = true;
#endif
        }
        STAMP(6);
      }
    }
  }

  STAMP(7);
  if (want_diag) {
#ifdef SO100_STAMPS
#pragma unroll
    for (int k = 0; k < 8; k++) diag.st[k] = st_acc_[k];
#endif
    float cc, f_fr, h, fc[4], hc[10];
    fr_eval(jfr, fr_fl, fr_R, fr_D, cc, f_fr, h);
    cone_eval(jc, c_D, c_Dm, c_mu, c_fr0, c_fr1, cc, fc, hc);
    diag.f_fr = f_fr;
    diag.f_n = own ? fc[0] : 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) diag.f_t[k] = own ? fc[1 + k] : 0.f;
    diag.iters = iters;
    diag.impr = last_impr;
  }
  return qacc;
}

// the solve with or without the overflow paths, chosen per wave (uniform)
template <class RecFn>
DEV float newton_solve_any(const DevModel* __restrict__ m, const NewtonRows& r, int lane, bool valid, bool want_diag,
                           NewtonDiag& diag, RecFn rec) {
  const int ncon_max = wave_max_row(r.ncon);
  if (ncon_max > kMaxCon) return newton_solve<true>(m, r, lane, valid, want_diag, diag, rec);
  return newton_solve<false>(m, r, lane, valid, want_diag, diag, rec);
}

}  // namespace so100
