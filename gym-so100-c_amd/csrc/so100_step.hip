// so100_step.hip — MI355X (gfx950) batched SO-ARM100 bin-a-cube simulator: the hot path's kernels.
//
// Replaces, for N envs per launch, gym_so100/env.py:172-182 SO100Env.step ->
// single_arm.py:33-38 before_step -> dm_control Physics.step(10) (MuJoCo mj_step x10 + mj_step1)
// -> single_arm.py get_reward / get_observation -> env.py:130-146 packing.
//
// Execution model:
//   * one wave64 workgroup = 4 envs; each env owns a 16-lane "lane group" = one DPP row;
//   * the fused step kernel (Newton, the default) runs a wave's 4 envs through the 10 substeps and the
//     epilogue in one launch, the state in registers; the split path (PGS, or on request) runs per substep a
//     stage kernel (assembly -> HBM record) and a solver kernel (so100_newton.hip / so100_pgs.hip).
// This translation unit holds the substep assembly, the epilogue, the kernels and their launchers; the device
// functions they are built from live in the headers:
//   so100_dynamics.h  kinematics-to-qacc_smooth (CRBA, RNE, actuators, weld)   so100_task.h  task layer
//   so100_boxbox.h    box-box, hull-table collision                             so100_rows.h  contact rows
//   so100_convex.h    GJK + EPA / MPR mesh collider and its broadphase          so100_newton.h  Newton solve
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include "so100_device.h"
#include "so100.h"
#include "so100_common.h"
#include "so100_kin.h"
#include "so100_newton.h"
#include "so100_dynamics.h"
#include "so100_task.h"
#include "so100_boxbox.h"
#include "so100_convex.h"
#include "so100_rows.h"

namespace so100 {

// Newton data of a contact of pair p at distance dist with J qvel = cv (MuJoCo mj_makeImpedance / mj_diagApprox /
// mj_referenceConstraint for an elliptic contact): aref, R (normal, friction rows: impratio), and the cone's mu
// with the friction coefficients (DR friction scale on the cube's pairs)
DEV void newton_contact_rows(const DevModel* __restrict__ m, int p, float dist, const float* cv, float fscale, float4& aref,
                             float4& Rv, float4& mu) {
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
  aref = make_float4(-Bd * cv[0] - K * imp * (dist - m->pair_margin[p]), -Bd * cv[1], -Bd * cv[2], -Bd * cv[3]);
  Rv = make_float4(R[0], R[1], R[2], R[3]);
  mu = make_float4(mu0 * __builtin_amdgcn_sqrtf(R[1] * __builtin_amdgcn_rcpf(R[0])), mu0, mu1, 0.f);
}

// PGS data of one contact (pair p, distance dist; the row reductions cA = (J M^-1 J')_upper, cV = J qvel,
// cAc = J qacc_smooth, cW = J qacc_warmstart): impedance, regularisers, the warmstart force by MuJoCo's dual map,
// the eigen-decomposition of the cone-scaled friction block for the QCQP; the solver block to cs (record slot,
// layout so100_device.h), the warmstart force to cf and its dual cost to cost_part
DEV void pgs_contact_block(const DevModel* __restrict__ m, int p, float dist, float fscale, const float* cA, const float* cV,
                           const float* cAc, const float* cW, float4* cs, float* cf, float& cost_part) {
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

DEV int wave_max_i(int v) { return wave_max_row(v); }   // (so100_common.h)

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

// Contact `slot` of the env's list: slots < kMaxCon on chip (the LDS contact area), the rest in the env's HBM
// contact record (crec, kGeoOff: read back by contact_jac_ovf).  The list holds every contact (kConCap: every
// pair at its collider's maximum), so nothing is dropped.
DEV void store_contact(EnvShared& sh, float* crec, int slot, const float* fr, float p0, float p1, float p2, float dist,
                       int pair) {
  if (slot < kMaxCon) {
#pragma unroll
    for (int t = 0; t < 9; t++) sh.con[slot].g.frame[t] = fr[t];
    sh.con[slot].g.pos[0] = p0; sh.con[slot].g.pos[1] = p1;
    sh.con[slot].g.pos[2] = p2; sh.con[slot].g.pos[3] = dist;
    sh.con_dist[slot] = dist;
    sh.con_pair[slot] = pair;
  } else if (crec) {               // (fused path: no record only if the pool ran out, which its sizing rules out)
    float4* g = reinterpret_cast<float4*>(crec + (size_t)slot * kConStride + kGeoOff);
    g[0] = make_float4(p0, p1, p2, dist);
    g[1] = make_float4(fr[0], fr[1], fr[2], fr[3]);
    g[2] = make_float4(fr[4], fr[5], fr[6], fr[7]);
    g[3] = make_float4(fr[8], 0.f, 0.f, 0.f);
    g[4] = make_float4(__int_as_float(pair), dist, 0.f, 0.f);
  }
}

// write one box-box pair's contacts into slots base, base+1, ...
DEV void put_box_contacts(EnvShared& sh, float* crec, const PairContacts& pc, int base, int p) {
  // one frame per pair (every contact of a box pair shares its normal)
  float fr[9] = {pc.normal[0], pc.normal[1], pc.normal[2], 0, 0, 0, 0, 0, 0};
  if (pc.n > 0) make_frame(fr);
#pragma unroll
  for (int c = 0; c < SO100_MAXCONPAIR; c++) {
    if (c < pc.n) store_contact(sh, crec, base + c, fr, pc.pos[c][0], pc.pos[c][1], pc.pos[c][2], pc.dist[c], p);
  }
}

// Finger pads vs the table and the bin boxes (oracle collision(): collide_box_pair), one candidate list in pair
// order, run through the box-box collider 16 at a time (a wave runs as many rounds as its busiest env needs):
//   pairs 152..159 (pad i, table): a box against the table mesh, the cube-table rule (the exact separating-axis
//     minimum penetration, one contact: collide_pair's collapse); candidate when the pad's lowest point (its centre
//     z minus its half extent along world z) is within 1e-4 of top + margin (else the table's z axis separates);
//   pairs 160..199 (pad i, bin box j): a conservative test (the pad's bounding sphere against the static box, 3
//     pairs per lane), behind a wave-uniform prefilter (no pad near the bin's AABB: no candidates);
//   (EE variant) pairs 200..208 (cube | pad i, the mocap marker box) join the candidates.
// Contacts are appended after `tot` in pair order; returns the new total.
template <bool kFused>
DEV int pad_contacts(const DevModel* __restrict__ m, const Workspace& w, EnvShared& sh, float* crec, int lane, int grp,
                     bool valid, int tot) {
  static_assert(SO100_PAIR_PADBIN0 == SO100_PAIR_PAD0 + SO100_NPAD, "the pad-bin pairs follow the pad-table pairs");
  static_assert(SO100_PAIR_MOCAPBOX0 == SO100_PAIR_PADBIN0 + SO100_NPAIR_PADBIN, "the marker pairs follow the pad-bin pairs");
  static_assert(SO100_NPAD + SO100_NPAIR_PADBIN + SO100_NPAIR_MOCAPBOX <= 64, "one candidate mask");
  // ---- pad-table candidates and the pad-bin prefilter (lanes 0..7)
  bool tcand = false, nearbin = false;
  if (valid && lane < SO100_NPAD) {
    const int p = SO100_PAIR_PAD0 + lane, g = m->pair_g1[p];
    const int b = m->pair_b1[p];                  // = geom_body[g] (so100_create), loaded beside g
    const float* bm = sh.jaw_mat[b - 6];
    const float* gm = m->geom_mat[g];
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
    float ext = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) ext += fabsf(bm[6] * gm[k] + bm[7] * gm[3 + k] + bm[8] * gm[6 + k]) * m->geom_size[g][k];
    tcand = pc[2] - ext - m->table_top < m->pair_margin[p] + 1e-4f;
  }
  const bool anybin = __ballot(nearbin) != 0ull;
  uint64_t cm = (__ballot(tcand) >> (grp * 16)) & 0xFFull;      // bit j: pair SO100_PAIR_PAD0 + j
  // ---- pad-bin candidates (3 pairs per lane); the whole wave skips them when no pad is near the bin
#pragma unroll
  for (int r = 0; r < 3; r++) {
    if (!anybin) break;
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
    cm |= ((__ballot(cand) >> (grp * 16)) & 0xFFFFull) << (SO100_NPAD + 16 * r);
  }
  // EE variant: the cube and the pads against the marker box (pairs 200..208, after the pad-bin pairs in pair
  // order): every one a candidate (collide_pair's bounding spheres decide)
  if (m->ee && valid) cm |= ((1ull << SO100_NPAIR_MOCAPBOX) - 1ull) << (SO100_NPAD + SO100_NPAIR_PADBIN);
  const int ncand = __popcll(cm);
  const int rounds = (wave_max_i(ncand) + kLanes - 1) / kLanes;
  for (int r = 0; r < rounds; r++) {
    const int idx = r * kLanes + lane;
    int p = -1;
    if (idx < ncand) {
      uint64_t x = cm;
      for (int k = 0; k < idx; k++) x &= x - 1ull;
      p = SO100_PAIR_PAD0 + __ffsll((unsigned long long)x) - 1;
    }
    PairContacts pc;
    pc.n = 0;
    if (p >= 0) collide_pair(m, sh, p, pc);
    sh.cnt[lane] = pc.n;
    __syncthreads();
    int off = 0, sum = 0;
#pragma unroll
    for (int k = 0; k < kLanes; k++) { const int c = sh.cnt[k]; off += (k < lane) ? c : 0; sum += c; }
    crec = ensure_rec<kFused>(w, &sh - grp, grp, lane, valid, tot + sum, crec);
    put_box_contacts(sh, crec, pc, tot + off, p);
    tot += sum;
    __syncthreads();
  }
  return tot;
}

constexpr int kStageWaves = 3;      // waves per SIMD the stage kernel's register budget is sized for

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
  if (m->ee && lane < 7) {
    // the mocap pose with its quaternion normalised once per env step (mj_kinematics normalises mocap_quat; the weld
    // and the marker box read it every substep)
    const float* src = B.mocap ? B.mocap + (size_t)e * 7 : m->mocap0;
    float q[4] = {src[3], src[4], src[5], src[6]};
    quat_normalize(q);
    sh.mocap[lane] = lane < 3 ? src[lane] : lane == 3 ? q[0] : lane == 4 ? q[1] : lane == 5 ? q[2] : q[3];
  }
}

// S3, collision, of the wave's 4 envs: hulls vs the table, the convex pairs (staged in LDS), one box pair per lane, the
// pads; the contacts compacted in pair order into the env's list (sh.ncon: its length).  The first kMaxCon on chip,
// the rest in the env's HBM record: crec on the split path; on the fused path the pool record an env takes when its
// list passes kMaxCon (ensure_rec, before each phase's stores).  recbase: the split path's record of the wave's first
// env, or the fused path's pool; sep: the wave's first env's separating-direction cache.
#ifdef SO100_STAGE_STAMPS
#define SSTAMP_PARAMS , unsigned long long& sst_prev_, unsigned long long* sst_acc_
#define SSTAMP_PASS , sst_prev_, sst_acc_
#else
#define SSTAMP_PARAMS
#define SSTAMP_PASS
#endif
template <bool kFused>
DEV void collide(const DevModel* __restrict__ m, const Workspace& w, float* recbase, float4* sep, EnvShared& sh, int lane,
                 int grp, bool valid, float* crec SSTAMP_PARAMS) {
  const int nmpr = mpr_contacts<kFused>(m, w, &sh - grp, recbase, sep, lane, grp, valid);
  SSTAMP(7);
  float hx, hy, hz;
  const bool hfound = hull_table(m, sh, lane, grp, valid, hx, hy, hz);
  const uint32_t hrow = (uint32_t)((__ballot(hfound) >> (grp * 16)) & 0xFFFFull);
  SSTAMP(6);
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
    // the box, table-hull and convex contacts' total is known here, before any of them is stored
    crec = ensure_rec<kFused>(w, &sh - grp, grp, lane, valid, tot + __popc(hrow) + nmpr, crec);
    put_box_contacts(sh, crec, pc, off, lane);
    const int hslot = tot + __popc(hrow & ((1u << lane) - 1u));
    if (hfound) {
      float fr[9] = {0.f, 0.f, 1.f, 0, 0, 0, 0, 0, 0};
      opaque(fr[2]);            // a constant frame: built here, not hoisted out of the fused substep loop
      make_frame(fr);
      const float top = m->table_top;
      store_contact(sh, crec, hslot, fr, hx, hy, 0.5f * (hz + top), hz - top, SO100_NPAIR_BOX + lane);
    }
    tot += __popc(hrow);
    // the convex collider's contacts, staged in order: staged contact j is contact tot + j (staged j >= kMaxCon
    // in the record, mpr_contacts)
    if (lane < nmpr) {
      const MprStage st = sh.mpr[lane];
      float fr[9] = {st.nrm[0], st.nrm[1], st.nrm[2], 0, 0, 0, 0, 0, 0};
      make_frame(fr);
      store_contact(sh, crec, tot + lane, fr, st.pos[0], st.pos[1], st.pos[2], st.pos[3], __float_as_int(st.nrm[3]));
    }
    for (int j0 = kMaxCon; j0 < wave_max_i(nmpr); j0 += kLanes) {   // rare: more than kMaxCon convex contacts
      const int j = j0 + lane;
      if (j < nmpr && crec) {
        const float4* stg = reinterpret_cast<const float4*>(crec + (size_t)j * kConStride + kMprStageOff);
        const float4 sp = stg[0], sn = stg[1];
        float fr[9] = {sn.x, sn.y, sn.z, 0, 0, 0, 0, 0, 0};
        make_frame(fr);
        store_contact(sh, crec, tot + j, fr, sp.x, sp.y, sp.z, sp.w, __float_as_int(sn.w));
      }
    }
    tot += nmpr;
    __syncthreads();
    tot = pad_contacts<kFused>(m, w, sh, crec, lane, grp, valid, tot);
    // every contact is kept (kConCap is the list's maximum), so none is dropped: 0 is written as the counter
    if (lane == 0) sh.ncon = tot;
  }
  __syncthreads();
}
// One substep's position/velocity stages and constraint assembly on the state in registers (after the
// previous substep's Euler): kinematics, CRBA/RNE, actuation, collision, the frictionloss / limit /
// contact rows.  Newton: the rows go to nr (kFused: kept in registers for newton_solve; split: stored to the
// HBM record); PGS: the solver record of so100_pgs_kernel.
template <int kSolver, bool kFused, bool kDebug = true>
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
    dynamics_par(m, sh, lane, mscale DSTAMP_ARGS);
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
    // (the convex pairs first: the other collision results are then not held across their narrowphase's register
    // peak; the contacts are compacted in pair order below whatever the order of computation)
    // the env's contact record in HBM, for the contacts beyond the kMaxCon held on chip: the split path's per-env
    // record (also its solver record); the fused path's pool record, taken only by an env whose list is longer
    float* crec = kFused ? nullptr : args.w.con + (size_t)e * kConEnv;
    float* const recbase = kFused ? args.w.pool : args.w.con + (size_t)(env - grp) * kConEnv;
    float4* const sep = args.w.sep + (size_t)(env - grp) * kSepPairs;
    collide<kFused>(m, args.w, recbase, sep, sh, lane, grp, valid, crec SSTAMP_PASS);
    // the env's record from here on, recomputed at each use (the contacts beyond kMaxCon are rare): not a pointer held
    // across the rows and the solve (the 3-wave build spilled it)
    auto recp = [&]() -> float* {
      return kFused ? pool_rec(args.w, (&sh - grp)->rec, grp) : args.w.con + (size_t)e * kConEnv;
    };
    if constexpr (!kFused) {
      if (valid && lane == 0 && B.ncon_dropped && sub == 0) B.ncon_dropped[env] = 0u;
    } else {
      // (the pool's safety valve, never reached in a measured run) no record came free: the first kMaxCon contacts
      if (valid && lane == 0 && sh.ncon > kMaxCon && (&sh - grp)->rec < 0) {
        sh.ndrop += sh.ncon - kMaxCon;
        sh.ncon = launder_v(kMaxCon);     // (a constant materialised here: not one held from the kernel entry)
      }
      __syncthreads();
    }
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

    // ---------------- S4/S5: M^-1 rows, frictionloss and joint-limit rows (lane = dof)
    float minv_row[6];
#pragma unroll
    for (int j = 0; j < 6; j++) minv_row[j] = (lane < 6) ? sh.minv[lane][j] : 0.f;
    const float invmc = (lane >= 6 && lane < 12) ? sh.inv_mcube[lane - 6] : 0.f;
    const float qs_r = (lane < SO100_NV) ? sh.qacc_smooth[lane] : 0.f;
    const bool has_fr = lane < SO100_NV;
    const float fr_R = has_fr ? m->fr_R[lane] : 1.f;
    const float fr_fl = has_fr ? m->fr_floss[lane] : 0.f;
    // the velocity from its LDS copy (S1, bitwise qvel_r): qvel_r need not stay live across collision
    const float qv_r = lane < SO100_NV ? sh.qvel[lane] : 0.f;
    const float fr_aref = -m->fr_B * qv_r;
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
      // the joint position from its LDS copy (S1, bitwise qpos_r): qpos_r need not stay live across collision
      const float q = sh.qpos[lane];
      const float dlo = q - m->jnt_lo[lane], dhi = m->jnt_hi[lane] - q;
      float dist = 0.f;
      if (dlo < 0.f) { lim_on = true; lim_s = 1.f; dist = dlo; }
      else if (dhi < 0.f) { lim_on = true; lim_s = -1.f; dist = dhi; }
      if (lim_on) {
        const float imp = getimpedance(m->lim_solimp, dist, 0.f);
        lim_R = fmaxf(kMinVal, (1.f - imp) * __builtin_amdgcn_rcpf(imp) * m->lim_invw[lane]);
        lim_aref = -m->lim_B * (lim_s * qv_r) - m->lim_K * imp * dist;
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
            if constexpr (!kFused) reinterpret_cast<float4*>(recp() + c * kConStride + kJOff)[lane] = J;
          }
          if constexpr (kFused) {
            if (c < kJReg) nr.J[c] = J;
            else jhi[c - kJReg] = J;
          }
          const bool mine = lane == c;
          const float v0 = rowsum16(J.x * qv_r), v1 = rowsum16(J.y * qv_r);
          const float v2 = rowsum16(J.z * qv_r), v3 = rowsum16(J.w * qv_r);
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
      if (lane < ncon) newton_contact_rows(m, sh.con_pair[lane], sh.con_dist[lane], cVn, fscale, nr.c_aref, nr.c_R, nr.c_mu);
      if (ncon_max > kMaxCon) {
        // the contacts beyond kMaxCon (rare): J and their aref / R / cone coefficients to the env's HBM record,
        // block by block of 16 (lane k: contact kMaxCon + 16 b + k), for both paths' newton_solve
        for (int b0 = kMaxCon; b0 < ncon_max; b0 += kLanes) {
          float cv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
          for (int k = 0; k < kLanes && b0 + k < ncon_max; k++) {
            const int c = b0 + k;
            float4 J = make_float4(0.f, 0.f, 0.f, 0.f);
            if (c < ncon && lane < SO100_NV) {
              J = contact_jac_ovf(m, sh, recp(), c, lane);
              reinterpret_cast<float4*>(recp() + (size_t)c * kConStride + kJOff)[lane] = J;
            }
            const float v0 = rowsum16(J.x * qv_r), v1 = rowsum16(J.y * qv_r);
            const float v2 = rowsum16(J.z * qv_r), v3 = rowsum16(J.w * qv_r);
            if (lane == k) { cv[0] = v0; cv[1] = v1; cv[2] = v2; cv[3] = v3; }
          }
          const int c = b0 + lane;
          if (c < ncon) {
            float4* sl = reinterpret_cast<float4*>(recp() + (size_t)c * kConStride);
            const float* g = recp() + (size_t)c * kConStride;
            float4 aref4, R4, mu4;
            newton_contact_rows(m, __float_as_int(g[kGeoPair]), g[kGeoDist], cv, fscale, aref4, R4, mu4);
            // the solve's per-contact constants, as newton_solve derives them for the resident contacts (D = 1 / R,
            // the middle zone's Dm), once here instead of at each of its reads (so100_newton.h ovf_load)
            const float4 D4 = make_float4(1.f / R4.x, 1.f / R4.y, 1.f / R4.z, 1.f / R4.w);
            mu4.w = D4.x / (mu4.x * mu4.x * (1.f + mu4.x * mu4.x));
            sl[0] = aref4;
            sl[1] = D4;
            sl[2] = mu4;
          }
        }
        __syncthreads();          // the record's J rows are read by the other lanes of the row in the solve
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
          // the contact counter (so100_contact_count) reads the last substep's count: the fused workspace's header is
          // one float per env (a 4-B store per env step, where the strided record header dirtied a whole line each)
          if (lane == 0 && sub == m->nsubstep - 1) args.w.hdr[e] = __int_as_float(ncon);
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
          reinterpret_cast<float4*>(recp() + c * kConStride + kJOff)[lane] = J;
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
          const float v = rowsum16(jv[r] * qv_r), ac = rowsum16(jv[r] * qs_r), w = rowsum16(jv[r] * warm_r);
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
    if (lane < ncon)
      pgs_contact_block(m, sh.con_pair[lane], sh.con_dist[lane], fscale, cA, cV, cAc, cW,
                        reinterpret_cast<float4*>(recp() + lane * kConStride), cf, cost_part);
    SSTAMP(4);
    // J' f of the warmstart forces: contact c's forces broadcast from lane c
#pragma unroll
    for (int c = 0; c < kMaxCon; c++) {
      if (c < ncon_max) {
        const float4 fc = bcast_row4(make_float4(cf[0], cf[1], cf[2], cf[3]), c);
        phi += Jr[c].x * fc.x + Jr[c].y * fc.y + Jr[c].z * fc.z + Jr[c].w * fc.w;
      }
    }
    if (ncon_max > kMaxCon) {
      // the contacts beyond kMaxCon (rare), block by block of 16 (lane k: contact kMaxCon + 16 b + k): J (-> the
      // record), the row reductions, the contact's block (-> the record) and warmstart force, J' f (J read back)
      for (int b0 = kMaxCon; b0 < ncon_max; b0 += kLanes) {
        float oA[10], oV[4], oAc[4], oW[4];
#pragma unroll
        for (int k = 0; k < 10; k++) oA[k] = 0.f;
#pragma unroll
        for (int r = 0; r < 4; r++) oV[r] = oAc[r] = oW[r] = 0.f;
#pragma unroll 1
        for (int k = 0; k < kLanes && b0 + k < ncon_max; k++) {
          const int c = b0 + k;
          float4 J = make_float4(0.f, 0.f, 0.f, 0.f);
          if (c < ncon && lane < SO100_NV) {
            J = contact_jac_ovf(m, sh, recp(), c, lane);
            reinterpret_cast<float4*>(recp() + (size_t)c * kConStride + kJOff)[lane] = J;
          }
          const float4 M = minv_times(J, minv_row, invmc, lane);
          const float jv[4] = {J.x, J.y, J.z, J.w}, mv[4] = {M.x, M.y, M.z, M.w};
          const bool mine = lane == k;
          int q2 = 0;
#pragma unroll
          for (int r = 0; r < 4; r++) {
#pragma unroll
            for (int q = r; q < 4; q++, q2++) {
              const float a = rowsum16(jv[r] * mv[q]);
              oA[q2] = mine ? a : oA[q2];
            }
            const float v = rowsum16(jv[r] * qv_r), ac = rowsum16(jv[r] * qs_r), w = rowsum16(jv[r] * warm_r);
            oV[r] = mine ? v : oV[r];
            oAc[r] = mine ? ac : oAc[r];
            oW[r] = mine ? w : oW[r];
          }
        }
        float of[4] = {0.f, 0.f, 0.f, 0.f};
        const int c = b0 + lane;
        if (c < ncon) {
          float4* cs = reinterpret_cast<float4*>(recp() + (size_t)c * kConStride);
          const float* g = recp() + (size_t)c * kConStride;
          pgs_contact_block(m, __float_as_int(g[kGeoPair]), g[kGeoDist], fscale, oA, oV, oAc, oW, cs, of, cost_part);
          cs[kBlkF] = make_float4(of[0], of[1], of[2], of[3]);     // zeroed below if the warmstart is dropped
        }
#pragma unroll 1
        for (int k = 0; k < kLanes && b0 + k < ncon_max; k++) {
          const float4 fk = shfl_row4(make_float4(of[0], of[1], of[2], of[3]), k);
          const float4 J = ovf_j(recp(), b0 + k, lane, ncon);
          phi += J.x * fk.x + J.y * fk.y + J.z * fk.z + J.w * fk.w;
        }
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
    if (lane < ncon) reinterpret_cast<float4*>(recp() + lane * kConStride)[kBlkF] = make_float4(cf[0], cf[1], cf[2], cf[3]);
    if (ncon_max > kMaxCon && cost > 0.f) {
      for (int c = kMaxCon + lane; c < ncon; c += kLanes)
        reinterpret_cast<float4*>(recp() + (size_t)c * kConStride)[kBlkF] = make_float4(0.f, 0.f, 0.f, 0.f);
    }

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
      // (without auto-reset an env left truncated keeps reporting truncated: its episode is counted once, at
      // the step that reached the limit; stepping a terminated env without a reset is outside the contract)
      const bool ended_before = args.max_steps > 0 && elapsed0 >= args.max_steps;
      if (B.ep_return && !ended_before) {
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
__global__ void __launch_bounds__(kThreads, kStageWaves) so100_stage_kernel(StageArgs args) {
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
// The whole env step in one launch (Newton solver, the default): each wave runs its 4 envs through the 10
// substeps — Euler, assembly, the Newton solve with the rows handed over in registers (no HBM record) —
// and the epilogue, with the state in registers throughout.  The split path's 21 launches end every
// substep at the slowest wave of the chip; here a wave only waits for itself.
// Results are those of the split path (so100_stage_kernel + so100_newton_kernel): the same device
// functions on the same values.  kDebug: the instantiation that also fills the debug buffer (launched when
// the caller passes one); the other has no debug code, which costs registers in the substep loop.
// kWaves: the waves per SIMD the register budget is sized for.  3 (168 VGPRs; 8 B/lane of scratch since round 6's
// quadratic-exact Newton stop: two floats of the arm's M row, reloaded twice per Newton step) when the
// grid exceeds 2 waves per SIMD; a grid of at most 2 waves per SIMD (8,192 envs on 256 CUs: all waves resident at
// once) takes the 2-wave build (its own translation unit, so100_fused2.hip, under LLVM's iterative-ILP scheduler:
// 249-256 VGPRs, no scratch).  Register allocation only: both give the same results bit for bit.
template <bool kDebug, int kWaves = 3>
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
  if (args.w.order) {   // the heavier half of the waves, by launch rank, issue first on their SIMD
    const unsigned rank = blockIdx.x, ng = gridDim.x;
    if (rank < ng / 8) __builtin_amdgcn_s_setprio(3);
    else if (rank < ng / 4) __builtin_amdgcn_s_setprio(2);
    else if (rank < ng / 2) __builtin_amdgcn_s_setprio(1);
  }
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
  if (lane == 0) {
    // shm[0].rec: the wave's pool entry (-1: none held); shm[1].rec / shm[2].rec: the entries it took and the requests
    // that found none free over the step (added to Workspace::pool_stat in the epilogue)
    sh.rec = grp == 0 ? -1 : 0;
    sh.ndrop = 0;                 // contacts left out over the step (0: the pool is sized never to run out)
  }
  const int nsub = args.m->nsubstep;
  const float h = args.m->timestep;
  for (int sub = 0; sub < nsub; sub++) {
    // the lane / env ids laundered per substep too: what derives from them (masks, addresses, per-lane
    // model values) is recomputed in each substep instead of hoisted and held live across the loop
    // recomputed from the wave's lane id (an opaque v_mbcnt pair, which LICM cannot hoist) and the
    // workgroup's scalar group index: no vector value of the ids is carried across the loop
    int lane, grp, env, e;
    fresh_ids(group, args.n, lane, grp, env, e);
    const bool valid = env < args.n;
    EnvShared& sh = shm[grp];
    TL_MARK(-1);
    if (sub > 0) euler_update(sh, lane, h, warm_r, qpos_r, qvel_r);
    // the model pointer laundered per substep: the model loads (uniform, ~1 KB) must not be hoisted out of
    // the substep loop, where they would stay live across it (register spills)
    StageArgs sa = args;
    {
      int zero;
      asm volatile("s_mov_b32 %0, 0" : "=s"(zero));
      sa.m = reinterpret_cast<const DevModel*>(reinterpret_cast<const char*>(args.m) + zero);
    }
    // the DR scales re-read per substep (from L2: 8 B per env), not carried across the loop in registers (the 3-wave
    // build spilled them at kernel entry: a scratch store per lane and launch)
    float mscale_s = 1.f, fscale_s = 1.f;
    if ((args.flags & SO100_FLAG_DR) && args.b.dr_params) {
      mscale_s = args.b.dr_params[(size_t)e * 4 + 0];
      fscale_s = args.b.dr_params[(size_t)e * 4 + 1];
    }
    NewtonRows nr;
    assemble<SO100_SOLVER_NEWTON, true, kDebug>(sa, sh, lane, grp, env, e, valid, qpos_r, qvel_r, warm_r, mscale_s,
                                                fscale_s, sub, nr);
    // the position and velocity state back from their LDS copies (assemble's S1 stores, untouched since): bitwise
    // the same values, and the registers are not held across collision's register peak (they were spilled there)
    qpos_r = lane < SO100_NQ ? sh.qpos[lane] : 0.f;
    qvel_r = lane < SO100_NV ? sh.qvel[lane] : 0.f;
    TL_MARK(0);
    NewtonDiag diag;
    const bool dbg = kDebug && args.b.debug && sub == nsub - 1;
    // the env's HBM contact record, for its contacts beyond kMaxCon (rare): its address recomputed from fresh ids
    // where needed, not held across the solve
    auto rec = [&]() -> float* {
      int l2, g2, en2, e2;
      fresh_ids(group, args.n, l2, g2, en2, e2);
      return pool_rec(args.w, shm[0].rec, g2);
    };
    const float qacc = newton_solve_any(sa.m, nr, lane, valid, dbg, diag, rec);
    if (dbg) {
      int row = env;
      asm volatile("" : "+v"(row));        // not the assembly's row address (GVN would hold that across the solve)
      newton_diag_write(args.b.debug + (size_t)row * SO100_DBG_STRIDE, lane, valid, qacc, diag);
      if (valid) newton_diag_write_ovf(args.b.debug + (size_t)row * SO100_DBG_STRIDE, rec(), nr.ncon, lane);
    }
    warm_r = lane < SO100_NV ? qacc : 0.f;
    {
      // the env's pool record back (its substep is done with it)
      int l2, g2, en2, e2;
      fresh_ids(group, args.n, l2, g2, en2, e2);
      if (l2 == 0 && g2 == 0) {
        const int ent = shm[0].rec;
        if (ent >= 0) pool_release(args.w, ent);
        if (ent != -1) shm[ent >= 0 ? 1 : 2].rec++;
        shm[0].rec = -1;                  // (also after a failed request's -2: the next substep asks again)
      }
    }
    TL_MARK(1);
  }
  TL_MARK(-1);
  {
    // fresh ids again: the epilogue's store addresses must not be the prologue's load addresses (CSE would
    // hold those across the substep loop)
    int lane, grp, env, e;
    fresh_ids(group, args.n, lane, grp, env, e);
    const bool valid = env < args.n;
    EnvShared& sh = shm[grp];
    euler_update(sh, lane, h, warm_r, qpos_r, qvel_r);
    // the step counters re-read (the kernel writes them only below, so they are the prologue's values): not held in
    // registers across the substep loop (the 3-wave build spilled them)
    int el0 = args.b.elapsed ? args.b.elapsed[e] : 0;
    uint32_t ep0 = args.b.episode ? args.b.episode[e] : 0u;
    final_stage(args, sh, lane, grp, env, e, valid, qpos_r, qvel_r, warm_r, el0, ep0);
    if (valid && lane == 0 && args.b.ncon_dropped) args.b.ncon_dropped[env] = (uint32_t)sh.ndrop;
    if (args.w.gcost && lane == 0 && grp == 0) args.w.gcost[group] = (uint32_t)(__builtin_amdgcn_s_memtime() - cost_t0);
    if (lane == 0 && grp == 0 && args.w.pool_stat) {
      const int took = shm[1].rec, none = shm[2].rec;
      if (took) __hip_atomic_fetch_add(args.w.pool_stat, (unsigned long long)took, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (none) __hip_atomic_fetch_add(args.w.pool_stat + 1, (unsigned long long)none, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  TL_MARK(2);
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

// The 2-wave product build of the fused kernel lives in its own translation unit (so100_fused2.hip, which includes this
// file with SO100_FUSED2_TU: only the device code above and launch_fused2 below), compiled with LLVM's iterative-ILP
// scheduler (Makefile): +3.8 % at 8,192 envs, same box (profiles/r05_ab_sched_8192.txt); the 3-wave build spills under
// that scheduler (220 B/lane), so it and everything else stay on the default one.
#ifndef SO100_FUSED2_TU
hipError_t launch_fused2(const DevModel* m, const StageArgs& a, dim3 grid, hipStream_t s);

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

// Heavy-first wave order for the fused kernel, per XCD.  Its waves run a whole env step each (0.4-1.8 ms) and the
// grid exceeds the resident slots (12 per CU) above 12,288 envs: a long wave dispatched late sets the step's
// tail.  Wave costs persist from step to step (correlation 0.65-0.74, measured), so the groups are launched
// in descending order of their previous step's cost.  Workgroups go to the XCDs round-robin (block b to XCD b % 8), so
// XCD x runs the blocks b = 8 r + x: they take the groups of one contiguous range (range x, as many groups as XCD x has
// blocks), its r-th costliest as block 8 r + x.  Neighbouring groups then write their shared cache lines of the state
// arrays (an env's qpos is 52 B, its reward 4 B: a 64-B line spans 1-16 envs) through one L2, which merges them before
// write-back, instead of one partial line per XCD (round 4's global order scattered neighbours over the 8 L2s).
// A counting sort on a 9-bit cost key (5 exponent bits from 2^1 up, 4 mantissa bits, 6 % buckets), one workgroup per
// range.  The order changes the schedule, never a result.
constexpr int kOrderXcd = 8;
constexpr int kOrderKeys = 512;
constexpr int kOrderMinGroups = 256;           // the order also sets the waves' issue priority
// blocks of XCD x (b % 8 == x) of a grid of ng blocks; range x starts at the sum of those of the XCDs before it
DEV int order_cnt(int ng, int x) { return (ng - x + kOrderXcd - 1) / kOrderXcd; }
__global__ void __launch_bounds__(1024) so100_order_kernel(const uint32_t* __restrict__ gcost, int ng,
                                                           int* __restrict__ order) {
  // one workgroup per XCD range (round 6: the 8 ranges sort independently, in parallel; one workgroup sorting all
  // of them took 15.6 us per step at 65,536 envs, 0.6 % of the step)
  __shared__ int hist[kOrderKeys];
  __shared__ int part[kOrderKeys];
  const int t = threadIdx.x, x = blockIdx.x;
  int start = 0;
  for (int y = 0; y < x; y++) start += order_cnt(ng, y);
  const int cnt = order_cnt(ng, x);
  auto key = [&](int g) {
    const uint32_t u = __float_as_uint((float)gcost[g]);
    const int ex = min(max((int)(u >> 23) - 128, 0), 31);
    return (kOrderKeys - 1) - ((ex << 4) | (int)((u >> 19) & 15u));
  };
  if (t < kOrderKeys) hist[t] = 0;
  __syncthreads();
  for (int i = t; i < cnt; i += 1024) atomicAdd(&hist[key(start + i)], 1);
  __syncthreads();
  const int own = t < kOrderKeys ? hist[t] : 0;
  if (t < kOrderKeys) part[t] = own;
  __syncthreads();
  for (int d = 1; d < kOrderKeys; d <<= 1) {     // inclusive scan of the bucket counts
    const int v = (t < kOrderKeys && t >= d) ? part[t - d] : 0;
    __syncthreads();
    if (t < kOrderKeys) part[t] += v;
    __syncthreads();
  }
  if (t < kOrderKeys) hist[t] = part[t] - own;   // the bucket's first rank
  __syncthreads();
  for (int i = t; i < cnt; i += 1024) {
    const int g = start + i;
    const int r = atomicAdd(&hist[key(g)], 1);   // rank in range x
    order[kOrderXcd * r + x] = g;
  }
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
      hipLaunchKernelGGL(so100_order_kernel, dim3(kOrderXcd), dim3(1024), 0, s, w.gcost, ng, w.order);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      if (ev) (void)hipEventRecord(ev[0], s);
    } else {
      a.w.order = nullptr;
    }
    const int build = fused_build(n, waves, b.debug != nullptr);
#ifndef SO100_RU_FUSED3_ONLY   // (Makefile ru3: only the 3-wave product build, for register-allocation work)
    if (build == 1) hipLaunchKernelGGL(so100_fused_kernel<true>, grid, dim3(kThreads), 0, s, m, a);
    else if (build == 2) (void)launch_fused2(m, a, grid, s);
    else
#endif
    hipLaunchKernelGGL((so100_fused_kernel<false, 3>), grid, dim3(kThreads), 0, s, m, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[k++], s);
    w.sub_count += (uint32_t)nsubstep;
    return hipSuccess;
  }
  for (int sub = 0; sub <= nsubstep; sub++) {
    a.sub = sub;
    a.par = (int)(w.sub_count & 1u);
#ifdef SO100_RU_FUSED3_ONLY
    if (false) {
#else
    if (solver == SO100_SOLVER_NEWTON) {
      if (sub == 0) hipLaunchKernelGGL((so100_stage_kernel<0, SO100_SOLVER_NEWTON>), grid, dim3(kThreads), 0, s, a);
      else if (sub < nsubstep) hipLaunchKernelGGL((so100_stage_kernel<1, SO100_SOLVER_NEWTON>), grid, dim3(kThreads), 0, s, a);
      else hipLaunchKernelGGL((so100_stage_kernel<2, SO100_SOLVER_NEWTON>), grid, dim3(kThreads), 0, s, a);
    } else {
      if (sub == 0) hipLaunchKernelGGL((so100_stage_kernel<0, SO100_SOLVER_PGS>), grid, dim3(kThreads), 0, s, a);
      else if (sub < nsubstep) hipLaunchKernelGGL((so100_stage_kernel<1, SO100_SOLVER_PGS>), grid, dim3(kThreads), 0, s, a);
      else hipLaunchKernelGGL((so100_stage_kernel<2, SO100_SOLVER_PGS>), grid, dim3(kThreads), 0, s, a);
#endif
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
// (hdr: the split path's record headers, stride kHdrEnv, or the fused path's compact counts, stride 1)
__global__ void so100_contact_count_kernel(const float* __restrict__ hdr, int n, int stride, unsigned long long* accum) {
  __shared__ int part[256];
  int s = 0;
  const int off = stride == 1 ? 0 : H_NCON;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    s += __float_as_int(hdr[(size_t)i * stride + off]);
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
__global__ void so100_contact_counts_kernel(const float* __restrict__ hdr, int n, int stride, int32_t* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = __float_as_int(hdr[(size_t)i * stride + (stride == 1 ? 0 : H_NCON)]);
}
hipError_t launch_contact_counts(const Workspace& w, int n, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(so100_contact_counts_kernel, dim3((n + 255) / 256), dim3(256), 0, s, w.hdr, n, w.hdr_stride, out);
  return hipGetLastError();
}
hipError_t launch_contact_count(const Workspace& w, int n, uint64_t* accum, hipStream_t s) {
  int blocks = (n + 255) / 256;
  if (blocks > 256) blocks = 256;
  hipLaunchKernelGGL(so100_contact_count_kernel, dim3(blocks), dim3(256), 0, s, w.hdr, n, w.hdr_stride,
                     reinterpret_cast<unsigned long long*>(accum));
  return hipGetLastError();
}

hipError_t free_workspace(Workspace* w);
hipError_t alloc_workspace(int n, Workspace* w) {
  *w = Workspace{};
  w->hdr_stride = kHdrEnv;
  hipError_t e = hipMalloc(&w->hdr, (size_t)n * kHdrEnv * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&w->con, (size_t)n * kConEnv * sizeof(float));
  // zero once: record slots a solver lane reads but never uses are then finite, never garbage
  if (e == hipSuccess) e = hipMemset(w->hdr, 0, (size_t)n * kHdrEnv * sizeof(float));
  if (e == hipSuccess) e = hipMemset(w->con, 0, (size_t)n * kConEnv * sizeof(float));
  const size_t ngroups = (size_t)(n + kPgsEnvs - 1) / kPgsEnvs;
  if (e == hipSuccess) e = hipMalloc(&w->gflag, 2 * ngroups * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&w->hcount, 2 * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&w->hlist, 2 * kHeavyCap * sizeof(int));
  if (e == hipSuccess) e = hipMemset(w->gflag, 0, 2 * ngroups * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(w->hcount, 0, 2 * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&w->sep, (size_t)n * kSepPairs * sizeof(float4));
  if (e == hipSuccess) e = hipMemset(w->sep, 0, (size_t)n * kSepPairs * sizeof(float4));
  if (e != hipSuccess) (void)free_workspace(w);
  return e;
}
hipError_t free_workspace(Workspace* w) {
  hipError_t r = hipSuccess;
  for (void* p : {(void*)w->hdr, (void*)w->con, (void*)w->gflag, (void*)w->hcount, (void*)w->hlist, (void*)w->gcost,
                  (void*)w->order, (void*)w->sep, (void*)w->pool, (void*)w->pool_bm, (void*)w->pool_stat}) {
    if (!p) continue;
    hipError_t e = hipFree(p);
    if (r == hipSuccess) r = e;
  }
  w->hdr = w->con = nullptr;
  w->gflag = w->gcost = nullptr;
  w->hcount = w->hlist = w->order = nullptr;
  w->sep = nullptr;
  w->pool = nullptr;
  w->pool_bm = nullptr;
  w->pool_stat = nullptr;
  return r;
}
// The fused path's workspace: the contact counts (one float per env), the wave-order buffers, the separating-direction
// cache, and the contact-record pool (Workspace::pool): per XCD one entry (a wave's 4 records of kConEnv floats, 288 KB
// each) per fused-kernel wave the XCD can hold resident at once — its CUs (the device's CUs / kPoolXcd) x the resident
// workgroups per CU of the fused instantiations (the occupancy API: 12, LDS-bound, for the 3-wave and debug builds;
// 8 for the 2-wave build), and no more than the grid's waves — so a wave that asks always finds a free entry
// (so100_pool.h).  3.5 GB at 6,144 envs and up (8 x 384 entries; 288 GB of HBM per GPU), for the waves holding an env
// whose list is longer than the kMaxCon held on chip (for one substep).
int fused_pool_recs(int n) {
  int dev = 0, cus = 256, occ3 = 0, occd = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ3, so100_fused_kernel<false, 3>, kThreads, 0) != hipSuccess) occ3 = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occd, so100_fused_kernel<true, 3>, kThreads, 0) != hipSuccess) occd = 0;
  (void)hipGetLastError();
  // 160 KB of LDS per CU over the kernels' static LDS caps every build (the 2-wave build at 8 by its registers)
  const int lds_cap = (160 * 1024) / (int)(sizeof(EnvShared) * kEnvsPerBlock);
  const int per_cu = std::max({occ3, occd, lds_cap});
  const int cus_per_xcd = (cus + kPoolXcd - 1) / kPoolXcd;
  const int waves = (n + kEnvsPerBlock - 1) / kEnvsPerBlock;
#ifdef SO100_POOL_R5   // (A/B switch: round 5's pool size, 8..32 entries per XCD by the env count)
  (void)cus_per_xcd; (void)per_cu; (void)waves;
  return std::min(32, std::max(8, (n + 256 * kPoolXcd - 1) / (256 * kPoolXcd)));
#else
  return std::max(1, std::min({kPoolSlots, cus_per_xcd * per_cu, waves}));
#endif
}
hipError_t alloc_fused_workspace(int n, Workspace* w) {
  *w = Workspace{};
  const size_t ng = (size_t)(n + kEnvsPerBlock - 1) / kEnvsPerBlock;
  w->hdr_stride = 1;                   // the contact counts only, one float per env
  hipError_t e = hipMalloc(&w->hdr, (size_t)n * sizeof(float));
  if (e == hipSuccess) e = hipMemset(w->hdr, 0, (size_t)n * sizeof(float));
  w->pool_recs = fused_pool_recs(n);
  if (e == hipSuccess) e = hipMalloc(&w->pool, (size_t)kPoolXcd * w->pool_recs * kEnvsPerBlock * kConEnv * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&w->pool_bm, (size_t)kPoolXcd * kPoolWords * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(w->pool_bm, 0, (size_t)kPoolXcd * kPoolWords * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&w->pool_stat, 2 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(w->pool_stat, 0, 2 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMalloc(&w->gcost, ng * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(w->gcost, 0, ng * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&w->order, ng * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&w->sep, (size_t)n * kSepPairs * sizeof(float4));
  if (e == hipSuccess) e = hipMemset(w->sep, 0, (size_t)n * kSepPairs * sizeof(float4));
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

#else   // SO100_FUSED2_TU
hipError_t launch_fused2(const DevModel* m, const StageArgs& a, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((so100_fused_kernel<false, 2>), grid, dim3(kThreads), 0, s, m, a);
  return hipGetLastError();
}
#endif  // SO100_FUSED2_TU

}  // namespace so100
