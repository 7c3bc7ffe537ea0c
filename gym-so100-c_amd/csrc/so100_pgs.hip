// so100_pgs.hip — the constraint solve of one substep: projected Gauss-Seidel, MuJoCo mj_solPGS
// semantics (engine_solver.c: frictionloss rows, joint limits, then elliptic condim-4 contacts with the
// mju_QCQP3 friction update; improvement-based early exit), on the record the stage kernel wrote.
//
// Layout: 4 lanes per env, lane q owns dofs 3q..3q+2 (q = 0,1 arm, 2,3 cube), 16 envs
// per wave64.  Every J·qacc row product is 3 FMAs + a 2-step quad DPP reduction; the per-contact scalar
// work (residual, normal projection, QCQP) runs once per 4 lanes instead of once per 16, which is what
// bounds this phase: it is issue-bound on per-env serial work, not on memory.
//   * arm M^-1 is dense 6x6: lane q holds its 3 rows (own 3 columns, partner-lane 3 columns), the
//     partner's 3 dof values arrive by one quad_perm swap;
//   * the arm and cube trees are decoupled (M block-diagonal, cube M diagonal: COM at the free-joint
//     origin, principal axes = body axes), so arm frictionloss row j and cube row 6+j update together;
//   * the first kResident contacts keep J in VGPRs and the solver block in LDS (10 KB per wave) for all
//     sweeps; further contacts (rare: >4 per env; the list holds up to kConCap) stream both from the HBM
//     record every sweep, loaded at use so the register peak stays at 168 (3 waves/SIMD), forces written
//     back to the record.
#include "so100_common.h"
#include "so100.h"

namespace so100 {

constexpr int kPgsWaves = 2;         // waves per SIMD the register budget is sized for: 2 (176 VGPRs, no scratch; round 5)
                                     // beat 3 (168, 52 B/lane of spill slots in the overflow path) by 2 %, and with the
                                     // memory-clause scheduler (Makefile) by 2.5 % (profiles/r05_ab_pgs_sched.txt)

struct PgsArgs {
  const DevModel* m;
  Workspace w;
  float* qacc_out;               // so100_buffers.qacc_warmstart: the solver's qacc (next warmstart)
  float* debug;
  int n;
  int last;                      // last substep of the env step: write the debug record
  int par;                       // substep parity (heavy-group list set)
  int nheavy_slots;              // leading blocks reserved for heavy groups
};

// One contact block (elliptic cone, condim 4) of a sweep: normal row by projection, then the friction
// rows by the QCQP on the cone scaled by the new normal force (mj_solPGS elliptic branch); qacc +=
// M^-1 J' (f_new - f_old).  Straight-line apart from the QCQP's Newton loop: every lane evaluates the
// block and `active` selects the result, so the block's LDS reads issue together at the top instead of
// being sunk into branches (three serialised LDS round trips per contact otherwise).
DEV void contact_update(const float4 (&v)[kBlk], const float4 (&J)[3], float (&qacc)[3], const float (&mrow)[3][6],
                        bool active, bool lead, bool arm, float& impr, float4& fout, int& newton) {
  const float j0 = quadsum(J[0].x * qacc[0] + J[1].x * qacc[1] + J[2].x * qacc[2]);
  const float j1 = quadsum(J[0].y * qacc[0] + J[1].y * qacc[1] + J[2].y * qacc[2]);
  const float j2 = quadsum(J[0].z * qacc[0] + J[1].z * qacc[1] + J[2].z * qacc[2]);
  const float j3 = quadsum(J[0].w * qacc[0] + J[1].w * qacc[1] + J[2].w * qacc[2]);
  // unpack (solver block layout: so100_device.h)
  const float a00 = v[0].x, a01 = v[0].y, a02 = v[0].z, a03 = v[0].w, a11 = v[1].x, a12 = v[1].y, a13 = v[1].z;
  const float a22 = v[1].w, a23 = v[2].x, a33 = v[2].y;
  const float P[9] = {v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w, v[4].x, v[4].y, v[4].z};
  const float lam[3] = {v[4].w, v[5].x, v[5].y};
  const float laminv[3] = {v[5].z, v[5].w, v[6].x};
  const float R0 = v[6].y, arinv0 = v[6].z, R1 = v[6].w, R3 = v[7].x;
  const float4 ar = v[kBlkAref], f4 = v[kBlkF];
  const float res[4] = {j0 - ar.x + R0 * f4.x, j1 - ar.y + R1 * f4.y, j2 - ar.z + R1 * f4.z, j3 - ar.w + R3 * f4.w};
  const float old[4] = {f4.x, f4.y, f4.z, f4.w};
  float f[4];
  f[0] = old[0] - res[0] * arinv0;
  const bool open = !(f[0] < kMinVal);           // contact separates: all four forces 0
  {
    const float dn = f[0] - old[0];
    float bf[3];
    bf[0] = res[1] + a01 * dn - (a11 * old[1] + a12 * old[2] + a13 * old[3]);
    bf[1] = res[2] + a02 * dn - (a12 * old[1] + a22 * old[2] + a23 * old[3]);
    bf[2] = res[3] + a03 * dn - (a13 * old[1] + a23 * old[2] + a33 * old[3]);
    float x[3];
    newton += qcqp3_eig(x, P, lam, laminv, bf, f[0], active && open);
    f[1] = open ? x[0] : 0.f;
    f[2] = open ? x[1] : 0.f;
    f[3] = open ? x[2] : 0.f;
    f[0] = open ? f[0] : 0.f;
  }
  float dl[4];
#pragma unroll
  for (int r = 0; r < 4; r++) dl[r] = active ? f[r] - old[r] : 0.f;
  const float q0 = a00 * dl[0] + a01 * dl[1] + a02 * dl[2] + a03 * dl[3];
  const float q1 = a01 * dl[0] + a11 * dl[1] + a12 * dl[2] + a13 * dl[3];
  const float q2 = a02 * dl[0] + a12 * dl[1] + a22 * dl[2] + a23 * dl[3];
  const float q3 = a03 * dl[0] + a13 * dl[1] + a23 * dl[2] + a33 * dl[3];
  const float ci = dl[0] * (res[0] + 0.5f * q0) + dl[1] * (res[1] + 0.5f * q1) + dl[2] * (res[2] + 0.5f * q2) +
                   dl[3] * (res[3] + 0.5f * q3);
  impr -= (lead && active) ? ci : 0.f;            // one lane per env carries the contact's improvement
  fout = active ? make_float4(f[0], f[1], f[2], f[3]) : f4;
  // qacc += M^-1 J' d: g = J_dof . d per lane, the partner lane's 3 values by a quad swap
  float g[3], gp[3];
#pragma unroll
  for (int i = 0; i < 3; i++) g[i] = (J[i].x * dl[0] + J[i].y * dl[1]) + (J[i].z * dl[2] + J[i].w * dl[3]);
  if (!arm) {
    // cube-only contact (table / bin): J has no arm entries, the arm lanes' g is 0 and the cube block
    // of M^-1 is diagonal: the full update below reduces to this exactly
#pragma unroll
    for (int i = 0; i < 3; i++) qacc[i] += mrow[i][i] * g[i];
    return;
  }
#pragma unroll
  for (int i = 0; i < 3; i++) gp[i] = quad_swap1(g[i]);
#pragma unroll
  for (int i = 0; i < 3; i++)
    qacc[i] += (mrow[i][0] * g[0] + mrow[i][1] * g[1] + mrow[i][2] * g[2]) +
               (mrow[i][3] * gp[0] + mrow[i][4] * gp[1] + mrow[i][5] * gp[2]);

}

__global__ void __launch_bounds__(64, kPgsWaves) so100_pgs_kernel(PgsArgs a) {
  __shared__ float4 blk[kResident][kPgsEnvs][kBlk];
  const DevModel* __restrict__ m = a.m;
  const int tid = threadIdx.x;
  const int q = tid & 3;
  const int ew = tid >> 2;
  // groups holding an env with many contacts take longest: they run in the leading blocks so their
  // tail overlaps the bulk; the in-place block of a listed group exits
  const int ngroups = (a.n + kPgsEnvs - 1) / kPgsEnvs;
  int grp;
  if ((int)blockIdx.x < a.nheavy_slots) {
    const int cnt = min(a.w.hcount[a.par], kHeavyCap);
    if ((int)blockIdx.x >= cnt) return;
    grp = a.w.hlist[a.par * kHeavyCap + blockIdx.x];
  } else {
    grp = blockIdx.x - a.nheavy_slots;
    if (tid == 0) {
      a.w.gflag[(a.par ^ 1) * ngroups + grp] = 0u;      // reset the set the next stage kernel fills
      if (grp == 0) a.w.hcount[a.par ^ 1] = 0;
    }
    if (a.w.gflag[a.par * ngroups + grp] == 1u) return;
  }
  const int env = grp * kPgsEnvs + ew;
  const bool valid = env < a.n;
  const int e = valid ? env : 0;
  STAMP_DECL
  STAMP(-1);
#ifdef SO100_TIMELINE
  uint64_t tl_start;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tl_start)::"memory");
#endif

  // ---------------- record -> registers (10 x dwordx4 per lane)
  float hv[kHdrLane];
  {
    const float4* hp = reinterpret_cast<const float4*>(a.w.hdr + (size_t)e * kHdrEnv + q * kHdrLane);
#pragma unroll
    for (int k = 0; k < kHdrLane / 4; k++) {
      const float4 t = hp[k];
      hv[4 * k] = t.x; hv[4 * k + 1] = t.y; hv[4 * k + 2] = t.z; hv[4 * k + 3] = t.w;
    }
  }
  float qacc[3], fr_f[3], fr_aref[3], fr_R[3], fr_fl[3], fr_ARinv[3];
  float lim_f[3], mrow[3][6];
  bool lim_on[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
#pragma unroll
    for (int j = 0; j < 6; j++) mrow[i][j] = hv[H_MROW + 6 * i + j];
    const int d = 3 * q + i;
    qacc[i] = hv[H_QACC + i];
    fr_aref[i] = hv[H_FRAREF + i];
    fr_f[i] = hv[H_FRF + i];
    fr_R[i] = m->fr_R[d];
    fr_fl[i] = m->fr_floss[d];
    fr_ARinv[i] = 1.f / (mrow[i][i] + fr_R[i]);
    lim_on[i] = hv[H_LIMS + i] != 0.f;
    lim_f[i] = hv[H_LIMF + i];
  }
  const int ncon = valid ? __float_as_int(hv[H_NCON]) : 0;
  int ncon_max = ncon;
  ncon_max = max(ncon_max, __shfl_xor(ncon_max, 4));
  ncon_max = max(ncon_max, __shfl_xor(ncon_max, 8));
  ncon_max = max(ncon_max, __shfl_xor(ncon_max, 16));
  ncon_max = max(ncon_max, __shfl_xor(ncon_max, 32));
  ncon_max = __builtin_amdgcn_readfirstlane(ncon_max);
  // joint-limit rows present anywhere in the wave, per hinge (bit j: arm row j)
  uint32_t lim_rows = 0;
#pragma unroll
  for (int j = 0; j < 6; j++)
    lim_rows |= (__ballot(valid && q == j / 3 && lim_on[j % 3]) != 0ull) ? (1u << j) : 0u;
  const float* const lrec = a.w.hdr + (size_t)e * kHdrEnv + q * kHdrLane;   // limit rows: re-read when present
  const int iterations = m->iterations;
  const float tolerance = m->tolerance, pgs_scale = m->pgs_scale;

  // every env owns kMaxCon record slots: loads of slots >= ncon are in bounds but stale (or never
  // written); J of such slots is zeroed so that masked lanes contribute exactly 0 to g = J d
  float* const crec = a.w.con + (size_t)e * kConEnv;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 J[kResident][3];
#pragma unroll
  for (int c = 0; c < kResident; c++) {
    const float4* rec = reinterpret_cast<const float4*>(crec + c * kConStride);
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const float4 t = rec[kBlk + 3 * q + i];
      J[c][i] = c < ncon ? t : zero4;
    }
    blk[c][ew][q] = rec[q];
    blk[c][ew][q + 4] = rec[q + 4];
    if (q < 2) blk[c][ew][q + 8] = rec[q + 8];
  }
  __syncthreads();
  // resident contact slots in which some env of the wave has a gripper contact (J with arm entries)
  uint32_t arm_res = 0;
#pragma unroll
  for (int c = 0; c < kResident; c++)
    arm_res |= (__ballot(valid && c < ncon && blk[c][ew][kBlkFlags].y != 0.f) != 0ull) ? (1u << c) : 0u;
  __syncthreads();

  STAMP(0);
  // ---------------- sweeps
  bool done = !valid;
  int iters = 0, newton = 0;
  float last_impr = 0.f;
  for (int it = 0; it < iterations; it++) {
    if (__ballot(!done) == 0ull) break;
    // keep the per-contact LDS loads inside the sweep (no LICM of the blocks into VGPRs)
    asm volatile("" ::: "memory");
    float impr = 0.f;
    // frictionloss rows: arm row j (lane j/3) with cube row 6+j (lane 2 + j/3) — decoupled trees
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const int k = j % 3;
      const bool own = ((q & 1) == j / 3) && !done;
      const float res = qacc[k] - fr_aref[k] + fr_R[k] * fr_f[k];
      const float fn = fminf(fmaxf(fr_f[k] - res * fr_ARinv[k], -fr_fl[k]), fr_fl[k]);
      const float dlt = own ? fn - fr_f[k] : 0.f;
      fr_f[k] += dlt;
      impr -= dlt * (res + 0.5f * (mrow[k][k] + fr_R[k]) * dlt);
      const float dp = quad_swap1(dlt);
#pragma unroll
      for (int i = 0; i < 3; i++) qacc[i] += mrow[i][k] * dlt + mrow[i][3 + k] * dp;
    }
    // joint-limit rows (hinge order)
    if (lim_rows) {
#pragma unroll
      for (int j = 0; j < 6; j++) {
        if (!((lim_rows >> j) & 1u)) continue;
        const int k = j % 3;
        const float lim_s = lrec[H_LIMS + k], lim_aref = lrec[H_LIMAREF + k], lim_R = lrec[H_LIMR + k];
        const float lim_AR = mrow[k][k] + lim_R;
        const bool own = (q == j / 3) && lim_on[k] && !done;
        const float res = lim_s * qacc[k] - lim_aref + lim_R * lim_f[k];
        const float fn = fmaxf(lim_f[k] - res * __builtin_amdgcn_rcpf(lim_AR), 0.f);
        float dlt = own ? fn - lim_f[k] : 0.f;
        lim_f[k] += dlt;
        impr -= dlt * (res + 0.5f * lim_AR * dlt);
        dlt *= lim_s;
        const float dp = quad_swap1(dlt);
#pragma unroll
        for (int i = 0; i < 3; i++) qacc[i] += mrow[i][k] * dlt + mrow[i][3 + k] * dp;
      }
    }
    STAMP(1);
    // contact blocks, on-chip
#pragma unroll
    for (int c = 0; c < kResident; c++) {
      if (c < ncon_max) {
        float4 v[kBlk];
#pragma unroll
        for (int k = 0; k < kBlk; k++) v[k] = blk[c][ew][k];
        float4 fn;
        const bool act = c < ncon && !done;
        contact_update(v, J[c], qacc, mrow, act, q == 0, (arm_res >> c) & 1u, impr, fn, newton);
        if (act) blk[c][ew][kBlkF] = fn;
      }
    }
    STAMP(2);
    // contact blocks beyond kResident (rare: >4 contacts): solver block and J rows streamed from the
    // record at use (a prefetch's double buffers would cost the third wave per SIMD), forces written
    // back to the record by lane 0
    if (ncon_max > kResident) {
      for (int c = kResident; c < ncon_max; c++) {
        float4 v[kBlk], Jo[3];
        const float4* rec = reinterpret_cast<const float4*>(crec + c * kConStride);
#pragma unroll
        for (int k = 0; k < kBlk; k++) v[k] = rec[k];
#pragma unroll
        for (int i = 0; i < 3; i++) {
          const float4 t = rec[kBlk + 3 * q + i];
          Jo[i] = c < ncon ? t : zero4;
        }
        const bool act = c < ncon && !done;
        const bool arm = __ballot(c < ncon && v[kBlkFlags].y != 0.f) != 0ull;
        float4 fn;
        contact_update(v, Jo, qacc, mrow, act, q == 0, arm, impr, fn, newton);
        if (act && q == 0) reinterpret_cast<float4*>(crec + c * kConStride)[kBlkF] = fn;
      }
      __threadfence_block();   // the forces are re-read by all 4 lanes next sweep
    }
    STAMP(3);
    const float improvement = quadsum(impr) * pgs_scale;
    if (!done) {
      iters = it + 1;
      last_impr = improvement;
      if (improvement < tolerance) done = true;
    }
  }

  STAMP(4);
#ifdef SO100_TIMELINE
  {
    uint64_t tl_end;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tl_end)::"memory");
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (a.last && a.debug && tid == 0) {
      float* dbg = a.debug + (size_t)(grp * kPgsEnvs) * SO100_DBG_STRIDE;   // record of the wave's first env
      dbg[92] = __uint_as_float((uint32_t)tl_start);
      dbg[93] = __uint_as_float((uint32_t)tl_end);
      dbg[94] = __uint_as_float(hw);
      dbg[95] = __uint_as_float((uint32_t)ncon_max | (xcc << 8) | ((uint32_t)iters << 16));
    }
  }
#endif
#ifdef SO100_STAMPS
  if (valid && a.last && a.debug && q == 0) {
    float* dbg = a.debug + (size_t)env * SO100_DBG_STRIDE;
#pragma unroll
    for (int k = 0; k < 5; k++) dbg[88 + k] = (float)st_acc_[k];
    dbg[93] = (float)newton;
  }
#endif
  // ---------------- qacc -> HBM (the next stage's Euler input and the next substep's warmstart)
  if (valid) {
#pragma unroll
    for (int i = 0; i < 3; i++) a.qacc_out[(size_t)env * SO100_NV + 3 * q + i] = qacc[i];
    if (a.last && a.debug) {
      float* dbg = a.debug + (size_t)env * SO100_DBG_STRIDE;
#pragma unroll
      for (int i = 0; i < 3; i++) { dbg[4 + 3 * q + i] = qacc[i]; dbg[76 + 3 * q + i] = fr_f[i]; }
      if (q == 0) {
        dbg[1] = (float)iters;
        dbg[2] = last_impr;
        for (int c = 0; c < kMaxCon; c++) {
          float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
          if (c < ncon) f = c < kResident ? blk[c][ew][kBlkF] : reinterpret_cast<const float4*>(crec + c * kConStride)[kBlkF];
          dbg[32 + c] = f.x;
          dbg[96 + 3 * c] = f.y;
          dbg[97 + 3 * c] = f.z;
          dbg[98 + 3 * c] = f.w;
        }
        for (int c = kMaxCon; c < ncon; c++) {      // the contacts beyond kMaxCon: geometry and force from the record
          const float* sl = crec + (size_t)c * kConStride;
          const float4 f = reinterpret_cast<const float4*>(sl)[kBlkF];
          float* d = dbg + SO100_DBG_OVF + 6 * (c - kMaxCon);
          d[0] = sl[kGeoDist];
          d[1] = (float)__float_as_int(sl[kGeoPair]);
          d[2] = f.x; d[3] = f.y; d[4] = f.z; d[5] = f.w;
        }
      }
    }
  }
}

hipError_t launch_pgs(const DevModel* m, const Workspace& w, float* qacc_out, float* debug, int n, int last, int par,
                      hipStream_t s) {
  const int ngroups = (n + kPgsEnvs - 1) / kPgsEnvs;
  const int heavy = ngroups < kHeavyCap ? ngroups : kHeavyCap;
  PgsArgs a{m, w, qacc_out, debug, n, last, par, heavy};
  hipLaunchKernelGGL(so100_pgs_kernel, dim3(ngroups + heavy), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace so100
