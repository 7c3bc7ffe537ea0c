// so100_pool.h — the fused step's contact-record pool (Workspace::pool): HBM records for the envs whose contact list is
// longer than the kMaxCon held on chip, taken per substep.  (internal; included by so100_convex.h)
#pragma once
#include "so100_common.h"
#include "so100_device.h"
#include "so100_kin.h"

namespace so100 {

// The fused path's contact-record pool (Workspace::pool): entries of kEnvsPerBlock records, one per env of a wave, taken
// by a wave for one substep the first time one of its envs' contact list passes kMaxCon, from the pool of the wave's
// XCD (its L2 holds every access of the entry), and returned after the solve.
//
// Never exhausted, by construction (round 6): alloc_fused_workspace sizes each XCD's pool to the most fused-kernel waves
// that XCD can hold resident at once (its CUs x the kernel's resident workgroups per CU, from the occupancy API, and no
// more than the grid's waves).  Only a resident wave holds an entry, and it holds at most one (taken whole, once per
// substep), so a wave that asks finds one free on its first scan: no wave ever waits, no contact is ever dropped, and
// the time a step takes does not depend on how many of its envs hold long lists.  (Round 5 sized the pool by the env
// count, 8-32 entries per XCD, and let a wave finding none sleep and retry, then after about a second keep its first
// kMaxCon contacts: a dropped contact depended on timing.)  The scan is bounded by kPoolScans; not finding an entry
// there would contradict the sizing, and is reported, not hidden: the entry is -2, the envs keep their first kMaxCon
// contacts counted in ncon_dropped (every test asserts 0) and Workspace::pool_stat[1] counts the event (the wave counts
// its takes and failures in LDS, shm[1].rec / shm[2].rec, and adds them to pool_stat once, in the epilogue: an atomic
// here, inside the collision phase's register peak, spilled the 3-wave build).
constexpr int kPoolScans = 64;
DEV int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & (kPoolXcd - 1);
}
DEV int pool_acquire(const Workspace& w) {
  const int x = xcc_id();
  uint32_t* bm = w.pool_bm + x * kPoolWords;
  const int nw = (w.pool_recs + 31) >> 5;
  for (int scan = 0; scan < kPoolScans; scan++) {
    for (int k = 0; k < nw; k++) {
      const int nb = min(32, w.pool_recs - 32 * k);
      const uint32_t full = nb == 32 ? 0xffffffffu : (1u << nb) - 1u;
      uint32_t cur = __hip_atomic_load(bm + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while ((cur & full) != full) {
        const int b = __builtin_ctz(~cur);
        // acquire: the entry's previous holder's accesses, released below, happen before this holder's;
        // the agent-scope acquire also drops this CU's L1 copies of the entry's lines
#ifdef SO100_POOL_R5   // (A/B switch: round 5's relaxed take)
        const uint32_t old = atomicOr(bm + k, 1u << b);
#else
        const uint32_t old = __hip_atomic_fetch_or(bm + k, 1u << b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
#endif
        if (!(old & (1u << b))) return x * kPoolSlots + 32 * k + b;
        cur = old | (1u << b);
      }
    }
  }
  return -2;
}
// env grp's record in pool entry `ent` (XCD ent / kPoolSlots, bit ent % kPoolSlots of its bitmap), or nullptr for
// ent < 0 (no entry held)
DEV float* pool_rec(const Workspace& w, int ent, int grp) {
  if (ent < 0) return nullptr;
  const int x = ent / kPoolSlots, b = ent % kPoolSlots;
  return w.pool + (((size_t)x * w.pool_recs + b) * kEnvsPerBlock + grp) * kConEnv;
}
DEV void pool_release(const Workspace& w, int ent) {
  // every load and store of the holder's substep completes before the entry's bit clears (the hardware wait), and the
  // "memory" clobber keeps the compiler from moving any of them past it (__builtin_amdgcn_s_waitcnt is not a
  // compiler barrier).  No data passes to the next holder (a holder reads only what it wrote in its own substep) and
  // both holders meet in this XCD's L2, so no L2 write-back is needed: the release orders completion, not visibility.
#ifdef SO100_POOL_R5
  __builtin_amdgcn_s_waitcnt(0);
#else
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
  const int x = ent / kPoolSlots, b = ent % kPoolSlots;
  __hip_atomic_fetch_and(w.pool_bm + x * kPoolWords + (b >> 5), ~(1u << (b & 31)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}
// The env's record for a list about to reach `total` contacts (every lane of the wave calls it; the envs' counts are
// uniform in their rows): the split path's per-env record as given; on the fused path, when an env's list passes
// kMaxCon and its wave holds no entry, the wave takes one (shm[0].rec: the wave's entry; -1: none yet, -2: none found,
// which the sizing rules out), and the env's lanes read back its record (nullptr: none).  Collision calls it before each
// phase stores its contacts, with that phase's total.  shm: the wave's 4 envs.
template <bool kFused>
DEV float* ensure_rec(const Workspace& w, EnvShared* shm, int grp, int lane, bool valid, int total, float* crec) {
  if constexpr (!kFused) {
    return crec;
  } else {
    const bool need = valid && total > kMaxCon;
    if (__ballot(need) != 0ull) {
      if (lane == 0 && grp == 0 && shm[0].rec == -1) shm[0].rec = pool_acquire(w);
      __syncthreads();
    }
    return pool_rec(w, shm[0].rec, grp);
  }
}

}  // namespace so100
