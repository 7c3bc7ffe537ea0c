// so100_pool.h — the fused step's contact-record pool (Workspace::pool): HBM records for the envs whose contact list is
// longer than the kMaxCon held on chip, taken per substep.  (internal; included by so100_convex.h)
#pragma once
#include "so100_common.h"
#include "so100_device.h"
#include "so100_kin.h"

namespace so100 {

// The fused path's contact-record pool (Workspace::pool): entries of kEnvsPerBlock records, one per env of a wave, taken
// by a wave for one substep the first time one of its envs' contact list passes kMaxCon, from the pool of the wave's
// XCD (its L2 holds every access of the entry: no cross-XCD coherence is needed), and returned after the solve.  A wave
// holds at most one entry and takes it whole, so it never waits while holding one: pool_acquire (one lane of the wave)
// takes the lowest free entry of this XCD's bitmap; with none free it sleeps and retries, and every holder is a running
// wave that returns its entry at the end of its substep, so one comes free.  (Per-env records, round 5's first cut,
// deadlocked under contention: a wave holding one env's record waited for another's.)  After kPoolSpins tries (about
// a second, never reached in any measured run) it gives up: -2, and the envs keep their first kMaxCon contacts, counted
// in ncon_dropped (a checked invariant: every test asserts 0).
constexpr int kPoolSpins = 1 << 22;
DEV int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & (kPoolXcd - 1);
}
DEV int pool_acquire(const Workspace& w) {
  const int x = xcc_id();
  uint32_t* bm = w.pool_bm + x * kPoolWords;
  const int nw = (w.pool_recs + 31) >> 5;
  for (int spin = 0; spin < kPoolSpins; spin++) {
    for (int k = 0; k < nw; k++) {
      const int nb = min(32, w.pool_recs - 32 * k);
      const uint32_t full = nb == 32 ? 0xffffffffu : (1u << nb) - 1u;
      uint32_t cur = __hip_atomic_load(bm + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while ((cur & full) != full) {
        const int b = __builtin_ctz(~cur);
        const uint32_t old = atomicOr(bm + k, 1u << b);
        if (!(old & (1u << b))) return x * kPoolSlots + 32 * k + b;
        cur = old | (1u << b);
      }
    }
    __builtin_amdgcn_s_sleep(8);
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
  __builtin_amdgcn_s_waitcnt(0);    // the substep's stores to the entry have reached L2 before another wave may take it
  const int x = ent / kPoolSlots, b = ent % kPoolSlots;
  atomicAnd(w.pool_bm + x * kPoolWords + (b >> 5), ~(1u << (b & 31)));
}
// The env's record for a list about to reach `total` contacts (every lane of the wave calls it; the envs' counts are
// uniform in their rows): the split path's per-env record as given; on the fused path, when an env's list passes
// kMaxCon and its wave holds no entry, the wave takes one (shm[0].rec: the wave's entry; -1: none yet, -2: the pool's
// safety valve), and the env's lanes read back its record (nullptr: none).  Collision calls it before each phase stores
// its contacts, with that phase's total.  shm: the wave's 4 envs.
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
