// so100_newton.hip — the split path's Newton kernel: one substep's constraint solve (so100_newton.h) on the
// record the stage kernel writes in Newton mode (so100_device.h NewtonHdr).  The default step runs the
// fused kernel instead (so100_step.hip so100_fused_kernel), which hands the same rows over in registers.
#include "so100_newton.h"
#include "so100.h"

namespace so100 {

constexpr int kNewtonWaves = 3;   // waves per SIMD the register budget is sized for

struct NewtonArgs {
  const DevModel* m;
  Workspace w;
  float* qacc_out;               // so100_buffers.qacc_warmstart: the solver's qacc (next warmstart)
  float* debug;
  int n;
  int last;                      // last substep of the env step: write the debug record
};

__global__ void __launch_bounds__(kThreads, kNewtonWaves) so100_newton_kernel(NewtonArgs a) {
  const int tid = threadIdx.x, grp = tid >> 4, lane = tid & 15;
  const int env = blockIdx.x * kEnvsPerBlock + grp;
  const bool valid = env < a.n;
  const int e = valid ? env : 0;
  __shared__ float4 jx_sh[kEnvsPerBlock][kJLds * SO100_NV];
  NewtonRows r;
  newton_rows_load(a.w, e, lane, valid, jx_sh[grp], r);
  __syncthreads();
  NewtonDiag diag;
  const bool dbg = a.last && a.debug;
  float* const crec = a.w.con + (size_t)e * kConEnv;      // contacts beyond kMaxCon (rare)
  const float qacc = newton_solve_any(a.m, r, lane, valid, dbg, diag, [&]() { return crec; });
  if (dbg) {
    newton_diag_write(a.debug + (size_t)env * SO100_DBG_STRIDE, lane, valid, qacc, diag);
    if (valid) newton_diag_write_ovf(a.debug + (size_t)env * SO100_DBG_STRIDE, crec, r.ncon, lane);
  }
  // qacc -> HBM (the next stage's Euler input and the next substep's warmstart)
  if (valid && lane < SO100_NV) a.qacc_out[(size_t)env * SO100_NV + lane] = qacc;
}

hipError_t launch_newton(const DevModel* m, const Workspace& w, float* qacc_out, float* debug, int n, int last,
                         hipStream_t s) {
  NewtonArgs a{m, w, qacc_out, debug, n, last};
  hipLaunchKernelGGL(so100_newton_kernel, dim3((n + kEnvsPerBlock - 1) / kEnvsPerBlock), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace so100
