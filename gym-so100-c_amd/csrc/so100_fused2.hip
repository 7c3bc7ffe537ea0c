// so100_fused2.hip — the 2-wave product build of the fused step kernel (so100_fused_kernel<false, 2>: grids of at most
// 2 waves per SIMD, e.g. the 8,192-env shard) in a translation unit of its own, so that the Makefile can compile it with
// LLVM's iterative-ILP scheduler without changing the other kernels' (so100_step.hip: launch_fused2).
#define SO100_FUSED2_TU
#include "so100_step.hip"
