// probe: fk_par (lane-parallel) against fk_stage (lane 0) on the start pose, one env row (tools/dev)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include "so100_kin.h"
static const float k_base_pos[] = {-0.469, 0.5, 0};
static const float k_base_quat[] = {0.707105483, 0, 0, 0.70710808};
static const float k_body_pos[] = {0, -0.0452, 0.0165, 0, 0.1025, 0.0306, 0, 0.11257, 0.028, 0, 0.0052, 0.1349, 0, -0.0601, 0, -0.0202, -0.0244, 0};
static const float k_body_quat[] = {0.707105281, 0.707108281, 0, 0, 0.707109018, 0.707104544, 0, 0, 0.707109018, -0.707104544, 0, 0, 0.707109018, -0.707104544, 0, 0, 0.707109018, 0, 0.707104544, 0, 1.34924e-11, -3.67321e-06, 1, -3.67321e-06};
static const float k_jnt_axis[] = {0, 1, 0, 1, 0, 0, 1, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1};
static const float k_site_ee[] = {0, -0.06, 0};
static const float k_qpos_h[] = {0, -0.96, 1.16, 0, 0, 0.02239, 0, 0.5, 0.02, 1, 0, 0, 0};
__device__ float k_qpos_d(int i) { const float q[13] = {0, -0.96f, 1.16f, 0, 0, 0.02239f, 0, 0.5f, 0.02f, 1, 0, 0, 0}; return q[i]; }
using namespace so100;
__global__ void k(const DevModel* m, float* out) {
  __shared__ EnvShared A, B;
  const int lane = threadIdx.x & 15;
  if (threadIdx.x < 16) {
    if (lane < 13) { A.qpos[lane] = k_qpos_d(lane); B.qpos[lane] = k_qpos_d(lane); }
  }
  __syncthreads();
  if (threadIdx.x < 16) joint_sincos(A, lane);
  __syncthreads();
  if (threadIdx.x == 0) fk_stage(m, A);
  __syncthreads();
  if (threadIdx.x < 16) fk_par(m, B, lane);
  __syncthreads();
  if (threadIdx.x == 0) {
    int o = 0;
    for (int a = 0; a < 6; a++) {
      for (int t = 0; t < 3; t++) { out[o++] = A.ser.xp[a][t]; out[o++] = B.ser.xp[a][t]; }
      for (int t = 0; t < 9; t++) { out[o++] = A.ser.xm[a][t]; out[o++] = B.ser.xm[a][t]; }
      for (int t = 0; t < 3; t++) { out[o++] = A.axis[a][t]; out[o++] = B.axis[a][t]; }
    }
    for (int t = 0; t < 3; t++) { out[o++] = A.site_ee[t]; out[o++] = B.site_ee[t]; }
  }
}

int main() {
  DevModel h;
  memset(&h, 0, sizeof(h));
  memcpy(h.base_pos, k_base_pos, sizeof(h.base_pos)); memcpy(h.base_quat, k_base_quat, sizeof(h.base_quat));
  memcpy(h.body_pos, k_body_pos, sizeof(h.body_pos)); memcpy(h.body_quat, k_body_quat, sizeof(h.body_quat));
  memcpy(h.jnt_axis, k_jnt_axis, sizeof(h.jnt_axis)); memcpy(h.site_ee, k_site_ee, sizeof(h.site_ee));
  DevModel* d; float* o;
  (void)hipMalloc(&d, sizeof(h)); (void)hipMalloc(&o, 4096);
  (void)hipMemcpy(d, &h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  float r[512]; (void)hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
  int n = 0;
  for (int a = 0; a < 6; a++) {
    printf("body %d:", a);
    for (int t = 0; t < 15; t++, n += 2) printf(" %.5f/%.5f", r[n], r[n + 1]);
    printf("\n");
  }
  printf("site_ee:"); for (int t = 0; t < 3; t++, n += 2) printf(" %.5f/%.5f", r[n], r[n + 1]); printf("\n");
  return 0;
}
