// so100_render.hip — batched camera images: the reference's default observation
// (obs_type="so100_pixels_agent_pos", gym_so100/__init__.py:4-32), the `top` camera rendered by
// dm_control's physics.render (gym_so100/env.py:84-94,130-136; scene_so100.xml:30), SURVEY §8 f.3.
//
// MuJoCo renders with OpenGL; this is a rasteriser of our own on the same scene description: the
// visible geoms (tools/compile_render.py: the arm's visual meshes, decimated, the table, bin and cube
// boxes, with their colours), the camera pose and field of view, the headlight and the scene's
// directional lights (Lambert diffuse + ambient, two-sided, flat per triangle; no specular, shadows or
// anti-aliasing).  It reproduces what is where in the image, not MuJoCo's pixel values: parity with
// MuJoCo's renderer is unpinned.
//
// Layout: one 256-thread workgroup per env.
//   * thread 0 runs the stage kernel's forward kinematics (so100_kin.h) into LDS, 9 body frames;
//   * the image is drawn in bands of up to kTilePx pixels; per band, an LDS depth buffer of 64-bit keys
//     (depth bits << 32 | RGB8) takes ds_min_u64 atomics, so the nearest surface wins and equal depths
//     resolve to the smaller colour: the image does not depend on thread order;
//   * phase A: thread t projects triangles t, t+256, ... and rasterises the small ones itself; triangles
//     covering more than kBigPx pixels of the band go to an LDS list and phase B rasterises each with all
//     256 threads (the table's two faces cover the whole image: one thread would serialise the block).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "so100_device.h"
#include "so100.h"
#include "so100_common.h"
#include "so100_kin.h"

namespace so100 {

constexpr int kRenderThreads = 256;
constexpr int kTilePx = 4096;           // depth-buffer pixels per band (32 KB of LDS)
constexpr int kBigPx = 64;              // triangles with a larger band bbox go to phase B
constexpr int kBigCap = 256;

struct RenderArgs {
  const DevModel* m;
  const float4* tri;                    // [ntri][3] body-frame vertices (w unused)
  const int* tri_body;                  // [ntri] body (0 world, 1 Base, 2..7 links, 8 cube)
  const uint32_t* tri_rgb;              // [ntri] RGB8 base colour
  int ntri;
  const float* qpos;                    // [n][13]
  const uint8_t* mask;                  // [n] or null: envs to draw
  so100_camera cam;
  int n, width, height;
  uint8_t* out;                         // [n][height][width][3]
};

DEV uint32_t shade(const RenderArgs& a, const float* cm, const float* p0, const float* p1, const float* p2,
                   uint32_t rgb) {
  float e1[3], e2[3], nrm[3];
#pragma unroll
  for (int k = 0; k < 3; k++) { e1[k] = p1[k] - p0[k]; e2[k] = p2[k] - p0[k]; }
  cross3(nrm, e1, e2);
  const float nl = sqrtf(dot3(nrm, nrm));
  const float inv = nl > 0.f ? 1.f / nl : 0.f;
#pragma unroll
  for (int k = 0; k < 3; k++) nrm[k] *= inv;
  // two-sided: the normal facing the camera
  float v[3] = {a.cam.pos[0] - p0[0], a.cam.pos[1] - p0[1], a.cam.pos[2] - p0[2]};
  if (dot3(nrm, v) < 0.f) { nrm[0] = -nrm[0]; nrm[1] = -nrm[1]; nrm[2] = -nrm[2]; }
  // headlight: along the view direction (camera -z), so its diffuse term is n . z_cam
  const float zc[3] = {cm[2], cm[5], cm[8]};
  float lum = a.cam.head_ambient + a.cam.head_diffuse * fmaxf(0.f, dot3(nrm, zc));
  for (int l = 0; l < a.cam.nlight; l++) lum += a.cam.light_diffuse[l] * fmaxf(0.f, -dot3(nrm, a.cam.light_dir[l]));
  uint32_t out = 0;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const float base = (float)((rgb >> (8 * c)) & 0xFFu) * (1.f / 255.f);
    const float val = fminf(fmaxf(base * lum, 0.f), 1.f);
    out |= (uint32_t)(val * 255.f + 0.5f) << (8 * c);
  }
  return out;
}

__global__ void __launch_bounds__(kRenderThreads) so100_render_kernel(RenderArgs a) {
  __shared__ EnvShared sh;
  __shared__ float frm[SO100_NBODY][12];           // body rotation (9) + position (3)
  __shared__ unsigned long long zb[kTilePx];
  __shared__ int big[kBigCap];
  __shared__ int nbig;
  __shared__ float cmat[9];                        // camera frame (columns x, y, z) for this env
  const DevModel* __restrict__ m = a.m;
  const int tid = threadIdx.x, env = blockIdx.x;
  if (env >= a.n || (a.mask && !a.mask[env])) return;     // uniform per block
  const int W = a.width, H = a.height;

  // ---- forward kinematics of this env (the stage kernel's fk_stage on thread 0)
  if (tid < SO100_NQ) sh.qpos[tid] = a.qpos[(size_t)env * SO100_NQ + tid];
  __syncthreads();
  joint_sincos(sh, tid);
  __syncthreads();
  if (tid == 0) {
    fk_stage(m, sh);
    float bq[4] = {m->base_quat[0], m->base_quat[1], m->base_quat[2], m->base_quat[3]}, bm[9];
    quat2mat(bm, bq);
    for (int b = 0; b < SO100_NBODY; b++) {
      float R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, P[3] = {0, 0, 0};
      if (b == 1) {
        for (int k = 0; k < 9; k++) R[k] = bm[k];
        for (int k = 0; k < 3; k++) P[k] = m->base_pos[k];
      } else if (b >= 2 && b <= 7) {
        for (int k = 0; k < 9; k++) R[k] = sh.ser.xm[b - 2][k];
        for (int k = 0; k < 3; k++) P[k] = sh.ser.xp[b - 2][k];
      } else if (b == SO100_CUBE_BODY) {
        for (int k = 0; k < 9; k++) R[k] = sh.cube_mat[k];
        for (int k = 0; k < 3; k++) P[k] = sh.cube_pos[k];
      }
      for (int k = 0; k < 9; k++) frm[b][k] = R[k];
      for (int k = 0; k < 3; k++) frm[b][9 + k] = P[k];
    }
    if (a.cam.track) {
      // mode="targetbody" on the ee body (scene_so100.xml:30 front_close -> vx300s_left/camera_focus, whose
      // origin is ee_site): MuJoCo's mj_camlight frame z = pos - target, x = (0,0,1) x z, y = z x x
      float z[3] = {a.cam.pos[0] - sh.site_ee[0], a.cam.pos[1] - sh.site_ee[1], a.cam.pos[2] - sh.site_ee[2]};
      float x[3], y[3];
      const float up[3] = {0.f, 0.f, 1.f};
      float n = sqrtf(dot3(z, z));
      if (n < 1e-15f) { z[0] = 1.f; z[1] = z[2] = 0.f; } else { z[0] /= n; z[1] /= n; z[2] /= n; }
      cross3(x, up, z);
      n = sqrtf(dot3(x, x));
      if (n < 1e-15f) { x[0] = 1.f; x[1] = x[2] = 0.f; } else { x[0] /= n; x[1] /= n; x[2] /= n; }
      cross3(y, z, x);
      for (int k = 0; k < 3; k++) { cmat[3 * k] = x[k]; cmat[3 * k + 1] = y[k]; cmat[3 * k + 2] = z[k]; }
    } else {
      for (int k = 0; k < 9; k++) cmat[k] = a.cam.mat[k];
    }
  }
  __syncthreads();

  const float th = tanf(0.5f * a.cam.fovy * 0.017453292519943295f);
  const float aspect = (float)W / (float)H;
  const int band = kTilePx / W > 0 ? kTilePx / W : 1;        // rows per band
  uint8_t* img = a.out + (size_t)env * H * W * 3;

  for (int y0 = 0; y0 < H; y0 += band) {
    const int y1 = min(H, y0 + band);
    const int npx = (y1 - y0) * W;
    for (int i = tid; i < npx; i += kRenderThreads) zb[i] = ~0ull;
    if (tid == 0) nbig = 0;
    __syncthreads();

    // screen-space triangle: pixel x to the right, y down; depth along the camera's -z
    auto setup = [&](int t, float* sx, float* sy, float* iz, uint32_t& col, int& bx0, int& bx1, int& by0,
                     int& by1) -> bool {
      const int b = a.tri_body[t];
      float pw[3][3];
      bool ok = true;
#pragma unroll
      for (int v = 0; v < 3; v++) {
        const float4 q = a.tri[3 * t + v];
        const float* R = frm[b];
        float w[3];
        w[0] = R[0] * q.x + R[1] * q.y + R[2] * q.z + R[9];
        w[1] = R[3] * q.x + R[4] * q.y + R[5] * q.z + R[10];
        w[2] = R[6] * q.x + R[7] * q.y + R[8] * q.z + R[11];
        const float d[3] = {w[0] - a.cam.pos[0], w[1] - a.cam.pos[1], w[2] - a.cam.pos[2]};
        const float cx = cmat[0] * d[0] + cmat[3] * d[1] + cmat[6] * d[2];
        const float cy = cmat[1] * d[0] + cmat[4] * d[1] + cmat[7] * d[2];
        const float cz = cmat[2] * d[0] + cmat[5] * d[1] + cmat[8] * d[2];
        const float depth = -cz;
        ok = ok && depth > a.cam.znear;
        const float id = 1.f / depth;
        sx[v] = (cx * id / (th * aspect) * 0.5f + 0.5f) * (float)W;
        sy[v] = (0.5f - cy * id / th * 0.5f) * (float)H;
        iz[v] = id;
#pragma unroll
        for (int k = 0; k < 3; k++) pw[v][k] = w[k];
      }
      if (!ok) return false;
      const float area = (sx[1] - sx[0]) * (sy[2] - sy[0]) - (sx[2] - sx[0]) * (sy[1] - sy[0]);
      if (!(fabsf(area) > 1e-12f)) return false;
      bx0 = max(0, (int)floorf(fminf(sx[0], fminf(sx[1], sx[2])) - 0.5f));
      bx1 = min(W - 1, (int)ceilf(fmaxf(sx[0], fmaxf(sx[1], sx[2])) - 0.5f));
      by0 = max(y0, (int)floorf(fminf(sy[0], fminf(sy[1], sy[2])) - 0.5f));
      by1 = min(y1 - 1, (int)ceilf(fmaxf(sy[0], fmaxf(sy[1], sy[2])) - 0.5f));
      if (bx0 > bx1 || by0 > by1) return false;
      col = shade(a, cmat, pw[0], pw[1], pw[2], a.tri_rgb[t]);
      return true;
    };
    // one pixel of a set-up triangle: edge functions at the pixel centre, perspective-correct depth
    auto raster = [&](const float* sx, const float* sy, const float* iz, uint32_t col, int x, int y) {
      const float px = (float)x + 0.5f, py = (float)y + 0.5f;
      const float area = (sx[1] - sx[0]) * (sy[2] - sy[0]) - (sx[2] - sx[0]) * (sy[1] - sy[0]);
      const float w0 = (sx[2] - sx[1]) * (py - sy[1]) - (sy[2] - sy[1]) * (px - sx[1]);
      const float w1 = (sx[0] - sx[2]) * (py - sy[2]) - (sy[0] - sy[2]) * (px - sx[2]);
      const float w2 = (sx[1] - sx[0]) * (py - sy[0]) - (sy[1] - sy[0]) * (px - sx[0]);
      const float sg = area > 0.f ? 1.f : -1.f;
      if (w0 * sg < 0.f || w1 * sg < 0.f || w2 * sg < 0.f) return;
      const float inv = 1.f / area;
      const float izp = (w0 * iz[0] + w1 * iz[1] + w2 * iz[2]) * inv;
      if (!(izp > 0.f)) return;
      const float depth = 1.f / izp;
      const unsigned long long key = ((unsigned long long)__float_as_uint(depth) << 32) | col;
      atomicMin(&zb[(y - y0) * W + x], key);
    };

    // ---- phase A: one triangle per thread; large ones are listed for phase B
    for (int t = tid; t < a.ntri; t += kRenderThreads) {
      float sx[3], sy[3], iz[3];
      uint32_t col;
      int bx0, bx1, by0, by1;
      if (!setup(t, sx, sy, iz, col, bx0, bx1, by0, by1)) continue;
      if ((bx1 - bx0 + 1) * (by1 - by0 + 1) > kBigPx) {
        const int k = atomicAdd(&nbig, 1);
        if (k < kBigCap) { big[k] = t; continue; }
      }
      for (int y = by0; y <= by1; y++)
        for (int x = bx0; x <= bx1; x++) raster(sx, sy, iz, col, x, y);
    }
    __syncthreads();
    // ---- phase B: each large triangle with all threads over its bbox
    const int nb = min(nbig, kBigCap);
    for (int k = 0; k < nb; k++) {
      float sx[3], sy[3], iz[3];
      uint32_t col;
      int bx0, bx1, by0, by1;
      if (!setup(big[k], sx, sy, iz, col, bx0, bx1, by0, by1)) continue;   // uniform: same triangle
      const int bw = bx1 - bx0 + 1, cnt = bw * (by1 - by0 + 1);
      for (int i = tid; i < cnt; i += kRenderThreads) raster(sx, sy, iz, col, bx0 + i % bw, by0 + i / bw);
    }
    __syncthreads();
    // ---- band -> image (background: black)
    for (int i = tid; i < npx; i += kRenderThreads) {
      const unsigned long long key = zb[i];
      const uint32_t col = key == ~0ull ? 0u : (uint32_t)(key & 0xFFFFFFu);
      uint8_t* px = img + ((size_t)y0 * W + i) * 3;
      px[0] = (uint8_t)(col & 0xFFu);
      px[1] = (uint8_t)((col >> 8) & 0xFFu);
      px[2] = (uint8_t)((col >> 16) & 0xFFu);
    }
    __syncthreads();
  }
}

hipError_t launch_render(const DevModel* m, const float4* tri, const int* body, const uint32_t* rgb, int ntri,
                         const float* qpos, const uint8_t* mask, const so100_camera& cam, int n, int width, int height, uint8_t* out,
                         hipStream_t s) {
  RenderArgs a{m, tri, body, rgb, ntri, qpos, mask, cam, n, width, height, out};
  hipLaunchKernelGGL(so100_render_kernel, dim3(n), dim3(kRenderThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace so100
