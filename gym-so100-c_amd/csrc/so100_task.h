// so100_task.h — the task layer the reference computes in numpy: action un-normalisation (constants.py:44-47,78-86,
// single_arm.py:33-38), the reward ladders (single_arm.py:149-215,246-285,322-380), the RandomState cube spawn
// (utils.py:18-29) and the counter-based hashes of the in-kernel resets and domain randomisation.
// (internal; included by so100_step.hip, the one translation unit of the step kernels)
#pragma once
#include "so100_common.h"

namespace so100 {

// ------------------------------------------------------------------ task prologue / epilogue
// constants.py:44-47,78-86 applied to a float32 copy (single_arm.py:33-38): float32 ops, no FMA.
// span = fp32(max_val - min_val) with the subtraction in double (python floats), as numpy does.
DEV float unnormalize_f32(float a, float lo, float hi, float span) {
#pragma clang fp contract(off)
  float t = a + 1.0f;
  float u = t / 2.0f;
  float v = u * span;
  float w = v + lo;
  w = w < lo ? lo : w;
  return w > hi ? hi : w;
}

// reward ladders — single_arm.py:322-380 / :149-215 / :246-285 (double, exactly as the reference)
DEV double task_reward(const DevModel* __restrict__ m, int task, const float* cube_f, const float* ee_f,
                       uint32_t bits) {
#pragma clang fp contract(off)
  double bmin[3], bmax[3];
  const double hw = m->bin_hw, h = m->bin_h;
  bmin[0] = m->bin_center[0] + -hw; bmin[1] = m->bin_center[1] + -hw; bmin[2] = m->bin_center[2] + 0.0;
  bmax[0] = m->bin_center[0] + hw;  bmax[1] = m->bin_center[1] + hw;  bmax[2] = m->bin_center[2] + h;
  const bool touch_gripper = (bits & ((1u << SO100_NPAIR_GRIPPER) - 1u)) != 0u;
  const bool touch_table = ((bits >> SO100_PAIR_TABLE) & 1u) != 0u;
  if (task == SO100_TASK_CUBE_TO_BIN || task == SO100_TASK_GOAL) {
    double c[3] = {(double)cube_f[0], (double)cube_f[1], (double)cube_f[2]};
    bool over = (bmin[0] < c[0] && c[0] < bmax[0]) && (bmin[1] < c[1] && c[1] < bmax[1]);
    bool inside = true;
    const float half = (float)m->cube_half;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      float lower = cube_f[k] - half, upper = cube_f[k] + half;
      inside = inside && ((double)lower > bmin[k]) && ((double)upper < bmax[k]);
    }
    bool released = inside && !touch_gripper;
    double r = 0.0;
    if (touch_gripper) r = 1.0;
    if (touch_gripper && !touch_table) r = 2.0;
    if (over) r = 2.5;
    if (inside) r = 3.0;
    if (released) r = 4.0;
    return r;
  }
  double dx = (double)ee_f[0] - (double)cube_f[0], dy = (double)ee_f[1] - (double)cube_f[1];
  double dz = (double)ee_f[2] - (double)cube_f[2];
  double dist = sqrt(dx * dx + dy * dy + dz * dz);
  bool success = touch_gripper && dist < 0.05;
  if (task == SO100_TASK_TOUCH_CUBE_SPARSE) return success ? m->max_reward : -0.2;
  double r = 0.0;
  if (dist < 0.7) r = fmax(r, 0.1 * (1.0 - dist / 0.7));
  if (dist < 0.5) r = fmax(r, 0.2 * (1.0 - dist / 0.5));
  if (dist < 0.3) r = fmax(r, 0.5 * (1.0 - dist / 0.3));
  if (dist < 0.1) r = fmax(r, 1.0 * (1.0 - dist / 0.1));
  if (dist < 0.05) r = fmax(r, 2.0 * (1.0 - dist / 0.05));
  if (touch_gripper) r += 1.0;
  if (success) return m->max_reward;
  return r - 0.2;
}

// ------------------------------------------------------------------ RNG: numpy legacy MT19937 spawn
// RandomState(seed).uniform(lo, hi) for 3 components (utils.py:18-29): init_genrand, one twist of the
// first 6 words (needs mt[0..6] and mt[397..402]), tempering, 53-bit doubles.
DEV uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
DEV void spawn_pose(const DevModel* __restrict__ m, uint32_t seed, double* pose) {
#pragma clang fp contract(off)
  uint32_t lo[7], hi[6];
  uint32_t s = seed;
  lo[0] = s;
#pragma unroll
  for (int i = 1; i < 7; i++) { s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i; lo[i] = s; }
  for (int i = 7; i < 397; i++) s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
#pragma unroll
  for (int i = 397; i < 403; i++) { s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i; hi[i - 397] = s; }
  uint32_t out[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    uint32_t y = (lo[i] & 0x80000000u) | (lo[i + 1] & 0x7fffffffu);
    uint32_t v = hi[i] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    out[i] = mt_temper(v);
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    uint32_t a = out[2 * k] >> 5, b = out[2 * k + 1] >> 6;
    // no contraction: numpy evaluates (a*2^26 + b) / 2^53 and low + (high-low)*u with rounded ops
    double u = ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
    double range = m->spawn_hi[k] - m->spawn_lo[k];
    double scaled = range * u;
    pose[k] = m->spawn_lo[k] + scaled;
  }
  pose[3] = 1.0; pose[4] = 0.0; pose[5] = 0.0; pose[6] = 0.0;
}
DEV uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
DEV uint32_t episode_seed(uint64_t base, uint32_t env, uint32_t episode) {
  return (uint32_t)splitmix64(base ^ splitmix64(((uint64_t)env << 32) | episode));
}
DEV float hash_uniform(uint64_t key) { return (float)(splitmix64(key) >> 40) * (1.0f / 16777216.0f); }
DEV float hash_normal(uint64_t key) {
  float u1 = fmaxf(hash_uniform(key), 1e-7f), u2 = hash_uniform(key ^ 0xA5A5A5A5A5A5A5A5ull);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// Diagnostic builds only: SSTAMP_RAW accumulates the shader cycles since the last stamp into slot (-1: none).
// With -DSO100_DYN_STAMPS the stage stamps cover the position / dynamics stage's phases instead (DSTAMP,

}  // namespace so100
