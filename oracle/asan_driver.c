/* asan_driver.c — TEST INFRASTRUCTURE: runs the oracle (so100_oracle.c) under AddressSanitizer and
 * UndefinedBehaviorSanitizer (SURVEY §5 "race detection / sanitizers": the CPU restatement under ASan/UBSan).
 *
 * The Python interpreter that drives the CPU suite is not instrumented, so the sanitizers run on this
 * instrumented executable instead (`make -C oracle asan`; tests/test_oracle_sanitizers.py runs it).  It
 * loads a model written by gym_so100.model (the so100_model struct's bytes) and drives every oracle stage
 * over contact-rich states: random arm poses within the joint ranges (self-collision, Base and pad/link
 * hull contacts through MPR), cubes pressed into a bin corner (up to 12 contacts: beyond the 16 the kernels hold on chip),
 * cubes spawned by RandomState seeds, and random actions, with the model's solver and variant.
 *
 * usage: oracle_asan_{64,32} <model.bin> <envs> <steps>      exit 0 = clean (a sanitizer report aborts)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "so100_oracle.h"

static unsigned long long rng_state = 0x9E3779B97F4A7C15ull;
static double urand(void) {   /* splitmix64 -> [0, 1) */
  unsigned long long z = (rng_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) / 9007199254740992.0;
}

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: %s model.bin envs steps\n", argv[0]); return 2; }
  so100_model m;
  FILE* f = fopen(argv[1], "rb");
  if (!f) { perror("model"); return 2; }
  if (fread(&m, 1, sizeof(m), f) != sizeof(m)) { fprintf(stderr, "model: short read (%zu B expected)\n", sizeof(m)); return 2; }
  fclose(f);
  const int nenv = atoi(argv[2]), steps = atoi(argv[3]);
  so100o_data* d = (so100o_data*)calloc((size_t)nenv, sizeof(so100o_data));
  long contacts = 0, dropped = 0, max_ncon = 0;
  for (int e = 0; e < nenv; e++) {
    double pose[7];
    so100o_spawn_pose(1000u + (unsigned)e, pose);
    const int kind = e % 4;
    if (kind == 1) {            /* pressed into the bin corner */
      pose[0] = -0.165 + 1e-3 * urand(); pose[1] = 0.735 + 1e-3 * urand(); pose[2] = 0.021 - 1e-3 * urand();
    } else if (kind == 2) {     /* on the Base top */
      pose[0] = -0.469; pose[1] = 0.5; pose[2] = 0.12;
    }
    so100o_reset(&m, &d[e], pose);
    if (kind != 0) {            /* a random arm pose: self / Base / pad-link contacts */
      for (int j = 0; j < 6; j++) d[e].qpos[j] = m.jnt_range[j][0] + (m.jnt_range[j][1] - m.jnt_range[j][0]) * urand();
    }
    if (m.ee) {
      for (int k = 0; k < 3; k++) d[e].mocap_pos[k] += 0.04 * (urand() - 0.5);
    }
  }
  float obs[SO100_NOBS], act[6];
  for (int s = 0; s < steps; s++) {
    for (int e = 0; e < nenv; e++) {
      for (int k = 0; k < 6; k++) act[k] = (float)(2 * urand() - 1);
      int term = 0;
      const double r = so100o_env_step(&m, &d[e], s % 3, act, obs, &term);
      contacts += d[e].snap_ncon;
      dropped += d[e].snap_ndrop;
      if (d[e].snap_ncon > max_ncon) max_ncon = d[e].snap_ncon;
      for (int k = 0; k < SO100_NQ; k++)
        if (!isfinite((double)d[e].qpos[k])) { fprintf(stderr, "env %d step %d: non-finite qpos\n", e, s); return 1; }
      if (!(r >= -1.0 && r <= 4.0)) { fprintf(stderr, "env %d step %d: reward %g\n", e, s, r); return 1; }
    }
  }
  /* the batched CPU baseline entry point (OpenMP) over the same states */
  float* acts = (float*)malloc(sizeof(float) * 6 * (size_t)nenv * 2);
  for (int i = 0; i < 6 * nenv * 2; i++) acts[i] = (float)(2 * urand() - 1);
  const long ran = so100o_batch_run(&m, d, nenv, 2, 0, acts, 2);
  free(acts);
  printf("ok: %d envs x %d steps (solver %d, ee %d, real %d B): contacts %ld (max %ld per env), dropped %ld, batch %ld\n",
         nenv, steps, m.solver, m.ee, so100o_real_bytes(), contacts, max_ncon, dropped, ran);
  free(d);
  return 0;
}
