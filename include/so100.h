/* so100.h — C-ABI of the MI355X-native batched SO-ARM100 simulator (libso100_hip.so).
 *
 * This boundary replaces, for N envs at once, what the reference reaches through dm_control:
 *   gym_so100/env.py:98-127   mujoco.Physics.from_xml_path + control.Environment   -> so100_create
 *   gym_so100/env.py:148-170  SO100Env.reset (BOX_POSE, reset_context, mj_forward)  -> so100_reset
 *   gym_so100/env.py:172-182  SO100Env.step -> control.Environment.step:
 *        single_arm.py:33-38  before_step (unnormalize, fp32 ctrl)
 *        env.py:174           Physics.step(10)  (mj_step2; mj_step x9; mj_step1)
 *        single_arm.py:322-380/149-215/246-285 get_reward,  :82-114 get_observation
 *        env.py:130-146,175   obs packing, terminated = reward == 4                 -> so100_step
 *   gym_so100/env.py:341-353  SO100GoalEnv.compute_reward (batched)                 -> so100_goal_reward
 *
 * Conventions: plain pointers and sizes only; every array is DEVICE memory allocated by the caller
 * (PyTorch-ROCm tensors in the Python layer); row-major [n_envs, dim].  Calls enqueue on `stream`
 * (a hipStream_t, NULL = default stream) and never synchronise the host.  Status: 0 = ok, < 0 = error
 * (message in so100_last_error()): -1 bad arguments / model, -2 a HIP error, -3 a C++ exception caught at the
 * boundary (e.g. host memory exhausted).  No C++ exceptions cross this boundary.
 */
#ifndef SO100_H
#define SO100_H
#include <stdint.h>
#include "so100_model.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SO100_ABI_VERSION 17  /* 17: so100_pool_stats (the fused step's contact-record pool, sized never to run out);  16: so100_source_hash;  15: the EE variant's mocap marker box collides (SO100_NGEOM 16, SO100_NPAIR 209, SO100_NCON_MAX 643, debug stride 3,922);  14: no per-env contact cap (SO100_NCON_MAX: every pair at its collider's maximum), debug stride 3,436 (SO100_DBG_OVF), ncon_dropped always 0, status -3 for a caught C++ exception;  13: so100_buffers.ep_return / ep_final / ep_accum (device-side episode statistics);  12: so100_model.convex (GJK/EPA mesh collider, MuJoCo 3.3.3 default), box-box up to 8 contacts, cube-table one convex contact;  11: so100_buffers.ncon_dropped, debug stride 160 (contact friction forces), so100_set_fused_build;  10: so100_hull_cells (MPR support lookup);  9: pad/link-hull pairs (SO100_NPAIR 191);  8: fused step kernel, so100_set_step_mode;  7: reward64 buffer;  6: Base hull + pad pairs (SO100_NPAIR 155, SO100_NHULL_ALL 10); 5: EE/mocap weld, render API */

/* tasks (gym_so100/__init__.py:4-32 ids; single_arm.py task classes) */
#define SO100_TASK_CUBE_TO_BIN 0          /* gym_so100/SO100CubeToBin-v0, TimeLimit 700 */
#define SO100_TASK_TOUCH_CUBE 1           /* gym_so100/SO100TouchCube-v0, TimeLimit 300 */
#define SO100_TASK_TOUCH_CUBE_SPARSE 2    /* gym_so100/SO100TouchCubeSparse-v0, TimeLimit 300 */
#define SO100_TASK_GOAL 3                 /* SO100GoalEnv (env.py:188-409), own 300-step limit */

/* step flags */
#define SO100_FLAG_AUTORESET 1            /* reset done envs in-kernel, final obs -> final_obs */
#define SO100_FLAG_DR 2                   /* per-env domain randomisation (dr_params)          */

typedef struct so100_buffers {
  /* per-env state, updated in place */
  float*    qpos;            /* [N,13]  hinges(6) cube pos(3) cube quat wxyz(4) */
  float*    qvel;            /* [N,12]  hinges(6) cube linear(3, world) angular(3, body) */
  float*    qacc_warmstart;  /* [N,12] */
  int32_t*  elapsed;         /* [N]     steps in the current episode (TimeLimit counter) */
  uint32_t* episode;         /* [N]     episodes started (drives in-kernel reset seeds) */
  /* inputs */
  const float* action;       /* [N,6]   in [-1,1] (action_space Box) */
  /* outputs (any may be NULL) */
  float*    obs;             /* [N,15]  box(3) bin(3) ee(3) qpos[:6] */
  float*    reward;          /* [N] */
  uint8_t*  terminated;      /* [N] */
  uint8_t*  truncated;       /* [N] */
  uint8_t*  success;         /* [N]     info["is_success"] */
  float*    final_obs;       /* [N,15]  obs of the finished episode when auto-reset fired */
  uint8_t*  diverged;        /* [N]     non-finite / exploding state detected (env reset) */
  uint32_t* contact_bits;    /* [N]     bit p: contact pair p active after the step */
  /* GoalEnv (task SO100_TASK_GOAL) */
  float*    achieved_goal;   /* [N,3] */
  float*    desired_goal;    /* [N,3] */
  int32_t*  total_steps;     /* [N]     curriculum counter (env.py:324) */
  /* domain randomisation (flag SO100_FLAG_DR): [N,4] = cube mass scale, friction scale,
   * action-noise sigma, reserved */
  const float* dr_params;
  /* diagnostics: [N, SO100_DBG_STRIDE] floats or NULL */
  float*    debug;
  /* EE / mocap variant (model.ee = 1): [N,7] mocap body pose, position(3) + quaternion wxyz(4), the
   * target the weld equality pulls ee_site to (teleop_ee.py:52-98 drives data.mocap_pos/quat); NULL =
   * the model's default pose */
  const float* mocap;
  /* [N] the reward in float64, as the reference returns it (task_reward computes in double; `reward`
   * holds its float32 rounding, exact for the CubeToBin / sparse / GoalEnv ladders, rounded for the dense
   * TouchCube shaping); NULL = not written */
  double*   reward64;
  /* [N] contacts left out of the env's contact list, summed over the step's substeps (the oracle's ncon_dropped).
   * Since ABI 14 the list holds every contact (SO100_NCON_MAX, as MuJoCo keeps every contact), so this is always
   * written as 0: kept as a checked invariant.  NULL = not written */
  uint32_t* ncon_dropped;
  /* Device-side episode statistics (what gymnasium's RecordEpisodeStatistics / SB3's VecMonitor keep on the
   * host, reference scripts/train_sac.py:290; SURVEY §5 Metrics), written by the step epilogue; the host reads
   * them only on demand.  ep_final and ep_accum are written only when ep_return is given.  NULL = not kept.
   *   ep_return [N]   return of the running episode: the sum of its float64 rewards so far; set to 0 when the
   *                   episode ends (terminated or truncated, with or without auto-reset) and by so100_reset;
   *                   without auto-reset, an env stepped on past its TimeLimit without a reset is counted once;
   *   ep_final  [N,2] return and length (steps) of the env's last finished episode, written at its end;
   *   ep_accum  [N,4] over the env's finished episodes: count, successes (ended with is_success), sum of
   *                   returns, sum of lengths; never cleared by the library (the caller zeroes it). */
  double*   ep_return;
  double*   ep_final;
  double*   ep_accum;
} so100_buffers;

/* Debug record per env (floats), written by the last substep of a step when `debug` is not NULL:
 *   [0] ncon  [1] solver iterations  [2] last improvement  [3] nefc  [4..15] qacc (the last solve)
 *   [16..31] contact dist  [32..47] contact normal force (efc_force row 0 of contact c)   (contacts c < 16)
 *   [48..63] contact pair id (-1 unused)  [64..75] qacc_smooth  [76..87] dof frictionloss forces
 *   [88..95] profiling stamps (diagnostic builds)
 *   [96..143] contact c's friction forces (efc_force rows 1..3 of contact c) at 96 + 3 c   (contacts c < 16)
 *   [144..159] reserved
 *   [SO100_DBG_OVF + 6 (c - 16) ...] contacts c >= 16 of the list: dist, pair id, normal force, 3 friction forces */
#define SO100_DBG_OVF 160
#define SO100_DBG_STRIDE (SO100_DBG_OVF + 6 * (SO100_NCON_MAX - SO100_MAXCON))   /* 3,922 */

typedef struct so100_env so100_env;   /* opaque: device model copy + launch config */

int         so100_abi_version(void);
const char* so100_last_error(void);
/* (ABI 16) the content hash (sha256, 16 hex digits) of the sources the library was built from: ties a committed
 * measurement (profiles/r05_pmc_step_*.json) to the kernels it measured (bench.py reports traffic only on a match) */
const char* so100_source_hash(void);
/* sizeof(so100_model), sizeof(so100_buffers) as compiled — lets bindings verify their mirrors. */
int         so100_struct_sizes(int* model_bytes, int* buffers_bytes);

/* Upload the model (converted to fp32) to `device`.  n_envs > 0.  Returns NULL on error. */
so100_env*  so100_create(const so100_model* model, int n_envs, int device);
int         so100_destroy(so100_env* env);
int         so100_num_envs(const so100_env* env);

/* Task selection: task id, TimeLimit (max_episode_steps; <= 0 = none), base seed for in-kernel resets,
 * global index of this shard's env 0 (multi-GPU sharding: in-kernel seeds use the global env id). */
int so100_configure(so100_env* env, int task, int max_episode_steps, uint64_t base_seed, int env_offset);

/* Reset the envs whose mask byte is non-zero (mask NULL = all).  seeds: [N] uint32 per-env seeds for
 * the reference's RandomState(seed) cube spawn (utils.py:18-29), or NULL -> in-kernel seed from
 * (base_seed, env, episode).  Writes obs (and GoalEnv goals). */
int so100_reset(so100_env* env, const so100_buffers* b, const uint8_t* mask, const uint32_t* seeds,
                void* stream);

/* One env step for all N envs (10 physics substeps + final position stage + reward/obs epilogue).
 * The N envs are split into up to 4 contiguous chunks (so100_chunk_info) whose launch sequences run
 * concurrently on internal streams forked from and joined back to `stream`: from the caller's side
 * the step is one ordered operation on `stream`. */
int so100_step(so100_env* env, const so100_buffers* b, int flags, void* stream);

/* Kernel timing for the benchmark's roofline (not needed for stepping).  so100_profile_enable(env,
 * max_steps) allocates HIP events for up to max_steps subsequent so100_step calls (0 frees them and
 * stops recording); while enabled each step records an event on its stream before its first launch
 * and after every launch (stage / solver kernels) of the first chunk.  so100_profile_read synchronises
 * on the last event and returns the summed device time of the solver and of the stage launches since
 * enabling. */
int so100_profile_enable(so100_env* env, int max_steps);
int so100_profile_read(so100_env* env, double* solver_ms, int* solver_launches, double* stage_ms,
                       int* stage_launches);

/* Step mode (Newton solver): 1 = the whole env step as ONE fused kernel launch over all N envs, the
 * substep's constraint rows handed from the assembly to the solve in registers; 0 = the split path, per
 * substep a stage kernel and a solver kernel exchanging an HBM record (2 nsubstep + 1 launches per env
 * chunk); -1 = auto (default): fused at every N (SO100_FUSED_MAX=n: split above n).  Both give
 * the same results bit for bit.  The PGS solver always runs split.  so100_step_mode returns the mode in
 * effect (0/1).  In fused mode so100_profile_read reports the fused launches as the solver launches
 * (stage: 0) and so100_chunk_info reports 1 chunk of N envs. */
int so100_set_step_mode(so100_env* env, int fused);
int so100_step_mode(const so100_env* env);

/* Register budget of the fused kernel's product build (the build launched when `debug` is NULL): 2 = 2 waves
 * per SIMD (186 VGPRs, no scratch), 3 = 3 waves per SIMD (168 VGPRs), 0 = auto (default: the 2-wave build
 * when the grid fits the chip at 2 waves per SIMD, <= 8 x CUs workgroups; the 3-wave build above).  The
 * SO100_FUSED_WAVES environment variable sets the initial value.  Register allocation only: every build
 * gives the same results bit for bit (tests/test_gpu_parity.py test_product_builds_bitwise).
 * so100_fused_build returns the build the next fused step of the env launches (1 = the debug build). */
int so100_set_fused_build(so100_env* env, int waves);
int so100_fused_build(const so100_env* env, int debug);

/* Support-direction cells of the convex hulls (host only; no device needed).  The MPR collider's hull
 * support (the first vertex maximising n . v, MuJoCo's mesh support by exhaustive scan) reads a candidate
 * list instead of the whole hull: the direction's cube-map face (largest |n_k|) and its G x G cell on that
 * face select the vertices that can be the support for some direction of the cell (a vertex beaten by one
 * other vertex by >= 1e-6 over the whole cell, its bounds widened by 1e-3, is left out), so the scan of the
 * list returns the same vertex as the scan of the hull.
 *   cells[SO100_NHULL_ALL * SO100_HULL_NCELL]: hull k, face f (2 axis + (n_axis < 0)), cell (cu, cv) at
 *     k * NCELL + (f * G + cu) * G + cv: start << 8 | count (count 0: scan the whole hull);
 *   cand[cap][4]: x, y, z (the hull vertex as float) and the vertex index within the hull (as float bits).
 * Returns the number of candidates (cand may be NULL to query it), -1 on error. */
/* (SO100_HULL_CELLG, SO100_HULL_NCELL: so100_model.h) */
int so100_hull_cells(const so100_model* model, uint32_t* cells, float* cand, int cap);

/* Number of env chunks and the env count of chunk 0 (the launches so100_profile_read times). */
int so100_chunk_info(const so100_env* env, int* nchunks, int* profiled_envs);

/* Adds the contact count of the last solver launch, summed over the N envs, to *accum (DEVICE
 * uint64).  Enqueued on `stream`, no synchronisation. */
int so100_contact_count(so100_env* env, uint64_t* accum, void* stream);
/* Writes each env's contact count of the last solver launch (the last substep's list) to out (DEVICE int32 [N]).
 * Enqueued on `stream`, no synchronisation.  (ABI 14) */
int so100_contact_counts(so100_env* env, int32_t* out, void* stream);
/* (ABI 17) The fused step's contact-record pool: out[0] = pool entries taken (wave-substeps whose
 * env lists passed the 16 held on chip), out[1] = entry requests that found none free (0 by construction: each XCD's
 * pool holds as many entries as the XCD can hold fused waves resident), out[2] = entries per XCD; the first two summed
 * over the steps since so100_create or the last reset != 0 call.  Synchronises the device (a benchmark / test hook). */
int so100_pool_stats(so100_env* env, uint64_t* out, int reset);

/* ---- camera images: the reference's default observation, obs_type
 * "so100_pixels_agent_pos" (gym_so100/__init__.py:4-32) = the `top` camera rendered by dm_control
 * (gym_so100/env.py:84-94,130-136; scene_so100.xml:30).  A rasteriser of its own (not MuJoCo's OpenGL
 * output): flat Lambert shading of the visible geoms under the scene's lights.  DESIGN.md §3.7. */
#define SO100_MAX_LIGHTS 4
typedef struct so100_camera {
  float pos[3];                     /* camera position (world) */
  float mat[9];                     /* row-major rotation; columns = camera x (right), y (up), z (backward) */
  int   track;                      /* 1: mode="targetbody" on the ee body, frame recomputed per env (mat unused) */
  float fovy;                       /* vertical field of view, degrees */
  float znear;                      /* triangles with a vertex nearer than this are not drawn */
  float head_ambient, head_diffuse; /* headlight (scene_so100.xml:9) */
  int   nlight;                     /* directional lights (scene_so100.xml:13-18) */
  float light_dir[SO100_MAX_LIGHTS][3];
  float light_diffuse[SO100_MAX_LIGHTS];
} so100_camera;
/* Upload the scene's triangles (host arrays): tri [ntri][3][3] vertices in their body's frame, body
 * [ntri] (0 world, 1 Base, 2..7 arm links, 8 cube), rgb [ntri][3] base colour in [0, 1]. */
int so100_render_mesh(so100_env* env, const float* tri, const int* body, const float* rgb, int ntri);
/* Render the N envs at qpos (device [N][13]) from `cam` into out (device [N][height][width][3] uint8);
 * mask (device [N] uint8, NULL = all) limits the envs drawn, the others' images are left as they were.
 * Enqueued on stream; width <= 4096 and width * height <= 1 << 22. */
int so100_render(so100_env* env, const float* qpos, const uint8_t* mask, const so100_camera* cam, int width,
                 int height, uint8_t* out, void* stream);

/* Batched sparse GoalEnv reward (env.py:341-353): out[i] = ||a_i - d_i|| < threshold ? 0 : -1. */
int so100_goal_reward(so100_env* env, int n, const float* achieved, const float* desired, float* out,
                      void* stream);

/* Task reward epilogue as a standalone op (for parity against the reference's golden vectors):
 * cube_site[n,3] fp32, ee_site[n,3] fp32, pair_bits[n] -> reward[n] fp32, using the same device
 * function as the step kernel. */
int so100_eval_reward(so100_env* env, int task, int n, const float* cube_site, const float* ee_site,
                      const uint32_t* pair_bits, float* reward, void* stream);

/* Reference spawn op: seeds[n] -> pose[n,7] (fp64) via device MT19937 (utils.py:18-29). */
int so100_spawn_pose(so100_env* env, int n, const uint32_t* seeds, double* pose, void* stream);

/* Action prologue as a standalone op: action[n,6] -> ctrl[n,6] (constants.py:78-86, fp32 write-back). */
int so100_unnormalize(so100_env* env, int n, const float* action, float* ctrl, void* stream);

#ifdef __cplusplus
}
#endif
#endif
