// so100_capi.cpp — extern "C" boundary of libso100_hip.so (declared in include/so100.h).
//
// so100_create converts the double-precision host model (so100_model) into the fp32 device model
// (DevModel) with the model-constant parts of MuJoCo's constraint setup precomputed on the host
// (frictionloss R at pos 0, solref -> K/B, pair invweight sums), uploads it once, and returns an
// opaque handle.  Every other call only validates arguments and enqueues a kernel on the caller's
// stream: no allocation, no synchronisation.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <cstring>
#include <string>
#include <exception>
#include <new>
#include <vector>
#include "so100.h"
#include "so100_device.h"

namespace so100 {
hipError_t launch_step(const DevModel*, int, int, int, int, Workspace&, const so100_buffers&, int, int, int, int,
                       uint64_t, int, hipStream_t, hipEvent_t*);
int fused_build(int n, int waves, bool debug);
hipError_t launch_contact_count(const Workspace&, int, uint64_t*, hipStream_t);
hipError_t launch_contact_counts(const Workspace&, int, int32_t*, hipStream_t);
hipError_t launch_render(const DevModel*, const float4*, const int*, const uint32_t*, int, const float*,
                         const uint8_t*, const so100_camera&, int, int, int, uint8_t*, hipStream_t);
hipError_t alloc_workspace(int, Workspace*);
hipError_t alloc_fused_workspace(int, Workspace*);
hipError_t free_workspace(Workspace*);
hipError_t launch_reset(const DevModel*, const so100_buffers&, int, int, uint64_t, int, const uint8_t*, const uint32_t*,
                        hipStream_t);
hipError_t launch_reward(const DevModel*, int, int, const float*, const float*, const uint32_t*, float*, hipStream_t);
hipError_t launch_spawn(const DevModel*, int, const uint32_t*, double*, hipStream_t);
hipError_t launch_unnormalize(const DevModel*, int, const float*, float*, hipStream_t);
hipError_t launch_goal_reward(const DevModel*, int, const float*, const float*, float*, hipStream_t);
}  // namespace so100

using so100::DevModel;
using so100::Workspace;

// A contiguous env range with its own substep workspace and stream.  With more than one chunk the
// chunks' launch sequences run concurrently (forked from / joined to the caller's stream), so one
// chunk's stage kernel fills the SIMD slots left idle by another chunk's solver tail.
struct Chunk {
  int start = 0, count = 0;
  Workspace ws{};               // substep hand-off record between the stage and solver kernels
  hipStream_t s = nullptr;      // nullptr: the caller's stream (single chunk)
  hipEvent_t done = nullptr;
};

struct StepGraph {
  hipGraphExec_t exec = nullptr;
  hipEvent_t done = nullptr;    // recorded after each replay (eviction waits for it)
  so100_buffers buf{};
  int flags = 0;
  uint32_t par = 0;             // substep-counter parity at the captured step's start
  uint64_t last_use = 0;
};
constexpr size_t kMaxStepGraphs = 32;

struct so100_env {
  int device;
  int n;
  DevModel* d_model;
  int nsubstep;
  int solver;                   // SO100_SOLVER_* of the model
  int fused;                    // step mode: 1 fused, 0 split, -1 auto (fused up to fused_max envs; Newton only)
  int fused_max;                // auto mode: the largest env count that runs fused
  Workspace fws{};              // fused launches: record header (contact counts) of all n envs, wave order
  bool last_fused = false;      // the mode of the last step (so100_contact_count reads its record)
  std::vector<Chunk> chunks;
  hipEvent_t fork = nullptr;
  int task;
  int max_steps;
  uint64_t base_seed;
  int env_offset;
  // camera render mesh (so100_render_mesh)
  float4* r_tri = nullptr;
  int* r_body = nullptr;
  uint32_t* r_rgb = nullptr;
  int r_ntri = 0;
  // profiling (so100_profile_enable): events[step][prof_per] (2 nsubstep + 2 split, 2 fused)
  std::vector<hipEvent_t> prof_ev;
  int prof_cap = 0, prof_used = 0, prof_per = 0;
  // step graphs: the 21 launches per chunk, the chunk fork and join, captured once per (buffers, flags,
  // substep parity) and replayed with one hipGraphLaunch when SO100_GRAPH=1.  A small LRU cache serves
  // callers that rotate a few action buffers (bench.py's pool of 16).  Off by default: the step is not
  // launch-bound (measured equal rates at 8,192 / 16,384 / 65,536 envs).
  bool use_graph = false;
  hipStream_t cap_s = nullptr;
  std::vector<StepGraph> graphs;
  uint64_t graph_clock = 0;
  float4* d_cand = nullptr;     // the hulls' support-cell candidates (DevModel::hull_cand)
  int fused_waves = 0;          // the fused product build: 2 | 3 waves per SIMD, 0 auto (so100_set_fused_build)
};

// An instantiated step graph can still be running when it is evicted: wait for its last replay first.
static void graph_destroy(StepGraph& g) {
  if (g.done) { (void)hipEventSynchronize(g.done); (void)hipEventDestroy(g.done); }
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  g.exec = nullptr;
  g.done = nullptr;
}

static void graph_free(so100_env* env) {
  for (StepGraph& g : env->graphs) graph_destroy(g);
  env->graphs.clear();
}

// The fused kernel implements the Newton solver only: PGS always takes the split launches.  Auto mode runs
// fused up to fused_max envs per GPU (SO100_FUSED_MAX; default: every size): round 3 measured the fused step
// faster at every shard size of the benchmark, 65,536 envs included (22.0 M vs 21.4 M env steps/s, +20 % at
// 32,768, +41 % at 16,384).
constexpr int kFusedAutoMax = 1 << 30;
static bool step_is_fused(const so100_env* env) {
  if (env->solver != SO100_SOLVER_NEWTON) return false;
  return env->fused < 0 ? env->n <= env->fused_max : env->fused != 0;
}

static hipError_t free_chunks(so100_env* env) {
  hipError_t e = hipSuccess;
  for (Chunk& c : env->chunks) {
    hipError_t e2 = so100::free_workspace(&c.ws);
    if (e == hipSuccess) e = e2;
    if (c.done) (void)hipEventDestroy(c.done);
    if (c.s) (void)hipStreamDestroy(c.s);
  }
  env->chunks.clear();
  if (env->fork) (void)hipEventDestroy(env->fork);
  env->fork = nullptr;
  return e;
}

// Chunk count: SO100_CHUNKS overrides; otherwise as many chunks as the process has hardware queues
// (GPU_MAX_HW_QUEUES, HIP's default 4; chunk 0 shares the caller's), at least 1,024 envs each.  More
// streams than queues serialise on shared queues (measured: 5-8 chunks run 1.6x slower than 4).
static int default_chunks(int n) {
  if (const char* v = getenv("SO100_CHUNKS")) {
    const int k = atoi(v);
    if (k >= 1 && k <= 16) return k;
  }
  int q = 4;
  if (const char* v = getenv("GPU_MAX_HW_QUEUES")) {
    const int k = atoi(v);
    if (k >= 1) q = k;
  }
  if (q > 4) q = 4;
  const int k = n / 1024;
  return k < 1 ? 1 : (k > q ? q : k);
}

static hipError_t make_chunks(so100_env* env, int nchunk) {
  const int n = env->n;
  const int unit = 64;                                   // whole stage blocks and solver groups
  const int units = (n + unit - 1) / unit;
  if (nchunk > units) nchunk = units;
  hipError_t e = hipSuccess;
  if (nchunk > 1) e = hipEventCreateWithFlags(&env->fork, hipEventDisableTiming);
  int start = 0;
  for (int k = 0; k < nchunk && e == hipSuccess; k++) {
    Chunk c;
    c.start = start;
    const int end = k == nchunk - 1 ? n : (int)((long)units * (k + 1) / nchunk) * unit;
    c.count = end - start;
    start = end;
    e = so100::alloc_workspace(c.count, &c.ws);
    // chunk 0 runs on the caller's stream: K chunks take K - 1 extra hardware queues
    if (e == hipSuccess && k > 0) e = hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking);
    if (e == hipSuccess && k > 0) e = hipEventCreateWithFlags(&c.done, hipEventDisableTiming);
    env->chunks.push_back(c);
  }
  return e;
}

// per-env buffer pointers of the env range starting at `s`
static so100_buffers offset_buffers(const so100_buffers& b, int s) {
  so100_buffers o = b;
  const size_t k = (size_t)s;
  auto off = [k](auto* p, int dim) { return p ? p + k * dim : p; };
  o.qpos = off(b.qpos, SO100_NQ);
  o.qvel = off(b.qvel, SO100_NV);
  o.qacc_warmstart = off(b.qacc_warmstart, SO100_NV);
  o.elapsed = off(b.elapsed, 1);
  o.episode = off(b.episode, 1);
  o.action = off(b.action, SO100_NU);
  o.obs = off(b.obs, SO100_NOBS);
  o.reward = off(b.reward, 1);
  o.terminated = off(b.terminated, 1);
  o.truncated = off(b.truncated, 1);
  o.success = off(b.success, 1);
  o.final_obs = off(b.final_obs, SO100_NOBS);
  o.diverged = off(b.diverged, 1);
  o.contact_bits = off(b.contact_bits, 1);
  o.achieved_goal = off(b.achieved_goal, 3);
  o.desired_goal = off(b.desired_goal, 3);
  o.total_steps = off(b.total_steps, 1);
  o.dr_params = off(b.dr_params, 4);
  o.debug = off(b.debug, SO100_DBG_STRIDE);
  o.mocap = off(b.mocap, 7);
  o.reward64 = off(b.reward64, 1);
  o.ncon_dropped = off(b.ncon_dropped, 1);
  o.ep_return = off(b.ep_return, 1);
  o.ep_final = off(b.ep_final, 2);
  o.ep_accum = off(b.ep_accum, 4);
  return o;
}

static void profile_free(so100_env* env) {
  for (hipEvent_t e : env->prof_ev) (void)hipEventDestroy(e);
  env->prof_ev.clear();
  env->prof_cap = env->prof_used = 0;
}

// the last error of this thread: a fixed buffer, so reporting an error never allocates (or throws)
static thread_local char g_err[512];

static int fail(const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return -1;
}
static int fail_hip(const char* where, hipError_t e) {
  snprintf(g_err, sizeof(g_err), "%s: %s", where, hipGetErrorString(e));
  return -2;
}

namespace {
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

void quat2mat(const double* q, double* m) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z);     m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z);     m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y);     m[7] = 2 * (y * z + w * x);     m[8] = 1 - 2 * (x * x + y * y);
}
void normq(const double* q, double* o) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int k = 0; k < 4; k++) o[k] = q[k] / n;
}
double clampimp(double v) { return v < 0.0001 ? 0.0001 : (v > 0.9999 ? 0.9999 : v); }
// MuJoCo getimpedance at pos == margin (x = 0) -> dmin (or the flat value)
double imp_at_zero(const double* solimp) {
  double dmin = clampimp(solimp[0]), dmax = clampimp(solimp[1]);
  if (dmin == dmax || solimp[2] <= 1e-15) return 0.5 * (dmin + dmax);
  return dmin;
}
void solref_kb(const double* solref, const double* solimp, double h, double* K, double* B) {
  double dmax = clampimp(solimp[1]);
  double tc = solref[0], dr = solref[1];
  if (tc > 0) {
    if (tc < 2 * h) tc = 2 * h;
    double den = dmax * dmax * tc * tc * dr * dr;
    *K = 1 / (den > 1e-15 ? den : 1e-15);
    double db = dmax * tc;
    *B = 2 / (db > 1e-15 ? db : 1e-15);
  } else {
    *K = -tc / (dmax * dmax);
    *B = -dr / dmax;
  }
}

int build_device_model(const so100_model* s, DevModel* d) {
  memset(d, 0, sizeof(*d));
  // structural assumptions of the specialised kernel
  for (int b = 2; b <= 7; b++)
    if (s->body_parent[b] != b - 1) return fail("model: arm bodies 2..7 must form a chain rooted at Base (1)");
  if (s->body_parent[1] != 0 || s->body_parent[SO100_CUBE_BODY] != 0) return fail("model: Base/cube must hang off world");
  for (int j = 0; j < SO100_NHINGE; j++)
    if (s->jnt_body[j] != j + 2) return fail("model: hinge j must sit on body j+2");
  for (int k = 0; k < 3; k++)
    if (fabs(s->body_ipos[SO100_CUBE_BODY][k]) > 1e-12) return fail("model: cube COM must be at the body origin");
  if (fabs(s->body_iquat[SO100_CUBE_BODY][0] - 1) > 1e-12) return fail("model: cube inertia must be body-aligned");
  if (s->site_ee_body != 6 || s->site_cube_body != SO100_CUBE_BODY) return fail("model: unexpected site bodies");
  for (int p = 0; p < SO100_NPAIR_BOX; p++)
    if (s->pair_condim[p] != 4) return fail("model: box-box pairs must have condim 4");
  if (s->geom_body[0] != 0 || fabs(s->geom_pos[0][2] + s->geom_size[0][2] - s->table_top) > 1e-9 ||
      fabs(s->geom_pos[0][0] - s->geom_size[0][0] - s->table_lo[0]) > 1e-6 ||
      fabs(s->geom_pos[0][0] + s->geom_size[0][0] - s->table_hi[0]) > 1e-6 ||
      fabs(s->geom_pos[0][1] - s->geom_size[0][1] - s->table_lo[1]) > 1e-6 ||
      fabs(s->geom_pos[0][1] + s->geom_size[0][1] - s->table_hi[1]) > 1e-6 || fabs(s->geom_quat[0][0] - 1) > 1e-12)
    return fail("model: geom 0 must be the table box, its top face table_top over table_lo..table_hi");
  for (int p = SO100_NPAIR_BOX; p < SO100_PAIR_MPR0; p++) {
    const int k = p - SO100_NPAIR_BOX;
    if (s->pair_condim[p] != 3 && s->pair_condim[p] != 4) return fail("model: hull pairs must have condim 3 or 4");
    if (s->pair_body1[p] != 0 || s->pair_body2[p] != s->hull_body[k]) return fail("model: hull pair k must be (table, hull k)");
    // the table is geom 0, a box (its mesh is an exact box) whose top face is table_top: the convex collider takes
    // it as obj1 (mpr_obj_setup's static box), the top-face rule as its top face and bottom
    if (s->pair_geom1[p] != 0 || s->pair_geom2[p] != -1 - k) return fail("model: hull pair k must be (geom 0 = the table, hull k)");
    if (s->pair_margin[p] != 0) return fail("model: table-hull pairs take no margin");
    if (s->hull_body[k] < 2 || s->hull_body[k] > 7) return fail("model: hulls must sit on arm bodies 2..7");
    if (s->hull_start[k] < 0 || s->hull_count[k] < 1 || s->hull_start[k] + s->hull_count[k] > SO100_HULL_NVERT)
      return fail("model: hull vertex range out of bounds");
  }
  // (box, hull) pairs of the MPR collider: box j = cube (geom 9) then the bin boxes (geoms 10..14), hull k
  for (int p = SO100_PAIR_MPR0; p < SO100_PAIR_SELF0; p++) {
    const int q = p - SO100_PAIR_MPR0, j = q / SO100_NHULL, k = q % SO100_NHULL;
    const int g = SO100_CUBE_GEOM + j;
    if (s->pair_geom1[p] != g || s->pair_geom2[p] != -1 - k) return fail("model: MPR pair p must be (box j, hull k)");
    if (s->pair_body1[p] != s->geom_body[g] || s->pair_body2[p] != s->hull_body[k]) return fail("model: MPR pair bodies");
    if (j > 0 && s->geom_body[g] != 0) return fail("model: bin boxes must be static");
    if (s->pair_condim[p] != 3 && s->pair_condim[p] != 4) return fail("model: MPR pairs must have condim 3 or 4");
    if (s->pair_margin[p] != 0) return fail("model: MPR pairs take no margin");
  }
  // the static Base hull: (cube, Base hull) then (Base hull, link hull k), all through MPR
  if (s->hull_body[SO100_HULL_BASE] != 1) return fail("model: hull 9 must be the Base's");
  if (s->hull_start[SO100_HULL_BASE] < 0 || s->hull_count[SO100_HULL_BASE] < 1 ||
      s->hull_start[SO100_HULL_BASE] + s->hull_count[SO100_HULL_BASE] > SO100_HULL_NVERT)
    return fail("model: Base hull vertex range out of bounds");
  if (s->body_parent[1] != 0) return fail("model: the Base must hang off the world");
  for (int p = SO100_PAIR_BASE0; p < SO100_PAIR_PADLINK0; p++) {
    const int g1 = s->pair_geom1[p], k2 = -1 - s->pair_geom2[p];
    if (p == SO100_PAIR_BASE0) {
      if (g1 != SO100_CUBE_GEOM || k2 != SO100_HULL_BASE) return fail("model: pair 98 must be (cube, Base hull)");
    } else if (g1 != -1 - SO100_HULL_BASE || k2 < 0 || k2 >= SO100_NHULL) {
      return fail("model: Base pairs must be (Base hull, link hull k)");
    }
    if (s->pair_condim[p] != 3 && s->pair_condim[p] != 4) return fail("model: Base pairs must have condim 3 or 4");
    if (s->pair_margin[p] != 0) return fail("model: MPR pairs take no margin");
  }
  // hull-hull self-collision pairs: two hulls on different arm links
  for (int p = SO100_PAIR_SELF0; p < SO100_PAIR_BASE0; p++) {
    const int k1 = -1 - s->pair_geom1[p], k2 = -1 - s->pair_geom2[p];
    if (k1 < 0 || k1 >= SO100_NHULL || k2 < 0 || k2 >= SO100_NHULL) return fail("model: self pair must be two hulls");
    if (s->pair_body1[p] != s->hull_body[k1] || s->pair_body2[p] != s->hull_body[k2] || k1 == k2)
      return fail("model: self pair bodies");
    if (s->pair_condim[p] != 3 && s->pair_condim[p] != 4) return fail("model: self pairs must have condim 3 or 4");
    if (s->pair_margin[p] != 0) return fail("model: MPR pairs take no margin");
  }
  // (finger pad, link hull) pairs through MPR: a pad box on a jaw against the Base or a link hull on bodies
  // 2..5 (the MPR kernel takes the pad's pose from its jaw's frame)
  for (int p = SO100_PAIR_PADLINK0; p < SO100_PAIR_MOCAPHULL0; p++) {
    const int g1 = s->pair_geom1[p], k2 = -1 - s->pair_geom2[p];
    if (g1 < 1 || g1 > SO100_NPAD || (s->geom_body[g1] != 6 && s->geom_body[g1] != 7))
      return fail("model: pad-link pair p must have a finger pad as geom1");
    if (k2 < 0 || k2 >= SO100_NHULL_ALL || s->hull_body[k2] > 5) return fail("model: pad-link pair p must have a link hull as geom2");
    if (s->pair_body1[p] != s->geom_body[g1] || s->pair_body2[p] != s->hull_body[k2]) return fail("model: pad-link pair bodies");
    if (s->pair_condim[p] != 3 && s->pair_condim[p] != 4) return fail("model: pad-link pairs must have condim 3 or 4");
    if (s->pair_margin[p] != 0) return fail("model: MPR pairs take no margin");
  }
  // the EE variant's mocap marker box (geom SO100_MOCAP_GEOM on the mocap body, centred on it: the kernels take its
  // pose as the mocap pose) against link hull k, through the convex collider
  if (s->geom_body[SO100_MOCAP_GEOM] != SO100_MOCAP_BODY) return fail("model: the marker box must sit on the mocap body");
  for (int k = 0; k < 3; k++)
    if (s->geom_pos[SO100_MOCAP_GEOM][k] != 0 || s->geom_quat[SO100_MOCAP_GEOM][1 + k] != 0)
      return fail("model: the marker box must be centred on the mocap body");
  for (int p = SO100_PAIR_MOCAPHULL0; p < SO100_PAIR_PAD0; p++) {
    const int k = p - SO100_PAIR_MOCAPHULL0;
    if (s->pair_geom1[p] != SO100_MOCAP_GEOM || s->pair_geom2[p] != -1 - k) return fail("model: pair p must be (marker, hull k)");
    if (s->pair_body1[p] != SO100_MOCAP_BODY || s->pair_body2[p] != s->hull_body[k]) return fail("model: marker-hull pair bodies");
    if (s->pair_condim[p] != 3 && s->pair_condim[p] != 4) return fail("model: marker pairs must have condim 3 or 4");
    if (s->pair_margin[p] != 0) return fail("model: MPR pairs take no margin");
  }
  // (cube | pad i, marker box) box-box pairs
  for (int p = SO100_PAIR_MOCAPBOX0; p < SO100_NPAIR; p++) {
    const int i = p - SO100_PAIR_MOCAPBOX0;
    if (s->pair_geom1[p] != (i == 0 ? SO100_CUBE_GEOM : i) || s->pair_geom2[p] != SO100_MOCAP_GEOM)
      return fail("model: pair p must be (cube | pad i, marker)");
    if (s->pair_body1[p] != s->geom_body[s->pair_geom1[p]] || s->pair_body2[p] != SO100_MOCAP_BODY)
      return fail("model: marker box pair bodies");
    if (s->pair_condim[p] != 3 && s->pair_condim[p] != 4) return fail("model: marker pairs must have condim 3 or 4");
  }
  // pad pairs: (finger pad i, table) at SO100_PAIR_PAD0 + i, (pad i, bin box j) at SO100_PAIR_PADBIN0 + 5 i + j
  for (int p = SO100_PAIR_PAD0; p < SO100_PAIR_MOCAPBOX0; p++) {
    const bool tbl = p < SO100_PAIR_PADBIN0;
    const int q = p - SO100_PAIR_PADBIN0;
    const int i = tbl ? p - SO100_PAIR_PAD0 : q / SO100_NBINBOX, j = tbl ? 0 : 1 + q % SO100_NBINBOX;
    const int g1 = s->pair_geom1[p], g2 = s->pair_geom2[p];
    if (g1 != 1 + i || g2 != (j == 0 ? 0 : SO100_CUBE_GEOM + j)) return fail("model: pad pair p must be (pad i, table | bin box j)");
    if (s->geom_body[g1] != 6 && s->geom_body[g1] != 7) return fail("model: pads must sit on the jaws");
    if (s->geom_body[g2] != 0) return fail("model: table and bin boxes must be static");
    if (s->pair_body1[p] != s->geom_body[g1] || s->pair_body2[p] != 0) return fail("model: pad pair bodies");
    if (s->pair_condim[p] != 3 && s->pair_condim[p] != 4) return fail("model: pad pairs must have condim 3 or 4");
  }
  for (int g = 0; g < SO100_NGEOM; g++) {
    int b = s->geom_body[g];
    if (!(b == 0 || b == 6 || b == 7 || b == SO100_CUBE_BODY || (g == SO100_MOCAP_GEOM && b == SO100_MOCAP_BODY)))
      return fail("model: geoms must be static, on the jaws, the cube or (the marker) the mocap body");
  }

  {
    double bq[4], bm[9];
    normq(s->body_quat[1], bq);
    quat2mat(bq, bm);
    for (int k = 0; k < 9; k++) d->base_xmat[k] = (float)bm[k];
    for (int k = 0; k < 3; k++) d->base_xpos[k] = (float)s->body_pos[1][k];
  }
  d->timestep = (float)s->timestep;
  d->nsubstep = s->nsubstep;
  d->iterations = s->iterations;
  if (s->solver != SO100_SOLVER_PGS && s->solver != SO100_SOLVER_NEWTON) return fail("model: unknown solver");
  d->solver = s->solver;
  if (s->convex != SO100_CONVEX_MPR && s->convex != SO100_CONVEX_EPA) return fail("model: unknown convex collider");
  d->convex = s->convex;
  d->tolerance = (float)s->tolerance;
  d->impratio = (float)s->impratio;
  for (int k = 0; k < 3; k++) d->gravity[k] = (float)s->gravity[k];
  d->pgs_scale = (float)(1.0 / (s->meaninertia * SO100_NV));
  double bq[4];
  normq(s->body_quat[1], bq);
  for (int k = 0; k < 3; k++) d->base_pos[k] = (float)s->body_pos[1][k];
  for (int k = 0; k < 4; k++) d->base_quat[k] = (float)bq[k];
  for (int a = 0; a < 6; a++) {
    int b = a + 2;
    double q[4], im[9];
    normq(s->body_quat[b], q);
    for (int k = 0; k < 3; k++) d->body_pos[a][k] = (float)s->body_pos[b][k];
    for (int k = 0; k < 4; k++) d->body_quat[a][k] = (float)q[k];
    for (int k = 0; k < 3; k++) d->body_ipos[a][k] = (float)s->body_ipos[b][k];
    normq(s->body_iquat[b], q);
    quat2mat(q, im);
    for (int k = 0; k < 9; k++) d->body_imat[a][k] = (float)im[k];
    d->body_mass[a] = (float)s->body_mass[b];
    for (int k = 0; k < 3; k++) d->body_inertia[a][k] = (float)s->body_inertia[b][k];
    for (int k = 0; k < 3; k++) d->jnt_axis[a][k] = (float)s->jnt_axis[a][k];
    d->jnt_lo[a] = (float)s->jnt_range[a][0];
    d->jnt_hi[a] = (float)s->jnt_range[a][1];
    d->armature[a] = (float)s->dof_armature[a];
  }
  d->cube_mass = (float)s->body_mass[SO100_CUBE_BODY];
  for (int k = 0; k < 3; k++) d->cube_inertia[k] = (float)s->body_inertia[SO100_CUBE_BODY][k];
  // frictionloss rows: pos = 0 -> imp = dmin; R = (1-imp)/imp * dof_invweight0
  double K, B;
  const double fimp = imp_at_zero(s->dof_solimp);
  for (int k = 0; k < SO100_NV; k++) {
    d->fr_floss[k] = (float)s->dof_frictionloss[k];
    double R = (1 - fimp) / fimp * s->dof_invweight0[k];
    d->fr_R[k] = (float)(R > 1e-15 ? R : 1e-15);
    if (!(s->dof_frictionloss[k] > 0)) return fail("model: the kernel expects frictionloss on every dof");
  }
  solref_kb(s->dof_solref, s->dof_solimp, s->timestep, &K, &B);
  d->fr_B = (float)B;
  solref_kb(s->jnt_solref, s->jnt_solimp, s->timestep, &K, &B);
  d->lim_K = (float)K;
  d->lim_B = (float)B;
  for (int k = 0; k < 5; k++) d->lim_solimp[k] = (float)s->jnt_solimp[k];
  // the kernels' impedance (so100_dynamics.h getimpedance) takes solimp power 1 or 2 (MuJoCo's power, clamped at 1)
  auto power_ok = [](const double* si) { const double pw = si[4] < 1 ? 1 : si[4]; return pw == 1 || pw == 2; };
  if (!power_ok(s->jnt_solimp) || !power_ok(s->dof_solimp) || !power_ok(s->weld_solimp))
    return fail("model: solimp power must be 1 or 2");
  for (int p = 0; p < SO100_NPAIR; p++)
    if (!power_ok(s->pair_solimp[p])) return fail("model: solimp power must be 1 or 2");
  for (int j = 0; j < 6; j++) d->lim_invw[j] = (float)s->dof_invweight0[j];
  for (int i = 0; i < SO100_NU; i++) {
    d->act_kp[i] = (float)s->act_kp[i];
    d->act_kv[i] = (float)s->act_kv[i];
    d->act_flo[i] = (float)s->act_forcerange[i][0];
    d->act_fhi[i] = (float)s->act_forcerange[i][1];
    d->act_clo[i] = (float)s->act_ctrlrange[i][0];
    d->act_chi[i] = (float)s->act_ctrlrange[i][1];
  }
  for (int g = 0; g < SO100_NGEOM; g++) {
    double q[4], gm[9];
    normq(s->geom_quat[g], q);
    quat2mat(q, gm);
    d->geom_body[g] = s->geom_body[g];
    for (int k = 0; k < 3; k++) d->geom_pos[g][k] = (float)s->geom_pos[g][k];
    for (int k = 0; k < 9; k++) d->geom_mat[g][k] = (float)gm[k];
    for (int k = 0; k < 3; k++) d->geom_size[g][k] = (float)s->geom_size[g][k];
    d->geom_rbound[g] = (float)sqrt(s->geom_size[g][0] * s->geom_size[g][0] + s->geom_size[g][1] * s->geom_size[g][1] +
                                    s->geom_size[g][2] * s->geom_size[g][2]);
  }
  for (int k = 0; k < 3; k++) { d->bin_lo[k] = 1e30f; d->bin_hi[k] = -1e30f; }
  for (int g = SO100_CUBE_GEOM + 1; g < SO100_CUBE_GEOM + 1 + SO100_NBINBOX; g++) {
    double q[4], gm[9];
    normq(s->geom_quat[g], q);
    quat2mat(q, gm);
    for (int k = 0; k < 3; k++) {
      const double r = fabs(gm[3 * k]) * s->geom_size[g][0] + fabs(gm[3 * k + 1]) * s->geom_size[g][1] +
                       fabs(gm[3 * k + 2]) * s->geom_size[g][2];
      d->bin_lo[k] = fminf(d->bin_lo[k], (float)(s->geom_pos[g][k] - r));
      d->bin_hi[k] = fmaxf(d->bin_hi[k], (float)(s->geom_pos[g][k] + r));
    }
  }
  for (int p = 0; p < SO100_NPAIR; p++) {
    // geoms: 0 <= g < SO100_NGEOM, or a hull -1 - k with 0 <= k < SO100_NHULL_ALL
    for (int g : {s->pair_geom1[p], s->pair_geom2[p]})
      if (g >= SO100_NGEOM || (g < 0 && -1 - g >= SO100_NHULL_ALL)) return fail("model: pair geom out of range");
    d->pair_g1[p] = s->pair_geom1[p];
    d->pair_g2[p] = s->pair_geom2[p];
    solref_kb(s->pair_solref[p], s->pair_solimp[p], s->timestep, &K, &B);
    d->pair_K[p] = (float)K;
    d->pair_B[p] = (float)B;
    for (int k = 0; k < 5; k++) d->pair_solimp[p][k] = (float)s->pair_solimp[p][k];
    d->pair_mu0[p] = (float)s->pair_friction[p][0];
    d->pair_mu1[p] = (float)s->pair_friction[p][1];
    d->pair_margin[p] = (float)s->pair_margin[p];
    const int b1 = s->pair_body1[p], b2 = s->pair_body2[p];
    // bodies 0..SO100_NBODY-1, or the mocap body (no dofs, welded to the world for the dynamics: invweight0 = 0)
    if (b1 < 0 || b1 > SO100_NBODY || b2 < 0 || b2 > SO100_NBODY) return fail("model: pair body out of range");
    static_assert(SO100_MOCAP_BODY == SO100_NBODY, "the mocap body follows the body arrays");
    // the kernels' box pairs take a geom's body from the pair (geom_pose_b)
    if ((s->pair_geom1[p] >= 0 && s->geom_body[s->pair_geom1[p]] != b1) ||
        (s->pair_geom2[p] >= 0 && s->geom_body[s->pair_geom2[p]] != b2))
      return fail("model: pair bodies must be their geoms' bodies");
    d->pair_b1[p] = b1;
    d->pair_b2[p] = b2;
    d->pair_cond4[p] = s->pair_condim[p] == 4;
    d->pair_arm[p] = (b1 >= 2 && b1 <= 7) || (b2 >= 2 && b2 <= 7);
    d->pair_cube[p] = b1 == SO100_CUBE_BODY || b2 == SO100_CUBE_BODY;
    auto invw = [&](int b, int k) { return b == SO100_MOCAP_BODY ? 0.0 : s->body_invweight0[b][k]; };
    d->pair_tran[p] = (float)(invw(b1, 0) + invw(b2, 0));
    d->pair_rot[p] = (float)(invw(b1, 1) + invw(b2, 1));
  }
  for (int k = 0; k < SO100_NHULL_ALL; k++) {
    // the convex collider's support ids hold a vertex index in 10 bits (so100_convex.h sup_from_id)
    if (s->hull_start[k] < 0 || s->hull_count[k] < 1 || s->hull_count[k] > 1024 ||
        s->hull_start[k] + s->hull_count[k] > SO100_HULL_NVERT)
      return fail("model: hull vertex range out of bounds (at most 1024 vertices per hull)");
    d->hull_body[k] = s->hull_body[k];
    d->hull_start[k] = s->hull_start[k];
    d->hull_count[k] = s->hull_count[k];
    d->hull_center[k] = {(float)s->hull_center[k][0], (float)s->hull_center[k][1], (float)s->hull_center[k][2], 0.f};
    d->hull_half[k] = {(float)s->hull_half[k][0], (float)s->hull_half[k][1], (float)s->hull_half[k][2],
                       (float)sqrt(s->hull_half[k][0] * s->hull_half[k][0] + s->hull_half[k][1] * s->hull_half[k][1] +
                                   s->hull_half[k][2] * s->hull_half[k][2])};
    d->hull_centroid[k] = {(float)s->hull_centroid[k][0], (float)s->hull_centroid[k][1], (float)s->hull_centroid[k][2], 0.f};
  }
  for (int v = 0; v < SO100_HULL_NVERT; v++)
    d->hull_vert[v] = {(float)s->hull_vert[v][0], (float)s->hull_vert[v][1], (float)s->hull_vert[v][2], 0.f};
  d->table_top = (float)s->table_top;
  d->table_bottom = (float)(s->table_top - 2 * s->geom_size[0][2]);
  for (int k = 0; k < 2; k++) {
    d->table_lo[k] = (float)s->table_lo[k];
    d->table_hi[k] = (float)s->table_hi[k];
  }
  for (int k = 0; k < 3; k++) {
    d->site_cube[k] = (float)s->site_cube_pos[k];
    d->site_ee[k] = (float)s->site_ee_pos[k];
    d->bin_center_f[k] = (float)s->bin_center[k];
    d->bin_center[k] = s->bin_center[k];
    d->spawn_lo[k] = s->spawn_lo[k];
    d->spawn_hi[k] = s->spawn_hi[k];
    d->goal_bin_lo[k] = (float)s->goal_bin_lo[k];
    d->goal_bin_hi[k] = (float)s->goal_bin_hi[k];
  }
  d->bin_hw = s->bin_hw;
  d->bin_h = s->bin_h;
  d->cube_half = s->cube_half;
  d->goal_threshold = s->goal_threshold;
  d->max_reward = s->max_reward;
  for (int i = 0; i < 6; i++) {
    d->start_qpos[i] = (float)s->start_qpos[i];
    d->action_lo[i] = (float)s->action_lo[i];
    d->action_hi[i] = (float)s->action_hi[i];
    d->action_span[i] = (float)(s->action_hi[i] - s->action_lo[i]);
  }
  // EE / mocap weld
  if (s->ee != 0 && s->ee != 1) return fail("model: ee must be 0 or 1");
  d->ee = s->ee;
  {
    double q[4], R[9];
    normq(s->weld_quat2, q);
    quat2mat(q, R);
    for (int k = 0; k < 9; k++) d->weld_mat2[k] = (float)R[k];
    for (int k = 0; k < 3; k++) d->weld_pos2[k] = (float)s->weld_pos2[k];
    for (int k = 0; k < 5; k++) d->weld_solimp[k] = (float)s->weld_solimp[k];
    solref_kb(s->weld_solref, s->weld_solimp, s->timestep, &K, &B);
    d->weld_K = (float)K;
    d->weld_B = (float)B;
    d->weld_ts = (float)s->weld_torquescale;
    for (int k = 0; k < 2; k++) d->weld_invw[k] = (float)s->weld_invweight0[k];
    for (int k = 0; k < 3; k++) d->mocap0[k] = (float)s->mocap_pos0[k];
    normq(s->mocap_quat0, q);
    for (int k = 0; k < 4; k++) d->mocap0[3 + k] = (float)q[k];
    if (s->ee && !(s->weld_invweight0[0] > 0 && s->weld_invweight0[1] > 0 && s->weld_solimp[2] > 0))
      return fail("model: weld parameters");
  }
  return 0;
}
}  // namespace

// Every exported entry point runs its implementation inside try / catch: host-side allocations (std::vector, new)
// can throw std::bad_alloc, and no C++ exception may cross the C-ABI (include/so100.h).  The error becomes status
// -3 (NULL for so100_create) with the message in so100_last_error().
static int caught(const char* where) {
  try {
    throw;
  } catch (const std::bad_alloc&) {
    snprintf(g_err, sizeof(g_err), "%s: out of host memory", where);
  } catch (const std::exception& e) {
    snprintf(g_err, sizeof(g_err), "%s: %s", where, e.what());
  } catch (...) {
    snprintf(g_err, sizeof(g_err), "%s: unknown C++ exception", where);
  }
  return -3;
}


static int so100_abi_version_impl(void) { return SO100_ABI_VERSION; }
static const char* so100_last_error_impl(void) { return g_err; }

// ---- support-direction cells of the hulls (so100_hull_cells, include/so100.h).  For each cube-map cell
// (face f: axis f / 2, sign f % 2; cell (cu, cv) of u = n_a / |n_axis|, v = n_b / |n_axis|, a < b the other
// axes) the candidates are the vertices not beaten over the whole cell by one vertex of a sample support set
// S by >= kCellMargin: (v_j - v_i) . d is affine in (u, v), so its minimum over the (widened) cell is at a
// corner.  A vertex that is the support for some direction of the cell, or within kCellMargin of it, is never
// left out, so fp32 scans of the list and of the hull agree (the fp32 winner is within rounding, << the
// margin, of the exact maximum).  Deterministic: a function of the model only.
static constexpr double kCellWiden = 1e-3, kCellMargin = 1e-6;
static void hull_cells_build(const so100_model* s, std::vector<uint32_t>& cells, std::vector<float>& cand) {
  constexpr int G = SO100_HULL_CELLG;
  cells.assign((size_t)SO100_NHULL_ALL * SO100_HULL_NCELL, 0u);
  cand.clear();
  std::vector<double> V, P;
  std::vector<int> S;
  for (int k = 0; k < SO100_NHULL_ALL; k++) {
    const int n = s->hull_count[k], s0 = s->hull_start[k];
    V.resize(3 * (size_t)n);
    for (int i = 0; i < n; i++)
      for (int t = 0; t < 3; t++) V[3 * i + t] = (double)(float)s->hull_vert[s0 + i][t];   // the device's values
    P.resize(4 * (size_t)n);
    for (int f = 0; f < 6; f++) {
      const int ax = f / 2, a = ax == 0 ? 1 : 0, b = ax == 2 ? 1 : 2;
      const double sg = (f & 1) ? -1.0 : 1.0;
      for (int cu = 0; cu < G; cu++)
        for (int cv = 0; cv < G; cv++) {
          const double u0 = -1.0 + 2.0 * cu / G - kCellWiden, u1 = -1.0 + 2.0 * (cu + 1) / G + kCellWiden;
          const double v0 = -1.0 + 2.0 * cv / G - kCellWiden, v1 = -1.0 + 2.0 * (cv + 1) / G + kCellWiden;
          auto score = [&](int i, double u, double v) { return sg * V[3 * i + ax] + u * V[3 * i + a] + v * V[3 * i + b]; };
          // sample supports (first maximal vertex) on a 7 x 7 grid of the widened cell
          S.clear();
          for (int su = 0; su < 7; su++)
            for (int sv = 0; sv < 7; sv++) {
              const double u = u0 + (u1 - u0) * su / 6.0, v = v0 + (v1 - v0) * sv / 6.0;
              int bi = 0;
              double bs = score(0, u, v);
              for (int i = 1; i < n; i++) {
                const double sc = score(i, u, v);
                if (sc > bs) { bs = sc; bi = i; }
              }
              if (std::find(S.begin(), S.end(), bi) == S.end()) S.push_back(bi);
            }
          const double cu4[4] = {u0, u0, u1, u1}, cv4[4] = {v0, v1, v0, v1};
          for (int i = 0; i < n; i++)
            for (int c = 0; c < 4; c++) P[4 * i + c] = score(i, cu4[c], cv4[c]);
          const size_t start = cand.size() / 4;
          int cnt = 0;
          for (int i = 0; i < n; i++) {
            bool beaten = false;
            for (int j : S) {
              if (j == i) continue;
              double mn = P[4 * j] - P[4 * i];
              for (int c = 1; c < 4; c++) mn = std::min(mn, P[4 * j + c] - P[4 * i + c]);
              if (mn >= kCellMargin) { beaten = true; break; }
            }
            if (beaten) continue;
            float w;
            std::memcpy(&w, &i, sizeof(w));
            cand.insert(cand.end(), {(float)V[3 * i], (float)V[3 * i + 1], (float)V[3 * i + 2], w});
            cnt++;
          }
          uint32_t& e = cells[(size_t)k * SO100_HULL_NCELL + (size_t)(f * G + cu) * G + cv];
          if (cnt > 255 || start > 0xFFFFFFu) {
            cand.resize(start * 4);          // too many for the 8-bit count: the kernel scans the whole hull
            e = 0u;
          } else {
            e = (uint32_t)start << 8 | (uint32_t)cnt;
          }
        }
    }
  }
}

static int so100_hull_cells_impl(const so100_model* model, uint32_t* cells, float* cand, int cap) {
  if (!model) return fail("so100_hull_cells: model is NULL");
  for (int k = 0; k < SO100_NHULL_ALL; k++)
    if (model->hull_start[k] < 0 || model->hull_count[k] < 1 || model->hull_start[k] + model->hull_count[k] > SO100_HULL_NVERT)
      return fail("so100_hull_cells: hull vertex range");
  std::vector<uint32_t> c;
  std::vector<float> v;
  hull_cells_build(model, c, v);
  const int nc = (int)(v.size() / 4);
  if (cells) std::memcpy(cells, c.data(), c.size() * sizeof(uint32_t));
  if (cand) {
    if (cap < nc) return fail("so100_hull_cells: cap too small");
    std::memcpy(cand, v.data(), v.size() * sizeof(float));
  }
  return nc;
}

static int so100_struct_sizes_impl(int* model_bytes, int* buffers_bytes) {
  if (model_bytes) *model_bytes = (int)sizeof(so100_model);
  if (buffers_bytes) *buffers_bytes = (int)sizeof(so100_buffers);
  return 0;
}

static so100_env* so100_create_impl(const so100_model* model, int n_envs, int device) {
  if (!model) { fail("so100_create: model is NULL"); return nullptr; }
  if (n_envs <= 0) { fail("so100_create: n_envs must be > 0"); return nullptr; }
  // the model check first: host-only, so a malformed model fails the same way with or without a device
  DevModel h;
  if (build_device_model(model, &h) != 0) return nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0) { fail_hip("so100_create: no HIP device", e == hipSuccess ? hipErrorNoDevice : e); return nullptr; }
  if (device < 0 || device >= ndev) { fail("so100_create: device index out of range"); return nullptr; }
  DeviceGuard g(device);
  // the hulls' support cells: the table in the model, the candidates in their own buffer
  std::vector<uint32_t> hc;
  std::vector<float> hv;
  hull_cells_build(model, hc, hv);
  std::memcpy(h.hull_cells, hc.data(), sizeof(h.hull_cells));
  // the candidate lists, then each cell's list as a fixed block of kCellBlk (padded with its last candidate;
  // longer lists keep the list path), in one buffer
  const size_t nlist = hv.size() / 4, ncell = hc.size();
  std::vector<float> all(hv);
  all.resize(4 * (nlist + ncell * so100::kCellBlk), 0.f);
  for (size_t c = 0; c < ncell; c++) {
    const uint32_t cnt = hc[c] & 255u, start = hc[c] >> 8;
    for (int i = 0; i < so100::kCellBlk && cnt > 0; i++) {
      const size_t src = start + std::min<uint32_t>((uint32_t)i, cnt - 1u);
      std::memcpy(&all[4 * (nlist + c * so100::kCellBlk + i)], &hv[4 * src], 4 * sizeof(float));
    }
  }
  float4* dcand = nullptr;
  e = hipMalloc(&dcand, all.size() * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(dcand, all.data(), all.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) { if (dcand) (void)hipFree(dcand); fail_hip("so100_create: hull cells", e); return nullptr; }
  h.hull_cand = reinterpret_cast<const so100::float4_t*>(dcand);
  h.hull_blk = reinterpret_cast<const so100::float4_t*>(dcand) + nlist;
  DevModel* dm = nullptr;
  e = hipMalloc(&dm, sizeof(DevModel));
  if (e != hipSuccess) { (void)hipFree(dcand); fail_hip("so100_create: hipMalloc", e); return nullptr; }
  e = hipMemcpy(dm, &h, sizeof(DevModel), hipMemcpyHostToDevice);
  if (e != hipSuccess) { (void)hipFree(dm); (void)hipFree(dcand); fail_hip("so100_create: hipMemcpy", e); return nullptr; }
  so100_env* env = new so100_env{device, n_envs, dm, h.nsubstep, h.solver, -1, kFusedAutoMax, {}, false, {}, nullptr, SO100_TASK_CUBE_TO_BIN, 700, 0, 0, {}, 0, 0};
  env->d_cand = dcand;
  if (const char* v = getenv("SO100_GRAPH")) env->use_graph = atoi(v) != 0;
  if (const char* v = getenv("SO100_FUSED")) env->fused = atoi(v) < 0 ? -1 : atoi(v) != 0;   // A/B: 0 split, 1 fused
  if (const char* v = getenv("SO100_FUSED_MAX")) env->fused_max = atoi(v);
  if (const char* v = getenv("SO100_FUSED_WAVES")) {
    const int w = atoi(v);
    env->fused_waves = (w == 2 || w == 3) ? w : 0;
  }
  // the split path's per-chunk workspaces (solver records) are allocated when the split path is first used
  // (here for PGS or a split default; else by so100_set_step_mode): each holds every env's whole contact list
  if (!step_is_fused(env)) e = make_chunks(env, default_chunks(n_envs));
  if (e == hipSuccess && env->solver == SO100_SOLVER_NEWTON) {
    // the fused launches: the record header (only its contact counts are written), the wave order, and the
    // contact record of the contacts beyond the kMaxCon held on chip
    e = so100::alloc_fused_workspace(n_envs, &env->fws);
  }
  if (e != hipSuccess) {
    (void)free_chunks(env);
    (void)hipFree(dm);
    (void)hipFree(dcand);
    delete env;
    fail_hip("so100_create: workspace", e);
    return nullptr;
  }
  return env;
}

static int so100_destroy_impl(so100_env* env) {
  if (!env) return 0;
  DeviceGuard g(env->device);
  profile_free(env);
  graph_free(env);
  if (env->cap_s) (void)hipStreamDestroy(env->cap_s);
  if (env->r_tri) (void)hipFree(env->r_tri);
  if (env->r_body) (void)hipFree(env->r_body);
  if (env->r_rgb) (void)hipFree(env->r_rgb);
  hipError_t e = hipFree(env->d_model);
  if (env->d_cand) (void)hipFree(env->d_cand);
  hipError_t e2 = free_chunks(env);
  if (e == hipSuccess) e = e2;
  if (e == hipSuccess) e = so100::free_workspace(&env->fws);
  else (void)so100::free_workspace(&env->fws);
  delete env;
  return e == hipSuccess ? 0 : fail_hip("so100_destroy", e);
}

static int so100_num_envs_impl(const so100_env* env) { return env ? env->n : -1; }

static int so100_configure_impl(so100_env* env, int task, int max_episode_steps, uint64_t base_seed, int env_offset) {
  if (!env) return fail("so100_configure: env is NULL");
  if (task < SO100_TASK_CUBE_TO_BIN || task > SO100_TASK_GOAL) return fail("so100_configure: unknown task");
  env->task = task;
  env->max_steps = max_episode_steps;
  env->base_seed = base_seed;
  if (env_offset < 0) return fail("so100_configure: env_offset < 0");
  env->env_offset = env_offset;
  graph_free(env);                           // kernel arguments changed
  return 0;
}

static int check_state(const so100_buffers* b) {
  if (!b) return fail("buffers is NULL");
  if (!b->qpos || !b->qvel || !b->qacc_warmstart) return fail("qpos/qvel/qacc_warmstart are required");
  return 0;
}

static int so100_reset_impl(so100_env* env, const so100_buffers* b, const uint8_t* mask, const uint32_t* seeds, void* stream) {
  if (!env) return fail("so100_reset: env is NULL");
  if (check_state(b)) return -1;
  if (env->task == SO100_TASK_GOAL && !b->desired_goal) return fail("so100_reset: GoalEnv needs desired_goal");
  DeviceGuard g(env->device);
  hipError_t e = so100::launch_reset(env->d_model, *b, env->n, env->task, env->base_seed, env->env_offset, mask, seeds,
                                     (hipStream_t)stream);
  return e == hipSuccess ? 0 : fail_hip("so100_reset", e);
}

// The launches of one env step on stream s: chunk 0 on s, chunks 1.. on their own streams forked from s
// and joined back to it.  The profiling events (if any) ride on chunk 0.
static hipError_t enqueue_step(so100_env* env, const so100_buffers* b, int flags, hipStream_t s, hipEvent_t* ev) {
  env->last_fused = step_is_fused(env);
  if (env->last_fused) {
    // one launch over all n envs (every wave runs its whole env step: no chunks needed to fill the gaps)
    return so100::launch_step(env->d_model, env->nsubstep, env->solver, 1, env->fused_waves, env->fws, *b, env->n, env->task, flags,
                              env->max_steps, env->base_seed, env->env_offset, s, ev);
  }
  if (env->chunks.empty()) return hipErrorNotReady;      // (so100_set_step_mode allocates them)
  if (env->chunks.size() == 1) {
    Chunk& c = env->chunks[0];
    return so100::launch_step(env->d_model, env->nsubstep, env->solver, 0, 0, c.ws, *b, c.count, env->task, flags, env->max_steps,
                              env->base_seed, env->env_offset, s, ev);
  }
  hipError_t e = hipEventRecord(env->fork, s);
  for (size_t k = 1; k < env->chunks.size() && e == hipSuccess; k++) {
    Chunk& c = env->chunks[k];
    e = hipStreamWaitEvent(c.s, env->fork, 0);
    if (e == hipSuccess)
      e = so100::launch_step(env->d_model, env->nsubstep, env->solver, 0, 0, c.ws, offset_buffers(*b, c.start), c.count, env->task, flags,
                             env->max_steps, env->base_seed, env->env_offset + c.start, c.s, nullptr);
    if (e == hipSuccess) e = hipEventRecord(c.done, c.s);
  }
  Chunk& c0 = env->chunks[0];
  if (e == hipSuccess)
    e = so100::launch_step(env->d_model, env->nsubstep, env->solver, 0, 0, c0.ws, *b, c0.count, env->task, flags, env->max_steps,
                           env->base_seed, env->env_offset, s, ev);
  for (size_t k = 1; k < env->chunks.size() && e == hipSuccess; k++) e = hipStreamWaitEvent(s, env->chunks[k].done, 0);
  return e;
}

// Capture the step for (b, flags) on the private capture stream and instantiate it into g.
// the split path's substep-counter parity (its PGS heavy-group lists alternate by it); the fused step has none
static uint32_t step_parity(const so100_env* env) {
  return (step_is_fused(env) || env->chunks.empty()) ? 0u : env->chunks[0].ws.sub_count & 1u;
}

static hipError_t build_step_graph(so100_env* env, const so100_buffers* b, int flags, StepGraph& g) {
  const uint32_t par = step_parity(env);
  hipError_t e = hipSuccess;
  if (!env->cap_s) e = hipStreamCreateWithFlags(&env->cap_s, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&g.done, hipEventDisableTiming);
  if (e != hipSuccess) return e;
  e = hipStreamBeginCapture(env->cap_s, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) return e;
  hipError_t el = enqueue_step(env, b, flags, env->cap_s, nullptr);
  hipGraph_t graph = nullptr;
  e = hipStreamEndCapture(env->cap_s, &graph);
  if (el != hipSuccess) e = el;
  if (e == hipSuccess) e = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
  if (graph) (void)hipGraphDestroy(graph);
  if (e != hipSuccess) { g.exec = nullptr; return e; }
  g.buf = *b;
  g.flags = flags;
  g.par = par;
  return hipSuccess;
}

// Replay the step graph for (b, flags) on s, capturing it first if it is not cached.
static hipError_t graph_step(so100_env* env, const so100_buffers* b, int flags, hipStream_t s) {
  const uint32_t par = step_parity(env);
  StepGraph* hit = nullptr;
  for (StepGraph& g : env->graphs)
    if (g.flags == flags && g.par == par && memcmp(&g.buf, b, sizeof(so100_buffers)) == 0) { hit = &g; break; }
  hipError_t e = hipSuccess;
  if (hit) {
    // the capture advanced the host substep counters as an eager step would; a replay does it here
    for (Chunk& c : env->chunks) c.ws.sub_count += (uint32_t)env->nsubstep;
  } else {
    if (env->graphs.size() >= kMaxStepGraphs) {
      size_t lru = 0;
      for (size_t i = 1; i < env->graphs.size(); i++)
        if (env->graphs[i].last_use < env->graphs[lru].last_use) lru = i;
      graph_destroy(env->graphs[lru]);
      env->graphs.erase(env->graphs.begin() + (long)lru);
    }
    StepGraph g;
    e = build_step_graph(env, b, flags, g);
    if (e != hipSuccess) { graph_destroy(g); return e; }
    env->graphs.push_back(g);
    hit = &env->graphs.back();
  }
  hit->last_use = ++env->graph_clock;
  e = hipGraphLaunch(hit->exec, s);
  if (e == hipSuccess) e = hipEventRecord(hit->done, s);
  return e;
}

static int so100_step_impl(so100_env* env, const so100_buffers* b, int flags, void* stream) {
  if (!env) return fail("so100_step: env is NULL");
  if (check_state(b)) return -1;
  if (!b->action) return fail("so100_step: action is NULL");
  if (env->task == SO100_TASK_GOAL && !b->desired_goal) return fail("so100_step: GoalEnv needs desired_goal");
  if ((flags & SO100_FLAG_DR) && !b->dr_params) return fail("so100_step: FLAG_DR needs dr_params");
  if ((flags & SO100_FLAG_AUTORESET) && !b->episode) return fail("so100_step: FLAG_AUTORESET needs episode");
  DeviceGuard g(env->device);
  hipEvent_t* ev = nullptr;
  if (env->prof_used < env->prof_cap) ev = env->prof_ev.data() + (size_t)(env->prof_used++) * env->prof_per;
  const hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (env->use_graph && !ev) {
    e = graph_step(env, b, flags, s);
  } else {
    e = enqueue_step(env, b, flags, s, ev);
  }
  return e == hipSuccess ? 0 : fail_hip("so100_step", e);
}

static int so100_profile_enable_impl(so100_env* env, int max_steps) {
  if (!env) return fail("so100_profile_enable: env is NULL");
  if (max_steps < 0) return fail("so100_profile_enable: max_steps < 0");
  DeviceGuard g(env->device);
  profile_free(env);
  env->prof_per = step_is_fused(env) ? 2 : 2 * env->nsubstep + 2;
  const size_t count = (size_t)max_steps * env->prof_per;
  env->prof_ev.resize(count);
  for (size_t i = 0; i < count; i++) {
    hipError_t e = hipEventCreate(&env->prof_ev[i]);
    if (e != hipSuccess) { env->prof_ev.resize(i); profile_free(env); return fail_hip("so100_profile_enable", e); }
  }
  env->prof_cap = max_steps;
  return 0;
}

static int so100_profile_read_impl(so100_env* env, double* solver_ms, int* solver_launches, double* stage_ms, int* stage_launches) {
  if (!env || !solver_ms || !solver_launches || !stage_ms || !stage_launches) return fail("so100_profile_read: bad arguments");
  DeviceGuard g(env->device);
  *solver_ms = *stage_ms = 0.0;
  *solver_launches = *stage_launches = 0;
  const int per = env->prof_per;
  if (env->prof_used > 0) {
    hipError_t e = hipEventSynchronize(env->prof_ev[(size_t)env->prof_used * per - 1]);
    if (e != hipSuccess) return fail_hip("so100_profile_read", e);
  }
  for (int st = 0; st < env->prof_used; st++) {
    const hipEvent_t* ev = env->prof_ev.data() + (size_t)st * per;
    if (per == 2) {                        // fused: the one launch contains the solves
      float ms = 0.f;
      hipError_t e = hipEventElapsedTime(&ms, ev[0], ev[1]);
      if (e != hipSuccess) return fail_hip("so100_profile_read", e);
      *solver_ms += ms;
      (*solver_launches)++;
      continue;
    }
    for (int k = 0; k + 1 < per; k++) {   // launch order: stage, solver, stage, solver, ..., final stage
      float ms = 0.f;
      hipError_t e = hipEventElapsedTime(&ms, ev[k], ev[k + 1]);
      if (e != hipSuccess) return fail_hip("so100_profile_read", e);
      if (k & 1) { *solver_ms += ms; (*solver_launches)++; }
      else { *stage_ms += ms; (*stage_launches)++; }
    }
  }
  return 0;
}

static int so100_set_step_mode_impl(so100_env* env, int fused) {
  if (!env) return fail("so100_set_step_mode: env is NULL");
  if (fused < -1 || fused > 1) return fail("so100_set_step_mode: mode must be -1 (auto), 0 (split) or 1 (fused)");
  if (env->prof_cap > 0) return fail("so100_set_step_mode: disable profiling first");
  DeviceGuard g(env->device);
  graph_free(env);                     // captured graphs hold the other mode's launches
  const int prev = env->fused;
  env->fused = fused;
  if (!step_is_fused(env) && env->chunks.empty()) {
    // first use of the split path: its chunk workspaces (one synchronising allocation, here, never in a step)
    hipError_t e = make_chunks(env, default_chunks(env->n));
    if (e != hipSuccess) {
      (void)free_chunks(env);
      env->fused = prev;
      return fail_hip("so100_set_step_mode: split workspace", e);
    }
  }
  return 0;
}

static int so100_step_mode_impl(const so100_env* env) {
  if (!env) return fail("so100_step_mode: env is NULL");
  return step_is_fused(env) ? 1 : 0;
}

static int so100_set_fused_build_impl(so100_env* env, int waves) {
  if (!env) return fail("so100_set_fused_build: env is NULL");
  if (waves != 0 && waves != 2 && waves != 3) return fail("so100_set_fused_build: waves must be 0 (auto), 2 or 3");
  if (env->prof_cap > 0) return fail("so100_set_fused_build: disable profiling first");
  DeviceGuard g(env->device);
  graph_free(env);                     // captured graphs hold the other build's launch
  env->fused_waves = waves;
  return 0;
}

static int so100_fused_build_impl(const so100_env* env, int debug) {
  if (!env) return fail("so100_fused_build: env is NULL");
  DeviceGuard g(env->device);
  return so100::fused_build(env->n, env->fused_waves, debug != 0);
}

static int so100_chunk_info_impl(const so100_env* env, int* nchunks, int* profiled_envs) {
  if (!env) return fail("so100_chunk_info: env is NULL");
  if (nchunks) *nchunks = (int)env->chunks.size();
  if (step_is_fused(env)) {     // one launch over all envs
    if (nchunks) *nchunks = 1;
    if (profiled_envs) *profiled_envs = env->n;
    return 0;
  }
  if (nchunks && env->chunks.empty()) *nchunks = default_chunks(env->n);
  if (profiled_envs) *profiled_envs = env->chunks.empty() ? 0 : env->chunks[0].count;
  return 0;
}

static int so100_contact_count_impl(so100_env* env, uint64_t* accum, void* stream) {
  if (!env || !accum) return fail("so100_contact_count: bad arguments");
  DeviceGuard g(env->device);
  hipError_t e = hipSuccess;
  if (env->last_fused) {
    if (env->fws.hdr) e = so100::launch_contact_count(env->fws, env->n, accum, (hipStream_t)stream);
  } else {
    for (const Chunk& c : env->chunks)
      if (e == hipSuccess) e = so100::launch_contact_count(c.ws, c.count, accum, (hipStream_t)stream);
  }
  return e == hipSuccess ? 0 : fail_hip("so100_contact_count", e);
}

static int so100_contact_counts_impl(so100_env* env, int32_t* out, void* stream) {
  if (!env || !out) return fail("so100_contact_counts: bad arguments");
  DeviceGuard g(env->device);
  hipError_t e = hipSuccess;
  if (env->last_fused) {
    if (env->fws.hdr) e = so100::launch_contact_counts(env->fws, env->n, out, (hipStream_t)stream);
  } else {
    for (const Chunk& c : env->chunks)
      if (e == hipSuccess) e = so100::launch_contact_counts(c.ws, c.count, out + c.start, (hipStream_t)stream);
  }
  return e == hipSuccess ? 0 : fail_hip("so100_contact_counts", e);
}

static int so100_pool_stats_impl(so100_env* env, uint64_t* out, int reset) {
  if (!env || !out) return fail("so100_pool_stats: bad arguments");
  DeviceGuard g(env->device);
  unsigned long long st[2] = {0, 0};
  hipError_t e = hipSuccess;
  if (env->fws.pool_stat) {
    e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(st, env->fws.pool_stat, sizeof(st), hipMemcpyDeviceToHost);
    if (e == hipSuccess && reset) e = hipMemset(env->fws.pool_stat, 0, sizeof(st));
  }
  if (e != hipSuccess) return fail_hip("so100_pool_stats", e);
  out[0] = st[0];
  out[1] = st[1];
  out[2] = (uint64_t)env->fws.pool_recs;
  return 0;
}

static int so100_goal_reward_impl(so100_env* env, int n, const float* a, const float* d, float* out, void* stream) {
  if (!env || !a || !d || !out || n < 0) return fail("so100_goal_reward: bad arguments");
  if (n == 0) return 0;
  DeviceGuard g(env->device);
  hipError_t e = so100::launch_goal_reward(env->d_model, n, a, d, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : fail_hip("so100_goal_reward", e);
}

static int so100_eval_reward_impl(so100_env* env, int task, int n, const float* cube, const float* ee, const uint32_t* bits,
                      float* out, void* stream) {
  if (!env || !cube || !ee || !bits || !out || n < 0) return fail("so100_eval_reward: bad arguments");
  if (task < SO100_TASK_CUBE_TO_BIN || task > SO100_TASK_GOAL) return fail("so100_eval_reward: unknown task");
  if (n == 0) return 0;
  DeviceGuard g(env->device);
  hipError_t e = so100::launch_reward(env->d_model, task, n, cube, ee, bits, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : fail_hip("so100_eval_reward", e);
}

static int so100_spawn_pose_impl(so100_env* env, int n, const uint32_t* seeds, double* pose, void* stream) {
  if (!env || !seeds || !pose || n < 0) return fail("so100_spawn_pose: bad arguments");
  if (n == 0) return 0;
  DeviceGuard g(env->device);
  hipError_t e = so100::launch_spawn(env->d_model, n, seeds, pose, (hipStream_t)stream);
  return e == hipSuccess ? 0 : fail_hip("so100_spawn_pose", e);
}

static int so100_unnormalize_impl(so100_env* env, int n, const float* action, float* ctrl, void* stream) {
  if (!env || !action || !ctrl || n < 0) return fail("so100_unnormalize: bad arguments");
  if (n == 0) return 0;
  DeviceGuard g(env->device);
  hipError_t e = so100::launch_unnormalize(env->d_model, n, action, ctrl, (hipStream_t)stream);
  return e == hipSuccess ? 0 : fail_hip("so100_unnormalize", e);
}


static int so100_render_mesh_impl(so100_env* env, const float* tri, const int* body, const float* rgb, int ntri) {
  if (!env || !tri || !body || !rgb || ntri <= 0) return fail("so100_render_mesh: bad arguments");
  std::vector<float4> t((size_t)ntri * 3);
  std::vector<uint32_t> c((size_t)ntri);
  for (int i = 0; i < ntri; i++) {
    if (body[i] < 0 || body[i] >= SO100_NBODY) return fail("so100_render_mesh: body out of range");
    for (int v = 0; v < 3; v++) {
      const float* p = tri + (size_t)9 * i + 3 * v;
      t[(size_t)3 * i + v] = make_float4(p[0], p[1], p[2], 0.f);
    }
    uint32_t col = 0;
    for (int k = 0; k < 3; k++) {
      const float x = rgb[(size_t)3 * i + k] < 0.f ? 0.f : (rgb[(size_t)3 * i + k] > 1.f ? 1.f : rgb[(size_t)3 * i + k]);
      col |= (uint32_t)(x * 255.f + 0.5f) << (8 * k);
    }
    c[i] = col;
  }
  DeviceGuard g(env->device);
  if (env->r_tri) (void)hipFree(env->r_tri);
  if (env->r_body) (void)hipFree(env->r_body);
  if (env->r_rgb) (void)hipFree(env->r_rgb);
  env->r_tri = nullptr; env->r_body = nullptr; env->r_rgb = nullptr; env->r_ntri = 0;
  hipError_t e = hipMalloc(&env->r_tri, t.size() * sizeof(float4));
  if (e == hipSuccess) e = hipMalloc(&env->r_body, (size_t)ntri * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&env->r_rgb, (size_t)ntri * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemcpy(env->r_tri, t.data(), t.size() * sizeof(float4), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(env->r_body, body, (size_t)ntri * sizeof(int), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(env->r_rgb, c.data(), (size_t)ntri * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail_hip("so100_render_mesh", e);
  env->r_ntri = ntri;
  return 0;
}

static int so100_render_impl(so100_env* env, const float* qpos, const uint8_t* mask, const so100_camera* cam, int width,
                 int height, uint8_t* out, void* stream) {
  if (!env || !qpos || !cam || !out) return fail("so100_render: bad arguments");
  if (env->r_ntri <= 0) return fail("so100_render: no render mesh (so100_render_mesh)");
  if (width <= 0 || height <= 0 || width > 4096 || (long)width * height > (1L << 22))
    return fail("so100_render: bad image size (width <= 4096, width*height <= 2^22)");
  if (cam->nlight < 0 || cam->nlight > SO100_MAX_LIGHTS || !(cam->fovy > 0.f && cam->fovy < 180.f))
    return fail("so100_render: bad camera");
  DeviceGuard g(env->device);
  hipError_t e = so100::launch_render(env->d_model, env->r_tri, env->r_body, env->r_rgb, env->r_ntri, qpos, mask, *cam,
                                      env->n, width, height, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : fail_hip("so100_render", e);
}


extern "C" {

int so100_abi_version(void) {
  try {
    return so100_abi_version_impl();
  } catch (...) {
    return caught("so100_abi_version");
  }
}

const char* so100_last_error(void) { return so100_last_error_impl(); }

#ifndef SO100_SRC_HASH
#define SO100_SRC_HASH "unknown"
#endif
// the Makefile's content hash of the sources this library was built from (ABI 16)
const char* so100_source_hash(void) { return SO100_SRC_HASH; }

int so100_hull_cells(const so100_model* model, uint32_t* cells, float* cand, int cap) {
  try {
    return so100_hull_cells_impl(model, cells, cand, cap);
  } catch (...) {
    return caught("so100_hull_cells");
  }
}

int so100_struct_sizes(int* model_bytes, int* buffers_bytes) {
  try {
    return so100_struct_sizes_impl(model_bytes, buffers_bytes);
  } catch (...) {
    return caught("so100_struct_sizes");
  }
}

so100_env* so100_create(const so100_model* model, int n_envs, int device) {
  try {
    return so100_create_impl(model, n_envs, device);
  } catch (...) {
    caught("so100_create");
    return nullptr;
  }
}

int so100_destroy(so100_env* env) {
  try {
    return so100_destroy_impl(env);
  } catch (...) {
    return caught("so100_destroy");
  }
}

int so100_num_envs(const so100_env* env) {
  try {
    return so100_num_envs_impl(env);
  } catch (...) {
    return caught("so100_num_envs");
  }
}

int so100_configure(so100_env* env, int task, int max_episode_steps, uint64_t base_seed, int env_offset) {
  try {
    return so100_configure_impl(env, task, max_episode_steps, base_seed, env_offset);
  } catch (...) {
    return caught("so100_configure");
  }
}

int so100_reset(so100_env* env, const so100_buffers* b, const uint8_t* mask, const uint32_t* seeds, void* stream) {
  try {
    return so100_reset_impl(env, b, mask, seeds, stream);
  } catch (...) {
    return caught("so100_reset");
  }
}

int so100_step(so100_env* env, const so100_buffers* b, int flags, void* stream) {
  try {
    return so100_step_impl(env, b, flags, stream);
  } catch (...) {
    return caught("so100_step");
  }
}

int so100_profile_enable(so100_env* env, int max_steps) {
  try {
    return so100_profile_enable_impl(env, max_steps);
  } catch (...) {
    return caught("so100_profile_enable");
  }
}

int so100_profile_read(so100_env* env, double* solver_ms, int* solver_launches, double* stage_ms, int* stage_launches) {
  try {
    return so100_profile_read_impl(env, solver_ms, solver_launches, stage_ms, stage_launches);
  } catch (...) {
    return caught("so100_profile_read");
  }
}

int so100_set_step_mode(so100_env* env, int fused) {
  try {
    return so100_set_step_mode_impl(env, fused);
  } catch (...) {
    return caught("so100_set_step_mode");
  }
}

int so100_step_mode(const so100_env* env) {
  try {
    return so100_step_mode_impl(env);
  } catch (...) {
    return caught("so100_step_mode");
  }
}

int so100_set_fused_build(so100_env* env, int waves) {
  try {
    return so100_set_fused_build_impl(env, waves);
  } catch (...) {
    return caught("so100_set_fused_build");
  }
}

int so100_fused_build(const so100_env* env, int debug) {
  try {
    return so100_fused_build_impl(env, debug);
  } catch (...) {
    return caught("so100_fused_build");
  }
}

int so100_chunk_info(const so100_env* env, int* nchunks, int* profiled_envs) {
  try {
    return so100_chunk_info_impl(env, nchunks, profiled_envs);
  } catch (...) {
    return caught("so100_chunk_info");
  }
}

int so100_contact_count(so100_env* env, uint64_t* accum, void* stream) {
  try {
    return so100_contact_count_impl(env, accum, stream);
  } catch (...) {
    return caught("so100_contact_count");
  }
}

int so100_pool_stats(so100_env* env, uint64_t* out, int reset) {
  try {
    return so100_pool_stats_impl(env, out, reset);
  } catch (...) {
    return caught("so100_pool_stats");
  }
}

int so100_contact_counts(so100_env* env, int32_t* out, void* stream) {
  try {
    return so100_contact_counts_impl(env, out, stream);
  } catch (...) {
    return caught("so100_contact_counts");
  }
}

int so100_goal_reward(so100_env* env, int n, const float* a, const float* d, float* out, void* stream) {
  try {
    return so100_goal_reward_impl(env, n, a, d, out, stream);
  } catch (...) {
    return caught("so100_goal_reward");
  }
}

int so100_eval_reward(so100_env* env, int task, int n, const float* cube, const float* ee, const uint32_t* bits,
                      float* out, void* stream) {
  try {
    return so100_eval_reward_impl(env, task, n, cube, ee, bits, out, stream);
  } catch (...) {
    return caught("so100_eval_reward");
  }
}

int so100_spawn_pose(so100_env* env, int n, const uint32_t* seeds, double* pose, void* stream) {
  try {
    return so100_spawn_pose_impl(env, n, seeds, pose, stream);
  } catch (...) {
    return caught("so100_spawn_pose");
  }
}

int so100_unnormalize(so100_env* env, int n, const float* action, float* ctrl, void* stream) {
  try {
    return so100_unnormalize_impl(env, n, action, ctrl, stream);
  } catch (...) {
    return caught("so100_unnormalize");
  }
}

int so100_render_mesh(so100_env* env, const float* tri, const int* body, const float* rgb, int ntri) {
  try {
    return so100_render_mesh_impl(env, tri, body, rgb, ntri);
  } catch (...) {
    return caught("so100_render_mesh");
  }
}

int so100_render(so100_env* env, const float* qpos, const uint8_t* mask, const so100_camera* cam, int width,
                 int height, uint8_t* out, void* stream) {
  try {
    return so100_render_impl(env, qpos, mask, cam, width, height, out, stream);
  } catch (...) {
    return caught("so100_render");
  }
}

}  // extern "C"
