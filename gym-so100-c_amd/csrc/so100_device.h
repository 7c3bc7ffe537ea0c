// so100_device.h — fp32 device copy of the model with host-side precomputation (internal).
#pragma once
#include <stdint.h>
#include "so100_model.h"

namespace so100 {

struct alignas(16) float4_t { float x, y, z, w; };   // host-visible float4 (the device reads it as float4)

constexpr int kLanes = 16;            // lanes per env ("env lane-group" = one DPP row)
constexpr int kEnvsPerBlock = 4;      // one wave64 per workgroup
constexpr int kThreads = kLanes * kEnvsPerBlock;
constexpr int kNArm = SO100_NHINGE;
constexpr int kMaxCon = SO100_MAXCON;     // contacts an env holds on chip (lane c of its row owns contact c)
constexpr int kConCap = SO100_NCON_MAX;   // the env's whole contact list: every pair at its collider's maximum

constexpr int kCellBlk = 16;   // candidates per support cell block (DevModel::hull_blk): one per lane of a row
struct DevModel {
  // options
  float timestep;
  int nsubstep;
  int iterations;
  int solver;                       // SO100_SOLVER_PGS | SO100_SOLVER_NEWTON
  int convex;                       // SO100_CONVEX_EPA | SO100_CONVEX_MPR (the mesh pairs' collider)
  float tolerance;
  float impratio;
  float gravity[3];
  float pgs_scale;                  // 1 / (meaninertia * nv)

  // arm chain: bodies 2..7 (index a = body-2), Base (body 1) is static
  float base_pos[3];
  float base_quat[4];
  float body_pos[6][3];
  float body_quat[6][4];
  float body_ipos[6][3];
  float body_imat[6][9];            // inertial frame rotation (from iquat) in the body frame
  float body_mass[6];
  float body_inertia[6][3];
  float jnt_axis[6][3];
  float jnt_lo[6], jnt_hi[6];
  float armature[6];

  // cube (free body, COM at the body origin, principal axes = body axes)
  float cube_mass;
  float cube_inertia[3];

  // frictionloss rows (pos = 0 -> imp = dmin, R constant)
  float fr_floss[12];
  float fr_R[12];
  float fr_B;                       // dof_solref -> B  (aref = -B * vel)

  // limit rows
  float lim_K, lim_B;
  float lim_solimp[5];
  float lim_invw[6];

  // actuators
  float act_kp[6], act_kv[6];
  float act_flo[6], act_fhi[6];
  float act_clo[6], act_chi[6];

  // geoms
  int geom_body[SO100_NGEOM];
  float geom_pos[SO100_NGEOM][3];   // body frame (world for static)
  float geom_mat[SO100_NGEOM][9];
  float geom_size[SO100_NGEOM][3];
  float geom_rbound[SO100_NGEOM];   // |half sizes| (box bounding sphere)
  float bin_lo[3], bin_hi[3];       // world AABB of the 5 bin boxes (pad-bin prefilter)
  float base_xmat[9], base_xpos[3]; // the static Base's world frame (the Base hull's frame, MPR)

  // pairs (0..13 box-box, 14..22 table-hull, 23..76 (cube | bin box, hull) through MPR)
  int pair_g1[SO100_NPAIR], pair_g2[SO100_NPAIR];
  int pair_b1[SO100_NPAIR], pair_b2[SO100_NPAIR];
  int pair_cond4[SO100_NPAIR];      // 1: condim 4 (torsion row), 0: condim 3 (J row 3 zero)
  int pair_arm[SO100_NPAIR];        // a body of the pair is an arm link: J has arm entries
  int pair_cube[SO100_NPAIR];       // the cube is in the pair: the DR friction scale applies
  float pair_K[SO100_NPAIR], pair_B[SO100_NPAIR];
  float pair_solimp[SO100_NPAIR][5];
  float pair_mu0[SO100_NPAIR], pair_mu1[SO100_NPAIR];
  float pair_margin[SO100_NPAIR];
  float pair_tran[SO100_NPAIR], pair_rot[SO100_NPAIR];   // diagApprox (body invweight sums)

  // arm/jaw collision hulls vs the table top (body-frame vertices and bounding box: center, half extents)
  int hull_body[SO100_NHULL_ALL], hull_start[SO100_NHULL_ALL], hull_count[SO100_NHULL_ALL];
  float4_t hull_center[SO100_NHULL_ALL], hull_half[SO100_NHULL_ALL];   // hull_half.w = |half extents|
  float4_t hull_centroid[SO100_NHULL_ALL];   // MPR portal centre (mesh volume centroid), body frame
  float4_t hull_vert[SO100_HULL_NVERT];
  // MPR support lookup (so100_hull_cells): hull k's cube-map cells at k * SO100_HULL_NCELL, start << 8 | count
  // into hull_cand (x, y, z, vertex index bits; count 0: scan the hull)
  uint32_t hull_cells[SO100_NHULL_ALL * SO100_HULL_NCELL];
  const float4_t* hull_cand;
  // the same lists as fixed blocks of kCellBlk per cell (cell c at c * kCellBlk; lists of <= kCellBlk padded
  // with their last candidate): a row loads its cell's candidates with one load issued beside the cell entry's
  const float4_t* hull_blk;
  float table_top, table_lo[2], table_hi[2];
  float table_bottom;               // the table box's bottom face (table_top - 2 x its half thickness)

  // sites
  float site_cube[3];               // cube body frame
  float site_ee[3];                 // Fixed_Jaw (body 6) frame
  float bin_center_f[3];

  // task (double: the reward runs in double exactly like the reference)
  double bin_center[3];
  double bin_hw, bin_h, cube_half;
  double goal_threshold;
  double max_reward;
  float start_qpos[6];
  float action_lo[6], action_hi[6], action_span[6];
  double spawn_lo[3], spawn_hi[3];
  float goal_bin_lo[3], goal_bin_hi[3];   // env.py:245-249

  // EE / mocap variant: weld of ee_site (Fixed_Jaw frame) to the mocap pose (so_arm100_ee.xml:171-173)
  int ee;
  float weld_pos2[3], weld_mat2[9];
  float weld_solimp[5];
  float weld_K, weld_B, weld_ts;
  float weld_invw[2];                     // tran, rot
  float mocap0[7];                        // default mocap pose (pos, quat)
};

// ------------------------------------------------------------------ substep workspace (HBM)
// The substep is split in two kernels: the stage kernel (16 lanes per env) assembles
// the constraint rows, the PGS kernel (4 lanes per env, 3 dofs per lane) solves them.  The hand-off
// is a per-env record in HBM, laid out for the solver's lanes:
//   hdr[env][q][kHdrLane]  lane q owns dofs 3q..3q+2 (q = 0,1: arm, q = 2,3: cube)
//   con[env][c][kConStride] for every contact c < kConCap: solver block (kBlk float4), J[dof][row] (12 x 4
//                           floats), then (contacts c >= kMaxCon only) the contact's geometry
// The fused step uses the same per-env contact record for the contacts beyond the kMaxCon it holds on chip.
constexpr int kHdrLane = 40;
constexpr int kHdrEnv = 4 * kHdrLane;
// Solver block of one contact, read by the PGS as kBlk x ds_read_b128 (float index: content):
//   0-9  A+R upper triangle 00 01 02 03 11 12 13 22 23 33     10-18  P = Q' D (row-major)
//   19-21 lam (eigenvalues of D A11 D = Q diag(lam) Q')       22-24  1 / lam
//   25 R0   26 1/(A+R)00   27 R1 (= R2)   28 R3   29 1 if a gripper-pad contact (J has arm entries) else 0
//   30-31 pad  32-35 aref   36-39 f (normal, t1, t2, torsion)
constexpr int kBlk = 10;
constexpr int kBlkFlags = 7;      // float4 slot holding R3 (x) and the arm flag (y)
constexpr int kBlkAref = 8;       // float4 slots
constexpr int kBlkF = 9;
constexpr int kJOff = 4 * kBlk;   // float offset of the J rows in the record
constexpr int kConRec = kJOff + 48;
// Contacts c >= kMaxCon (the rest of the list, which does not fit on chip): their geometry follows J in the
// record slot (ConGeom: pos + dist, frame; then the pair id as int bits and the dist), and the Newton solve
// keeps its per-contact state in the block's floats 12..23 (jar at the iterate, J s, force); the convex
// collider stages such contacts in floats 24..31 (dead from the compaction on)
constexpr int kGeoOff = kConRec;            // 16 floats: pos[4] (pos[3] = dist), frame[12]
constexpr int kGeoPair = kGeoOff + 16;      // pair index (int bits)
constexpr int kGeoDist = kGeoOff + 17;
constexpr int kConStride = kGeoOff + 24;    // 112 floats = 448 B per contact slot
constexpr int kOvfJc = 12, kOvfJs = 16, kOvfF = 20;   // Newton overflow state (floats of the block)
constexpr int kMprStageOff = 24;            // convex-collider staging (MprStage) of staged contacts >= kMaxCon
constexpr size_t kConEnv = (size_t)kConCap * kConStride;   // floats per env
// the convex pairs' separating-direction cache (so100_convex.h mpr_contacts): one float4 per (env, convex pair)
constexpr int kSepPairs = 140;   // >= the 138 convex items (120 wave-shared pairs, the EE marker's 9, the 9 table hulls)
enum HdrField : int {
  H_QACC = 0,       // qacc at the solver start (qacc_smooth, plus M^-1 J' f of the kept warmstart)
  H_FRAREF = 3,     // frictionloss rows: aref = -B vel
  H_FRF = 6,        //   warmstart force
  H_LIMS = 9,       // joint-limit rows (arm lanes): side +-1, 0 = inactive
  H_LIMAREF = 12,
  H_LIMR = 15,
  H_LIMF = 18,
  H_MROW = 21,      // 3 x 6: M^-1 rows of this lane's dofs, own 3 columns then the partner lane's 3
                    // (cube lanes: the diagonal inverse mass, partner columns 0)
  H_NCON = 39,      // contact count (int bits)
};
static_assert(H_NCON + 1 == kHdrLane && kHdrLane % 4 == 0 && kConRec % 4 == 0, "workspace record layout");
// Newton solver record (model.solver = SO100_SOLVER_NEWTON): the same buffers, one 160-float header per
// env (H_NCON kept at its PGS offset for the contact counter) and per contact the block
//   0-3 aref, 4-7 R (normal, t1, t2, torsion), 8 cone mu (= friction0 sqrt(R1/R0)), 9 friction0,
//   10 friction1 (torsion), then J at kJOff as for PGS.
enum NewtonHdr : int {
  N_QS = 0,         // qacc_smooth [12]
  N_WARM = 12,      // qacc_warmstart [12]
  N_FRAREF = 24,    // frictionloss rows: aref = -B vel [12]
  N_LIMS = 40,      // joint-limit rows: side +-1, 0 = inactive [6]
  N_LIMAREF = 46,   // [6]
  N_LIMR = 52,      // [6]
  N_M = 58,         // arm M (incl. armature), row-major 6x6
  N_MC = 94,        // cube diagonal masses (m, m, m, I0, I1, I2)
};
static_assert(N_FRAREF + 12 <= H_NCON && N_MC + 6 <= kHdrEnv, "Newton header layout");
constexpr int kPgsEnvs = 16;      // solver: envs per wave64 (4 lanes each) = one "group"
constexpr int kResident = 6;      // solver: contacts per env held on-chip across the sweeps (round 6: 4 -> 6, +1 %, profiles/r05_ab_pgs_resident.txt)
constexpr int kHeavyCap = 512;    // solver: groups with > kResident contacts dispatched first (cap)
struct Workspace {
  float* hdr;
  int hdr_stride;   // floats per env of hdr: kHdrEnv (the split path's record headers), 1 (the fused path: its counts)
  float* con;
  // heavy-group list, double-buffered by substep parity: the stage kernel flags/list groups holding an
  // env with more than kResident contacts, the solver dispatches those first and clears the other set
  uint32_t* gflag;  // [2][ngroups]  1 = listed, 3 = heavy but over the cap (solved in place)
  int* hcount;      // [2]
  int* hlist;       // [2][kHeavyCap]
  uint32_t sub_count;   // host-side substep counter (parity)
  // fused path (so100_fused_kernel): heavy-first wave order from the previous step's per-wave cost
  uint32_t* gcost;  // [ngroups] shader cycles of each 4-env wave in the last fused step
  int* order;       // [ngroups] launch order of the groups (so100_order_kernel), nullptr = natural
  // [n][kSepPairs] the direction that last proved a convex pair separated (w = 1) or w = 0: a certificate the next
  // substep re-checks with one support evaluation before it runs GJK (results unchanged: mpr_contacts)
  float4* sep;
  // fused path: the contact records of the envs whose list is longer than the kMaxCon held on chip (every contact
  // beyond them: geometry, J, the rows and the Newton solve's per-contact state; kConEnv floats each), a pool of
  // entries (a wave's kEnvsPerBlock records) per XCD with a free bitmap (pool_bm[xcd * kPoolWords ..]).  A wave takes
  // one for a substep when one of its envs' lists passes kMaxCon and returns it after the solve (so100_pool.h);
  // pool_recs entries per XCD: as many as the XCD can hold fused-kernel waves resident, so one is always free.
  // pool_stat [2]: entries taken (wave-substeps that held one) and scans that found none (0 by the sizing), summed
  // over steps (so100_pool_stats).
  // The split path keeps its per-env record in con.
  float* pool;
  uint32_t* pool_bm;
  int pool_recs;
  unsigned long long* pool_stat;
};
constexpr int kPoolXcd = 8;       // MI355X: 8 XCDs (HW_REG_XCC_ID), one pool each: a record stays in its XCD's L2
constexpr int kPoolWords = 16;    // <= 512 entries per XCD (32 CUs x 12 resident fused waves = 384)
constexpr int kPoolSlots = 32 * kPoolWords;   // a pool id: XCD x kPoolSlots + bitmap entry

}  // namespace so100
