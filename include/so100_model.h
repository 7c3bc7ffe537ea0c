/* so100_model.h — plain-data layout of the derived SO-ARM100 bin-a-cube model.
 *
 * This is the ONLY structure that crosses the C-ABI at create time (so100_create, so100.h).
 * It is filled on the host from gym_so100/assets/so100_model.json (written by
 * tools/compile_model.py from /root/reference/gym_so100/assets/so100_transfer_cube.xml).
 * Double precision on the host; the device copy is converted to fp32 inside so100_create.
 *
 * Numbering (build-owned, compact):
 *   bodies 0 world | 1 Base (static, welded) | 2 Rotation_Pitch | 3 Upper_Arm | 4 Lower_Arm |
 *          5 Wrist_Pitch_Roll | 6 Fixed_Jaw | 7 Moving_Jaw | 8 box (free joint)
 *   dofs   0..5 arm hinges (Rotation, Pitch, Elbow, Wrist_Pitch, Wrist_Roll, Jaw),
 *          6..8 cube linear (world frame), 9..11 cube angular (body frame)  (MuJoCo free-joint layout)
 *   qpos   0..5 hinges, 6..8 cube position, 9..12 cube quaternion (w,x,y,z)
 *   geoms  0 table | 1..4 fixed_jaw_pad_1..4 | 5..8 moving_jaw_pad_1..4 | 9 red_box | 10..14 bin walls+floor |
 *          15 the EE variant's mocap marker box (so_arm100_ee.xml:155; body SO100_MOCAP_BODY: its pose is the env's
 *          mocap input)
 *   pairs  0..7 pad-vs-red_box | 8 (red_box, table) | 9..13 (red_box, bin_*)   (box-box)
 *          14..22 (table, hull k): arm/jaw collision hulls vs the table top
 *          23..31 (red_box, hull k) | 32..76 (bin box j, hull k) at 32 + 9 j + k, j = bin_wall,
 *          bin_wall2..4, bin_floor: box vs convex hull through the MPR convex collider
 *          77..97 (hull k1, hull k2): self-collision of hulls on non-adjacent arm links (MPR)
 *          98..106 (red_box, Base hull) and (Base hull, hull k), k = 1..8: the static Base (MPR)
 *          107..142 (finger pad, link hull)
 *          143..151 (mocap marker box, link hull k) (EE variant only, convex collider)
 *          152..159 (finger pad i, table); 160..199 (finger pad i, bin box j) at 160 + 5 i + j
 *          200..208 (cube | finger pad i, mocap marker box) (EE variant only, box-box)
 *   hulls  0 Rotation_Pitch | 1 Upper_Arm | 2 Lower_Arm | 3 Wrist_Pitch_Roll |
 *          4..5 Fixed_Jaw_Collision_1..2 | 6..8 Moving_Jaw_Collision_1..3
 */
#ifndef SO100_MODEL_H
#define SO100_MODEL_H

#define SO100_NBODY 9
#define SO100_NHINGE 6
#define SO100_NQ 13
#define SO100_NV 12
#define SO100_NU 6
#define SO100_NGEOM 16
#define SO100_MOCAP_GEOM 15         /* the EE variant's mocap marker box */
#define SO100_MOCAP_BODY 9          /* its body: the mocap body (no dofs; not in the body arrays)         */
#define SO100_NPAIR_BOX 14         /* box-box pairs 0..13 */
#define SO100_NHULL 9               /* arm/jaw collision hulls (moving links) */
#define SO100_HULL_BASE 9           /* hull 9: the static Base's collision hull */
#define SO100_NHULL_ALL 10          /* hull arrays: the 9 link hulls + the Base hull */
#define SO100_NBINBOX 5             /* bin walls + floor (geoms 10..14) */
#define SO100_PAIR_MPR0 (SO100_NPAIR_BOX + SO100_NHULL)     /* 23: first (box, hull) MPR pair */
#define SO100_NPAIR_MPR ((1 + SO100_NBINBOX) * SO100_NHULL) /* 54: (cube | bin box j, hull k) */
#define SO100_PAIR_SELF0 (SO100_PAIR_MPR0 + SO100_NPAIR_MPR)  /* 77: first hull-hull self-collision pair */
#define SO100_NPAIR_SELF 21                                 /* hulls on non-adjacent arm links */
#define SO100_PAIR_BASE0 (SO100_PAIR_SELF0 + SO100_NPAIR_SELF)  /* 98: (cube, Base hull), then (Base hull, hull k) */
#define SO100_NPAIR_BASE 9                                  /* 99..106: hull k = 1..8 (Rotation_Pitch excluded) */
#define SO100_PAIR_PADLINK0 (SO100_PAIR_BASE0 + SO100_NPAIR_BASE)  /* 107: first (pad, link hull) pair */
#define SO100_NPAIR_PADLINK 36                              /* 107..142: pads vs Base, Rotation_Pitch, Upper_Arm,
                                                               Lower_Arm, Wrist_Pitch_Roll (not the fixed pads' parent) */
#define SO100_NPAIR_CONVEX (SO100_NPAIR_MPR + SO100_NPAIR_SELF + SO100_NPAIR_BASE + SO100_NPAIR_PADLINK)  /* 120 through MPR */
#define SO100_PAIR_MOCAPHULL0 (SO100_PAIR_PADLINK0 + SO100_NPAIR_PADLINK)  /* 143: (mocap box, link hull k), EE only */
#define SO100_NPAIR_MOCAPHULL SO100_NHULL                   /* 9 */
#define SO100_PAIR_PAD0 (SO100_PAIR_MOCAPHULL0 + SO100_NPAIR_MOCAPHULL)  /* 152: first (pad, table | bin box) pair */
#define SO100_NPAD 8                                        /* finger pads: geoms 1..8 */
#define SO100_PAIR_PADBIN0 (SO100_PAIR_PAD0 + SO100_NPAD)   /* 160: (pad i, bin box j) at 160 + 5 i + j */
#define SO100_NPAIR_PADBIN (SO100_NPAD * SO100_NBINBOX)     /* 40, box-box */
#define SO100_NPAIR_PAD (SO100_NPAD + SO100_NPAIR_PADBIN)   /* 48: 143..150 (pad i, table), then pad-bin */
#define SO100_PAIR_MOCAPBOX0 (SO100_PAIR_PAD0 + SO100_NPAIR_PAD)  /* 200: (cube | pad i, mocap box), EE only */
#define SO100_NPAIR_MOCAPBOX (1 + SO100_NPAD)               /* 9, box-box */
#define SO100_NPAIR (SO100_PAIR_MOCAPBOX0 + SO100_NPAIR_MOCAPBOX)  /* 209: every pair MuJoCo's filters leave (the
                                                               joint variant's 191 and the EE variant's 18 more) */
#define SO100_NPAIR_BITS SO100_PAIR_MPR0                    /* contact_bits covers pairs 0..22 */
#define SO100_HULL_NVERT 2560       /* hull vertex capacity, all hulls */
#define SO100_HULL_CELLG 8          /* support-direction cells per cube-map face edge (so100_hull_cells) */
#define SO100_HULL_NCELL (6 * SO100_HULL_CELLG * SO100_HULL_CELLG)   /* cells per hull */
#define SO100_CUBE_BODY 8
#define SO100_CUBE_GEOM 9
#define SO100_PAIR_TABLE 8          /* ("red_box", "table") — single_arm.py:354 touch_table */
#define SO100_NPAIR_GRIPPER 8       /* pairs 0..7 — single_arm.py:348-352 touch_gripper   */
#define SO100_MAXCONPAIR 8          /* contacts per box-box pair: every clipped point, as mjc_BoxBox */
/* box-box pairs that keep every clipped point: the cube against the 8 pads and the 5 bin boxes (pairs 0..13
 * but the cube-table pair 8, whose table is a mesh: one convex contact), the 40 pad-bin pairs and (EE variant) the
 * cube and the pads against the mocap marker box */
#define SO100_NPAIR_MULTI (SO100_NPAIR_BOX - 1 + SO100_NPAIR_PADBIN + SO100_NPAIR_MOCAPBOX)  /* 62 */
/* The contact list of an env holds up to SO100_NCON_MAX contacts: every pair at its collider's maximum (8 for
 * a multi-point box-box pair, 1 for the convex collider and the table rules), so no contact MuJoCo would keep
 * can be left out (MuJoCo has no per-env cap).  The kernels hold the first SO100_MAXCON of them on chip (the
 * solver's lane c owns contact c); the rest live in the env's HBM record (include/so100.h). */
#define SO100_NCON_MAX (SO100_NPAIR_MULTI * SO100_MAXCONPAIR + SO100_NPAIR - SO100_NPAIR_MULTI)  /* 643 */
#define SO100_MAXCON 16             /* contacts an env holds on chip (LDS / registers) per position stage */
#define SO100_CONDIM 4              /* max condim: cube pairs mix to 4, table/bin-hull pairs are 3 */
#define SO100_NEFC_MAX (SO100_NV + SO100_NHINGE + SO100_NCON_MAX * SO100_CONDIM)
#define SO100_SOLVER_PGS 0          /* projected Gauss-Seidel on the dual (mj_solPGS)               */
#define SO100_SOLVER_NEWTON 1       /* primal Newton with exact line search (mj_solNewton)          */
#define SO100_CONVEX_MPR 0          /* mesh pairs through libccd's MPR (MuJoCo behind mjDSBL_NATIVECCD)  */
#define SO100_CONVEX_EPA 1          /* mesh pairs through GJK + EPA (MuJoCo 3.3.3's default native ccd)  */
#define SO100_NOBS 15               /* box(3) bin(3) ee(3) qpos(6) — env.py:137-145      */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct so100_model {
  /* options (MuJoCo defaults + so_arm100.xml:4) */
  double timestep;                  /* 0.002 */
  int    nsubstep;                  /* control_timestep / timestep = 10 (env.py:120-127) */
  int    iterations;                /* solver iterations: PGS sweeps / Newton steps (MuJoCo default 100) */
  int    solver;                    /* SO100_SOLVER_PGS (north_star) or SO100_SOLVER_NEWTON (MuJoCo's default) */
  double tolerance;                 /* 1e-8 */
  double impratio;                  /* 10 */
  double gravity[3];
  double meaninertia;               /* mean diag(M) at qpos0, scales the PGS improvement */

  /* bodies */
  int    body_parent[SO100_NBODY];
  double body_pos[SO100_NBODY][3];
  double body_quat[SO100_NBODY][4];
  double body_ipos[SO100_NBODY][3];
  double body_iquat[SO100_NBODY][4];
  double body_mass[SO100_NBODY];
  double body_inertia[SO100_NBODY][3];
  double body_invweight0[SO100_NBODY][2];

  /* hinges (one per arm body 2..7) */
  int    jnt_body[SO100_NHINGE];
  double jnt_axis[SO100_NHINGE][3];
  double jnt_range[SO100_NHINGE][2];
  double jnt_solref[2];
  double jnt_solimp[5];

  /* dofs */
  double dof_armature[SO100_NV];
  double dof_frictionloss[SO100_NV];
  double dof_invweight0[SO100_NV];
  double dof_solref[2];
  double dof_solimp[5];

  /* position actuators (gear 1 on hinge i) */
  double act_kp[SO100_NU];
  double act_kv[SO100_NU];
  double act_forcerange[SO100_NU][2];
  double act_ctrlrange[SO100_NU][2];

  /* collision boxes: pos/quat in the body frame (world frame for body 0) */
  int    geom_body[SO100_NGEOM];
  double geom_pos[SO100_NGEOM][3];
  double geom_quat[SO100_NGEOM][4];
  double geom_size[SO100_NGEOM][3];

  /* contact pairs with mixed parameters (a hull geom is -1 - hull index: geom2 of the hull pairs, both
   * geoms of the self-collision pairs) */
  int    pair_geom1[SO100_NPAIR];
  int    pair_geom2[SO100_NPAIR];
  int    pair_body1[SO100_NPAIR];
  int    pair_body2[SO100_NPAIR];
  int    pair_condim[SO100_NPAIR];
  double pair_friction[SO100_NPAIR][3];
  double pair_solref[SO100_NPAIR][2];
  double pair_solimp[SO100_NPAIR][5];
  double pair_margin[SO100_NPAIR];

  /* arm/jaw collision hulls: convex hulls of the collision meshes, vertices in the body frame,
   * body-frame bounding box (center, half extents) for the broadphase; the table's top face (z, x-y
   * footprint) */
  int    hull_body[SO100_NHULL_ALL];
  int    hull_start[SO100_NHULL_ALL];
  int    hull_count[SO100_NHULL_ALL];
  double hull_center[SO100_NHULL_ALL][3];
  double hull_half[SO100_NHULL_ALL][3];
  double hull_centroid[SO100_NHULL_ALL][3];   /* mesh volume centroid = the mesh geom's frame origin */
  double hull_vert[SO100_HULL_NVERT][3];
  double table_top;
  double table_lo[2];
  double table_hi[2];

  /* sites */
  int    site_cube_body;
  double site_cube_pos[3];
  int    site_ee_body;
  double site_ee_pos[3];
  double bin_center[3];

  /* task constants (reference file:line cited in gym_so100/constants.py) */
  double start_qpos[SO100_NU];      /* constants.py:32-39 */
  double action_lo[SO100_NU];       /* constants.py:78-86 */
  double action_hi[SO100_NU];
  double spawn_lo[3];               /* utils.py:18-22 */
  double spawn_hi[3];
  double bin_hw;                    /* single_arm.py:69 */
  double bin_h;                     /* single_arm.py:70 */
  double cube_half;                 /* single_arm.py:75 */
  double goal_threshold;            /* env.py:252 */
  double max_reward;                /* single_arm.py:130,227,297 */
  double goal_bin_lo[3];            /* env.py:245-249 bin_goal_space (constants.py:29-30) */
  double goal_bin_hi[3];

  /* EE / mocap variant (so100_transfer_cube_ee.xml with trs_so_arm100/so_arm100_ee.xml:155,171-173): a
   * weld equality between the mocap body's site and ee_site drives the end effector to a per-env pose */
  int    ee;                        /* 1: weld on (so100_buffers.mocap), 0: the reference's default model */
  double weld_pos2[3];              /* ee_site in the Fixed_Jaw frame */
  double weld_quat2[4];             /* ee_site frame orientation in the Fixed_Jaw frame */
  double weld_solref[2];            /* so_arm100_ee.xml:172 */
  double weld_solimp[5];
  double weld_torquescale;
  double weld_invweight0[2];        /* body_invweight0 (tran, rot) of the ee_site body; the mocap body's is 0 */
  double mocap_pos0[3];             /* so_arm100_ee.xml:155 mocap body pose (default of the mocap input) */
  double mocap_quat0[4];

  /* the convex collider of the mesh pairs 23..142 (mjc_Convex): SO100_CONVEX_EPA (MuJoCo 3.3.3's default: the
   * minimum penetration) or SO100_CONVEX_MPR (libccd's MPR: the penetration along the centres' ray) */
  int    convex;
} so100_model;

#ifdef __cplusplus
}
#endif
#endif
