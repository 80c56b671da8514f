// hsim -- MI355X-native batched humanoid engine: compiled-model layout shared by the host
// compiler (mjcf.cpp) and the HIP step kernel (hs_kernels.hip).
//
// Replaces the reference's `mujoco.MjModel.from_xml_path` product (custom_env.py:53): a
// read-only model shared by every env of a batch.  The host compiler keeps an fp64
// `HostModel`; the device gets a `DevModel<T>` (T = float for throughput, double for the
// parity mode) plus derived topology tables (levels, chain/subtree bitmasks, static
// collision pairs with pre-mixed contact parameters) that let one wavefront step one env.
#pragma once
#include <cstdint>

namespace hs {

// Engine capacity (compile time).  hs_batch_create rejects models that exceed it.
constexpr int MAXBODY = 20;   // bodies incl. world (<= 32: one half-wave lane per body)
constexpr int MAXDOF = 32;    // <= 32 so dof sets fit a 32-bit mask and one lane per dof
constexpr int MAXQ = 40;
constexpr int MAXJNT = 24;    // <= 32
constexpr int MAXGEOM = 24;   // <= 32
constexpr int MAXTEN = 4;
constexpr int MAXWRAP = 4;    // joints per fixed tendon
constexpr int MAXU = 24;
constexpr int MAXPAIR = 192;  // static candidate geom pairs
// Contact / constraint-row capacity per env comes in two tiers (hs_kernels.hip):
//  * resident tier: what every launch runs with, sized so all 4096 envs of configs[1] stay
//    resident (LDS) -- 2.3x / 2.5x the worst full-episode counts measured on the oracle
//    (14 contacts, 52 rows over 48 episodes x tapes T0/T1/T2);
//  * wide tier: an env whose contacts or rows overflow the resident tier in any substep is not
//    committed; a second (small-grid) launch re-runs that env's whole step from the same inputs
//    with this capacity.  Only overflow of the wide tier drops contacts (warning word).
constexpr int MAXCON = 32;    // resident tier: contacts per env (one half-wave lane each)
constexpr int MAXEFC = 128;   // resident tier: constraint rows per env (4 per half-wave lane)
// fp64 resident tier: the same capacity.  (Halving it to 16 / 96 cuts the fp64 scratch to 5 env pairs
// per CU of LDS, but the fp64 engine's registers already hold it to 4 -- 1 wave per SIMD -- so it
// bought nothing; measured r2c.)
constexpr int MAXCON_F64 = 32;
constexpr int MAXEFC_F64 = 128;
constexpr int MAXCON_WIDE = 64;    // wide tier (2 contacts per lane)
constexpr int MAXEFC_WIDE = 256;   // wide tier (8 rows per lane)
// A flat-lying body -- every non-plane geom against the floor at once, 2 contacts per capsule, 4
// pyramid rows per condim-3 contact, one row per joint / tendon limit -- always fits the wide tier
// for any model within the other capacities (mjcf.cpp contact_bound; build_dev_model also checks
// the model's own count).  Only body-body pile-ups on top of it can overflow (HS_WARN_OVERFLOW).
static_assert(2 * (MAXGEOM - 1) <= MAXCON_WIDE, "wide tier must hold every geom on the floor");
static_assert(4 * 2 * (MAXGEOM - 1) + MAXJNT + MAXTEN <= MAXEFC_WIDE, "wide tier rows: every geom on the floor");
constexpr int MAXLEVEL = 16;
constexpr int MAXJPB = 3;     // hinge joints per body (kinematics keeps their rotations in registers)
// solimp on the device: MuJoCo's (d0, dwidth, width, midpoint, power) followed by derived constants
// (1/width, 1/mid^(power-1), 1/(1-mid)^(power-1)) so the impedance sigmoid takes one pow at most
constexpr int SOLIMP = 8;

enum GeomType { GEOM_PLANE = 0, GEOM_SPHERE = 2, GEOM_CAPSULE = 3 };
enum JointType { JNT_FREE = 0, JNT_HINGE = 3 };
enum PairFn { PAIR_PLANE_SPHERE = 0, PAIR_PLANE_CAPSULE = 1, PAIR_SPHERE_SPHERE = 2, PAIR_SPHERE_CAPSULE = 3,
              PAIR_CAPSULE_CAPSULE = 4 };

template <typename T>
struct DevModel {
  int nq, nv, nu, nbody, njnt, ngeom, ntendon, npair, nlevel, nhinge_limited;
  T timestep, gravity[3];
  T newton_scale;                     // 1 / (meaninertia * nv)  (MuJoCo solver scaling)
  T total_mass;
  int level_adr[MAXLEVEL + 1], level_body[MAXBODY];   // bodies grouped by tree depth
  int body_parentid[MAXBODY], body_jntadr[MAXBODY], body_jntnum[MAXBODY], body_depth[MAXBODY];
  int body_dofadr[MAXBODY], body_dofnum[MAXBODY];
  uint32_t body_chainmask[MAXBODY];   // dofs on the path world -> body (incl. own)
  uint32_t body_descmask[MAXBODY];    // bodies in the subtree rooted at body (incl. self)
  T body_pos[MAXBODY][3], body_quat[MAXBODY][4], body_ipos[MAXBODY][3];
  T body_inert[MAXBODY][6];           // inertia about COM in body frame: xx yy zz xy xz yz
  T body_mass[MAXBODY], body_invweight_tran[MAXBODY];
  int jnt_type[MAXJNT], jnt_qposadr[MAXJNT], jnt_dofadr[MAXJNT], jnt_bodyid[MAXJNT], jnt_limited[MAXJNT];
  T jnt_pos[MAXJNT][3], jnt_axis[MAXJNT][3], jnt_range[MAXJNT][2];
  T jnt_solref[MAXJNT][2], jnt_solimp[MAXJNT][SOLIMP], jnt_margin[MAXJNT];
  int dof_bodyid[MAXDOF], dof_jntid[MAXDOF], dof_qposadr[MAXDOF];   // qposadr: hinge dofs, else -1
  uint32_t dof_ancmask[MAXDOF];       // dof ancestors incl. self (dof_parentid chain)
  uint32_t dof_relmask[MAXDOF];       // dof ancestors and descendants incl. self (nonzeros of a row of M)
  uint32_t dof_dotmask[MAXDOF];       // dofs whose motion precedes this dof in mj_comVel
  T dof_armature[MAXDOF], dof_damping[MAXDOF], dof_invweight0[MAXDOF];
  T dof_stiffness[MAXDOF], dof_springref[MAXDOF];
  int dof_actuator[MAXDOF];           // motor driving this dof (-1 none)
  int act_dof[MAXU], act_ctrllimited[MAXU];
  T act_gear[MAXU], act_ctrlrange[MAXU][2];
  int geom_type[MAXGEOM], geom_bodyid[MAXGEOM];
  T geom_pos[MAXGEOM][3], geom_zaxis[MAXGEOM][3], geom_size[MAXGEOM][2];
  // static candidate pairs, canonical (MuJoCo) processing order; g1 has the lower geom type
  int pair_g1[MAXPAIR], pair_g2[MAXPAIR], pair_b1[MAXPAIR], pair_b2[MAXPAIR];
  int pair_fn[MAXPAIR], pair_dim[MAXPAIR];
  T pair_mu[MAXPAIR], pair_margin[MAXPAIR], pair_solref[MAXPAIR][2], pair_solimp[MAXPAIR][SOLIMP];
  // what the narrow phase of one pair needs, packed into two 16-byte records per pair (one
  // dwordx4 load each, no dependent geom-table lookup): {g1, g2, fn, dim}, {r1, h1, r2, h2}
  alignas(16) int pair_info[MAXPAIR][4];
  alignas(16) T pair_size[MAXPAIR][4];
  int ten_nwrap[MAXTEN], ten_wrapdof[MAXTEN][MAXWRAP], ten_wrapqadr[MAXTEN][MAXWRAP], ten_limited[MAXTEN];
  T ten_wrapcoef[MAXTEN][MAXWRAP], ten_range[MAXTEN][2], ten_solref[MAXTEN][2], ten_solimp[MAXTEN][SOLIMP];
  T ten_margin[MAXTEN], ten_invweight0[MAXTEN];
  T qpos0[MAXQ];
  T pgs_tol;                          // <option tolerance> (the PGS stopping rule; Newton solves exactly)
};

}  // namespace hs
