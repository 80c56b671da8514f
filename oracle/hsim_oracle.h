/* ORACLE (test infrastructure only): fp64 CPU restatement of MuJoCo 3.2.5 mj_step for the
 * model class of the reference's XML/humanoid.xml. Never linked into the product.
 * See hsim_oracle.c for the per-stage citations. Parity against real MuJoCo is UNPINNED
 * (MuJoCo is not installable here). */
#ifndef HSIM_ORACLE_H
#define HSIM_ORACLE_H

#define OMAXB 32
#define OMAXJ 32
#define OMAXV 40
#define OMAXQ 48
#define OMAXG 32
#define OMAXT 8
#define OMAXW 32
#define OMAXU 32
#define OMAXCON 160
#define OMAXEFC 640
#define OMAXPAIR 512

typedef struct {
  int nq, nv, nu, nbody, njnt, ngeom, ntendon, npair;
  double timestep, gravity[3], impratio, tolerance, meaninertia;
  int iterations;
  int solver;                                  /* 0 = Newton (MuJoCo default), 1 = PGS */
  int body_parentid[OMAXB], body_rootid[OMAXB], body_weldid[OMAXB];
  int body_jntnum[OMAXB], body_jntadr[OMAXB], body_dofnum[OMAXB], body_dofadr[OMAXB];
  double body_pos[OMAXB][3], body_quat[OMAXB][4], body_ipos[OMAXB][3];
  double body_inertia_full[OMAXB][9];          /* inertia about COM, body frame (== iquat*diag*iquat') */
  double body_mass[OMAXB], body_subtreemass[OMAXB], body_invweight0[OMAXB][2];
  int jnt_type[OMAXJ], jnt_qposadr[OMAXJ], jnt_dofadr[OMAXJ], jnt_bodyid[OMAXJ], jnt_limited[OMAXJ];
  double jnt_pos[OMAXJ][3], jnt_axis[OMAXJ][3], jnt_range[OMAXJ][2], jnt_stiffness[OMAXJ];
  double jnt_solref[OMAXJ][2], jnt_solimp[OMAXJ][5], jnt_margin[OMAXJ];
  int dof_bodyid[OMAXV], dof_jntid[OMAXV], dof_parentid[OMAXV];
  double dof_armature[OMAXV], dof_damping[OMAXV], dof_invweight0[OMAXV];
  double qpos0[OMAXQ], qpos_spring[OMAXQ];
  int geom_type[OMAXG], geom_bodyid[OMAXG], geom_condim[OMAXG], geom_priority[OMAXG];
  double geom_size[OMAXG][3], geom_pos[OMAXG][3], geom_quat[OMAXG][4], geom_friction[OMAXG][3];
  double geom_solref[OMAXG][2], geom_solimp[OMAXG][5], geom_margin[OMAXG], geom_gap[OMAXG];
  double geom_solmix[OMAXG], geom_rbound[OMAXG];
  int tendon_adr[OMAXT], tendon_num[OMAXT], tendon_limited[OMAXT];
  double tendon_range[OMAXT][2], tendon_solref[OMAXT][2], tendon_solimp[OMAXT][5];
  double tendon_margin[OMAXT], tendon_invweight0[OMAXT];
  int wrap_jnt[OMAXW]; double wrap_coef[OMAXW];
  int actuator_trnid[OMAXU], actuator_ctrllimited[OMAXU];
  double actuator_gear[OMAXU], actuator_ctrlrange[OMAXU][2];
  int pair_geom[OMAXPAIR][2];                  /* static candidate pairs in processing order */
} OrcModel;

typedef struct {
  double pos[3], frame[9], dist, includemargin, friction[5], solref[2], solimp[5];
  int geom[2], dim, efc_address;
} OrcContact;

typedef struct {
  double time;
  double qpos[OMAXQ], qvel[OMAXV], ctrl[OMAXU], qacc_warmstart[OMAXV], qacc[OMAXV], qacc_smooth[OMAXV];
  double xpos[OMAXB][3], xquat[OMAXB][4], xmat[OMAXB][9], xipos[OMAXB][3], ximat[OMAXB][9];
  double xanchor[OMAXJ][3], xaxis[OMAXJ][3], geom_xpos[OMAXG][3], geom_xmat[OMAXG][9];
  double subtree_com[OMAXB][3], cinert[OMAXB][10], cdof[OMAXV][6], cvel[OMAXB][6], cdof_dot[OMAXV][6];
  double crb[OMAXB][10];
  double qM[OMAXV][OMAXV];
  double ten_length[OMAXT], ten_J[OMAXT][OMAXV];
  double actuator_force[OMAXU];
  double qfrc_bias[OMAXV], qfrc_passive[OMAXV], qfrc_actuator[OMAXV], qfrc_smooth[OMAXV];
  double qfrc_constraint[OMAXV];
  double cfrc_ext[OMAXB][6], subtree_linvel[OMAXB][3];   /* zero unless orc_step_full */
  int ncon;
  OrcContact contact[OMAXCON];
  int nefc;
  int efc_type[OMAXEFC], efc_id[OMAXEFC];
  double efc_J[OMAXEFC][OMAXV];
  double efc_pos[OMAXEFC], efc_margin[OMAXEFC], efc_vel[OMAXEFC], efc_aref[OMAXEFC];
  double efc_R[OMAXEFC], efc_D[OMAXEFC], efc_diagApprox[OMAXEFC], efc_KBIP[OMAXEFC][4];
  double efc_force[OMAXEFC];
  int solver_niter;
  int warning_badqpos, warning_badqvel, warning_badqacc, warning_overflow;
} OrcData;

enum { ORC_LIMIT_JOINT = 3, ORC_LIMIT_TENDON = 4, ORC_CONTACT_FRICTIONLESS = 5, ORC_CONTACT_PYRAMIDAL = 6 };

#ifdef __cplusplus
extern "C" {
#endif
int orc_sizeof_model(void);
int orc_sizeof_data(void);
void orc_reset_data(const OrcModel* m, OrcData* d);
void orc_forward(const OrcModel* m, OrcData* d);
void orc_step(const OrcModel* m, OrcData* d);
void orc_step_n(const OrcModel* m, OrcData* d, const double* ctrl, int nsub);
extern int orc_variant;   /* known-wrong physics switches (hsim_oracle.c), 0 = the restatement */
extern double orc_mp_tol;          /* gradient stop of the mixed-precision Newton variant (16) */
extern long orc_stat_nfactor;      /* Newton factorizations so far (statistics) */
extern int orc_mp_euler_refine;    /* refinements of the fp32-factored Euler solve (variant 64) */
extern double orc_ls_tolerance;    /* MuJoCo's opt.ls_tolerance for the inexact line search (variant 32) */
extern int orc_ls_iterations;      /* MuJoCo's opt.ls_iterations (variant 32) */
extern long orc_stat_ls_evals;     /* inexact line-search cost evaluations so far (statistics) */
/* full-state option: after mj_forward, the contact part of mj_rnePostConstraint (cfrc_ext) and
 * mj_subtreeVel (subtree_linvel), i.e. what MuJoCo computes when those fields are requested;
 * the reference never requests them (zeros), so this is hsim's opt-in "full_state" mode. */
void orc_contact_forces(const OrcModel* m, OrcData* d);
void orc_step_n_full(const OrcModel* m, OrcData* d, const double* ctrl, int nsub, int full);
#ifdef __cplusplus
}
#endif
#endif
