// hsim host-side MJCF compiler (product code).  Replaces MuJoCo's mj_loadXML + mj_setConst
// for the constructs used by the reference's XML/humanoid.xml (custom_env.py:53 loads it via
// mujoco.MjModel.from_xml_path).  Produces an fp64 HostModel with MuJoCo field names, then a
// DevModel<T> for the kernels.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "hs_model.h"

namespace hs {

struct HostModel {
  int nq = 0, nv = 0, nu = 0, nbody = 0, njnt = 0, ngeom = 0, ntendon = 0;
  double timestep = 0.002, gravity[3] = {0, 0, -9.81}, meaninertia = 1;
  int iterations = 100;          // <option iterations> (MuJoCo default): the default Newton cap
  double tolerance = 1e-8;       // <option tolerance> (Newton solves to the exact minimiser; PGS stops on it)
  int solver = 0;                // <option solver>: 0 Newton (MuJoCo default), 1 PGS
  std::vector<std::string> body_name, jnt_name, geom_name, actuator_name, tendon_name;
  std::vector<int> body_parentid, body_rootid, body_weldid, body_jntadr, body_jntnum, body_dofadr, body_dofnum;
  std::vector<double> body_pos, body_quat, body_ipos, body_iquat, body_inertia, body_inertia_full;  // 3,4,3,4,3,9
  std::vector<double> body_mass, body_subtreemass, body_invweight0;                                  // 1,1,2
  std::vector<int> jnt_type, jnt_qposadr, jnt_dofadr, jnt_bodyid, jnt_limited;
  std::vector<double> jnt_pos, jnt_axis, jnt_range, jnt_stiffness, jnt_springref, jnt_solref, jnt_solimp, jnt_margin;
  std::vector<int> dof_bodyid, dof_jntid, dof_parentid;
  std::vector<double> dof_armature, dof_damping, dof_invweight0;
  std::vector<double> qpos0, qpos_spring;
  std::vector<int> geom_type, geom_bodyid, geom_condim, geom_contype, geom_conaffinity, geom_priority;
  std::vector<double> geom_size, geom_pos, geom_quat, geom_friction, geom_solref, geom_solimp;  // 3,3,4,3,2,5
  std::vector<double> geom_margin, geom_gap, geom_solmix, geom_rbound;
  std::vector<int> tendon_adr, tendon_num, tendon_limited, wrap_jnt;
  std::vector<double> wrap_coef, tendon_range, tendon_solref, tendon_solimp, tendon_margin, tendon_invweight0;
  std::vector<int> actuator_trnid, actuator_ctrllimited;
  std::vector<double> actuator_gear, actuator_ctrlrange;
  std::vector<std::pair<int, int>> exclude;     // body pairs (min, max)
  std::vector<std::pair<int, int>> pair_geom;   // static collision candidates, canonical order
  std::map<std::string, std::vector<double>> keyframes;
};

// Parse + compile. Returns false and fills err on failure.
bool compile_mjcf_file(const std::string& path, HostModel& out, std::string& err);

// Export a named field as doubles (introspection for tests / the Python mirror).
// Returns number of values written (or needed, if n is too small), -1 if unknown.
int model_field(const HostModel& m, const std::string& name, double* out, int n);

// Worst-case contact / constraint-row counts of one env, from the static collision pair list:
// MuJoCo keeps every contact (custom_env.py:160 mj_step has no per-env cap).  Per pair, the most
// contacts its narrow phase can return (plane-capsule 2, capsule-capsule 2, the sphere pairs 1);
// per contact, its rows (condim 1: 1, condim 3 pyramidal: 4); plus one row per limited hinge and
// per limited tendon (at most one side of a limit is violated at a time).  `all`: every pair
// touching at once (a geometric bound, far above any reachable state); `floor`: every geom against
// the plane at once (a humanoid lying flat) -- the engine's wide tier must hold it (build_dev_model).
struct ContactBound { int con_all, efc_all, con_floor, efc_floor; };
ContactBound contact_bound(const HostModel& m);

// Build the device layout; returns false (with err) if the model exceeds engine capacity.
template <typename T>
bool build_dev_model(const HostModel& m, DevModel<T>& d, std::string& err);

}  // namespace hs
