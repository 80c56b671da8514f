// Host sanitizer harness for the product's MJCF compiler (mjcf.cpp), the code that replaces
// mujoco.MjModel.from_xml_path (reference custom_env.py:53).  Built with
// -fsanitize=address,undefined by `make -C mujocoposelearning_amd/csrc asan` and run by
// tests/test_sanitizers.py over the shipped model, option overrides and malformed inputs.
// For each path: compile; on success read every model field through model_field and build both
// device layouts (what hs_model_load + hs_batch_create do on the host); print one line
// "OK <nq> <nv> <nu> <npair>" or "ERR <message>".
#include <cstdio>
#include <string>
#include <vector>

#include "../mujocoposelearning_amd/csrc/mjcf.h"

int main(int argc, char** argv) {
  const char* fields[] = {"nq", "nv", "nu", "nbody", "njnt", "ngeom", "ntendon", "body_pos", "body_quat", "body_mass",
                          "body_inertia_full", "jnt_range", "jnt_solimp", "geom_size", "geom_solimp", "tendon_range",
                          "wrap_coef", "actuator_gear", "actuator_ctrlrange", "collision_pairs", "qpos0", "key_squat",
                          "no_such_field"};
  for (int a = 1; a < argc; a++) {
    hs::HostModel m;
    std::string err;
    if (!hs::compile_mjcf_file(argv[a], m, err)) {
      std::printf("ERR %s\n", err.c_str());
      continue;
    }
    for (const char* f : fields) {
      int n = hs::model_field(m, f, nullptr, 0);
      if (n > 0) {
        std::vector<double> v((size_t)n);
        hs::model_field(m, f, v.data(), n);
      }
    }
    auto* d32 = new hs::DevModel<float>();
    auto* d64 = new hs::DevModel<double>();
    std::string e32, e64;
    const bool ok = hs::build_dev_model<float>(m, *d32, e32) && hs::build_dev_model<double>(m, *d64, e64);
    delete d32;
    delete d64;
    if (!ok) std::printf("ERR device layout: %s%s\n", e32.c_str(), e64.c_str());
    else std::printf("OK %d %d %d %d\n", m.nq, m.nv, m.nu, (int)m.pair_geom.size());
  }
  return 0;
}
