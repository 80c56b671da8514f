// hsim MJCF compiler (product).  Semantics follow MuJoCo 3.2.5's compiler for the subset the
// reference model uses (XML/humanoid.xml): default classes (:35-102), childclass (:110),
// freejoint (:111), hinge joints in degrees, capsule/sphere/plane geoms with inertiafromgeom
// (density 1000), fixed tendons (:191-200), motors (:202-224), contact excludes (:186-189),
// keyframes (:226-266); then mj_setConst's body/dof/tendon invweight0 and meaninertia.
#include "mjcf.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <set>
#include <sstream>

namespace hs {
namespace {

constexpr double kMinVal = 1e-15;
constexpr double kPi = 3.14159265358979323846;

// ------------------------------------------------------------------ minimal XML reader
struct XNode {
  std::string tag;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<XNode>> kids;
  const char* get(const char* k) const {
    for (auto& a : attrs)
      if (a.first == k) return a.second.c_str();
    return nullptr;
  }
};

struct XParser {
  const std::string& s;
  size_t i = 0;
  std::string err;
  explicit XParser(const std::string& src) : s(src) {}
  void skip_ws() { while (i < s.size() && isspace((unsigned char)s[i])) i++; }
  bool skip_misc() {  // comments, <?...?>, <!...>
    for (;;) {
      skip_ws();
      if (s.compare(i, 4, "<!--") == 0) {
        size_t e = s.find("-->", i + 4);
        if (e == std::string::npos) { err = "unterminated comment"; return false; }
        i = e + 3;
      } else if (s.compare(i, 2, "<?") == 0) {
        size_t e = s.find("?>", i + 2);
        if (e == std::string::npos) { err = "unterminated <?"; return false; }
        i = e + 2;
      } else if (s.compare(i, 2, "<!") == 0) {
        size_t e = s.find('>', i + 2);
        if (e == std::string::npos) { err = "unterminated <!"; return false; }
        i = e + 1;
      } else {
        return true;
      }
    }
  }
  std::unique_ptr<XNode> element() {
    if (!skip_misc()) return nullptr;
    if (i >= s.size() || s[i] != '<') { err = "expected '<'"; return nullptr; }
    i++;
    auto n = std::make_unique<XNode>();
    while (i < s.size() && !isspace((unsigned char)s[i]) && s[i] != '>' && s[i] != '/') n->tag += s[i++];
    for (;;) {
      skip_ws();
      if (i >= s.size()) { err = "eof in tag"; return nullptr; }
      if (s[i] == '/') {
        if (s.compare(i, 2, "/>") != 0) { err = "bad '/'"; return nullptr; }
        i += 2;
        return n;
      }
      if (s[i] == '>') { i++; break; }
      std::string k;
      while (i < s.size() && s[i] != '=' && !isspace((unsigned char)s[i])) k += s[i++];
      skip_ws();
      if (i >= s.size() || s[i] != '=') { err = "expected '=' after " + k; return nullptr; }
      i++;
      skip_ws();
      char q = s[i];
      if (q != '"' && q != '\'') { err = "expected quote"; return nullptr; }
      size_t e = s.find(q, i + 1);
      if (e == std::string::npos) { err = "unterminated attribute"; return nullptr; }
      n->attrs.emplace_back(k, s.substr(i + 1, e - i - 1));
      i = e + 1;
    }
    for (;;) {  // children until </tag>
      if (!skip_misc()) return nullptr;
      if (i >= s.size()) { err = "eof in <" + n->tag + ">"; return nullptr; }
      if (s.compare(i, 2, "</") == 0) {
        size_t e = s.find('>', i);
        if (e == std::string::npos) { err = "bad close tag"; return nullptr; }
        i = e + 1;
        return n;
      }
      if (s[i] != '<') {  // text content: skip
        while (i < s.size() && s[i] != '<') i++;
        continue;
      }
      auto c = element();
      if (!c) return nullptr;
      n->kids.push_back(std::move(c));
    }
  }
};

std::vector<double> nums(const char* s) {
  std::vector<double> v;
  if (!s) return v;
  std::istringstream is(s);
  double x;
  while (is >> x) v.push_back(x);
  return v;
}

// ------------------------------------------------------------------ small math
void quat_mul(double* r, const double* a, const double* b) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  std::memcpy(r, t, sizeof t);
}
void quat2mat(double* R, const double* q) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
void mv3(double* r, const double* R, const double* v) {
  double t[3] = {R[0] * v[0] + R[1] * v[1] + R[2] * v[2], R[3] * v[0] + R[4] * v[1] + R[5] * v[2],
                 R[6] * v[0] + R[7] * v[1] + R[8] * v[2]};
  std::memcpy(r, t, sizeof t);
}
void cross(double* r, const double* a, const double* b) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  std::memcpy(r, t, sizeof t);
}
// mju_quatZ2Vec
void quat_z2vec(double* q, const double* vec) {
  q[0] = 1; q[1] = q[2] = q[3] = 0;
  double v[3] = {vec[0], vec[1], vec[2]};
  double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (n < kMinVal) return;
  for (double& x : v) x /= n;
  double z[3] = {0, 0, 1}, ax[3];
  cross(ax, z, v);
  double a = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
  if (std::fabs(a) < kMinVal) {
    if (v[2] < 0) { q[0] = 0; q[1] = 1; }
    return;
  }
  for (double& x : ax) x /= a;
  double ang = std::atan2(a, v[2]);
  q[0] = std::cos(ang / 2);
  for (int k = 0; k < 3; k++) q[k + 1] = ax[k] * std::sin(ang / 2);
}
// Jacobi eigen-decomposition of a symmetric 3x3 (columns of V = eigenvectors)
void eig3(const double* A, double* w, double* V) {
  double a[9];
  std::memcpy(a, A, sizeof a);
  for (int i = 0; i < 9; i++) V[i] = (i % 4 == 0);
  for (int sweep = 0; sweep < 50; sweep++) {
    double off = a[1] * a[1] + a[2] * a[2] + a[5] * a[5];
    if (off < 1e-30) break;
    for (int p = 0; p < 2; p++)
      for (int q = p + 1; q < 3; q++) {
        double apq = a[3 * p + q];
        if (std::fabs(apq) < 1e-300) continue;
        double theta = (a[3 * q + q] - a[3 * p + p]) / (2 * apq);
        double t = (theta >= 0 ? 1 : -1) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < 3; k++) {  // A = J' A J
          double akp = a[3 * k + p], akq = a[3 * k + q];
          a[3 * k + p] = c * akp - s * akq;
          a[3 * k + q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; k++) {
          double apk = a[3 * p + k], aqk = a[3 * q + k];
          a[3 * p + k] = c * apk - s * aqk;
          a[3 * q + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; k++) {
          double vkp = V[3 * k + p], vkq = V[3 * k + q];
          V[3 * k + p] = c * vkp - s * vkq;
          V[3 * k + q] = s * vkp + c * vkq;
        }
      }
  }
  for (int k = 0; k < 3; k++) w[k] = a[4 * k];
}
void mat2quat(double* q, const double* R) {
  double t = R[0] + R[4] + R[8];
  if (t > 0) {
    double s = std::sqrt(t + 1) * 2;
    q[0] = 0.25 * s; q[1] = (R[7] - R[5]) / s; q[2] = (R[2] - R[6]) / s; q[3] = (R[3] - R[1]) / s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    double s = std::sqrt(1 + R[0] - R[4] - R[8]) * 2;
    q[0] = (R[7] - R[5]) / s; q[1] = 0.25 * s; q[2] = (R[1] + R[3]) / s; q[3] = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    double s = std::sqrt(1 + R[4] - R[0] - R[8]) * 2;
    q[0] = (R[2] - R[6]) / s; q[1] = (R[1] + R[3]) / s; q[2] = 0.25 * s; q[3] = (R[5] + R[7]) / s;
  } else {
    double s = std::sqrt(1 + R[8] - R[0] - R[4]) * 2;
    q[0] = (R[3] - R[1]) / s; q[1] = (R[2] + R[6]) / s; q[2] = (R[5] + R[7]) / s; q[3] = 0.25 * s;
  }
  double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int k = 0; k < 4; k++) q[k] /= (q[0] < 0 ? -n : n);
}

// ------------------------------------------------------------------ default classes
using Attrs = std::map<std::string, std::string>;
struct DefClass {
  std::map<std::string, Attrs> el;   // element tag -> attributes
};

struct Compiler {
  HostModel& m;
  std::string& err;
  std::map<std::string, DefClass> classes;
  std::map<std::string, int> jnt_by_name, body_by_name;
  Compiler(HostModel& mm, std::string& e) : m(mm), err(e) {}

  // exactly n numbers in attribute text s (what = the attribute, for the message)
  bool numsn(const char* s, size_t n, const char* what, std::vector<double>& v) {
    v = nums(s);
    if (v.size() == n) return true;
    err = std::string("attribute '") + what + "' needs " + std::to_string(n) + " number(s), got '" + (s ? s : "") + "'";
    return false;
  }
  bool num1(const char* s, const char* what, double& x) {
    std::vector<double> v;
    if (!numsn(s, 1, what, v)) return false;
    x = v[0];
    return true;
  }

  void parse_defaults(const XNode* n, const DefClass* parent) {
    DefClass d = parent ? *parent : DefClass();
    for (auto& k : n->kids)
      if (k->tag != "default")
        for (auto& a : k->attrs) d.el[k->tag][a.first] = a.second;
    const char* cls = n->get("class");
    std::string name = cls ? cls : "main";
    classes[name] = d;
    for (auto& k : n->kids)
      if (k->tag == "default") parse_defaults(k.get(), &classes[name]);
  }

  Attrs resolve(const std::string& tag, const XNode* n, const std::string& cls) {
    Attrs a;
    const char* c = n->get("class");
    auto it = classes.find(c ? c : cls);
    if (it != classes.end()) {
      auto e = it->second.el.find(tag);
      if (e != it->second.el.end()) a = e->second;
    }
    for (auto& kv : n->attrs) a[kv.first] = kv.second;
    return a;
  }
  static std::vector<double> getv(const Attrs& a, const char* k, std::vector<double> def) {
    auto it = a.find(k);
    if (it == a.end()) return def;
    auto v = nums(it->second.c_str());
    for (size_t i = v.size(); i < def.size(); i++) v.push_back(def[i]);
    return v;
  }
  static std::string gets(const Attrs& a, const char* k, const char* def) {
    auto it = a.find(k);
    return it == a.end() ? def : it->second;
  }

  bool add_geom(const XNode* n, int body, const std::string& cls) {
    Attrs a = resolve("geom", n, cls);
    std::string t = gets(a, "type", "sphere");
    int type = t == "plane" ? GEOM_PLANE : t == "sphere" ? GEOM_SPHERE : t == "capsule" ? GEOM_CAPSULE : -1;
    if (type < 0) { err = "unsupported geom type '" + t + "'"; return false; }
    auto size = getv(a, "size", {0, 0, 0});
    double pos[3] = {0, 0, 0}, quat[4] = {1, 0, 0, 0};
    if (a.count("fromto")) {
      auto ft = nums(a["fromto"].c_str());
      if (ft.size() != 6) { err = "bad fromto"; return false; }
      double dv[3];
      for (int k = 0; k < 3; k++) { pos[k] = 0.5 * (ft[k] + ft[k + 3]); dv[k] = ft[k + 3] - ft[k]; }
      quat_z2vec(quat, dv);
      size[1] = 0.5 * std::sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
    } else {
      auto p = getv(a, "pos", {0, 0, 0});
      for (int k = 0; k < 3; k++) pos[k] = p[k];
      std::vector<double> z, q;
      if (a.count("zaxis")) {
        if (!numsn(a["zaxis"].c_str(), 3, "zaxis", z)) return false;
        quat_z2vec(quat, z.data());
      }
      if (a.count("quat")) {
        if (!numsn(a["quat"].c_str(), 4, "quat", q)) return false;
        double nq = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        if (!(nq > 0)) { err = "zero geom quat"; return false; }
        for (int k = 0; k < 4; k++) quat[k] = q[k] / nq;
      }
    }
    auto fr = getv(a, "friction", {1, 0.005, 0.0001});
    auto sr = getv(a, "solref", {0.02, 1});
    auto si = getv(a, "solimp", {0.9, 0.95, 0.001, 0.5, 2});
    m.geom_name.push_back(n->get("name") ? n->get("name") : "");
    m.geom_type.push_back(type);
    m.geom_bodyid.push_back(body);
    m.geom_condim.push_back((int)getv(a, "condim", {3})[0]);
    m.geom_contype.push_back((int)getv(a, "contype", {1})[0]);
    m.geom_conaffinity.push_back((int)getv(a, "conaffinity", {1})[0]);
    m.geom_priority.push_back((int)getv(a, "priority", {0})[0]);
    for (int k = 0; k < 3; k++) m.geom_size.push_back(k < (int)size.size() ? size[k] : 0);
    for (double x : pos) m.geom_pos.push_back(x);
    for (double x : quat) m.geom_quat.push_back(x);
    for (int k = 0; k < 3; k++) m.geom_friction.push_back(fr[k]);
    for (int k = 0; k < 2; k++) m.geom_solref.push_back(sr[k]);
    for (int k = 0; k < 5; k++) m.geom_solimp.push_back(si[k]);
    m.geom_margin.push_back(getv(a, "margin", {0})[0]);
    m.geom_gap.push_back(getv(a, "gap", {0})[0]);
    m.geom_solmix.push_back(getv(a, "solmix", {1})[0]);
    double r = size.empty() ? 0 : size[0];
    m.geom_rbound.push_back(type == GEOM_PLANE ? 0 : type == GEOM_SPHERE ? r : r + size[1]);
    geom_density.push_back(getv(a, "density", {1000})[0]);
    return true;
  }
  std::vector<double> geom_density;

  bool add_joint(const XNode* n, int body, const std::string& cls, bool free) {
    int id = (int)m.jnt_type.size();
    if (n->get("name")) jnt_by_name[n->get("name")] = id;
    m.jnt_name.push_back(n->get("name") ? n->get("name") : "");
    m.jnt_bodyid.push_back(body);
    if (free) {  // MJCF <freejoint>: stiffness/damping/armature forced to 0, no limits
      m.jnt_type.push_back(JNT_FREE);
      for (int k = 0; k < 3; k++) m.jnt_pos.push_back(0);
      m.jnt_axis.insert(m.jnt_axis.end(), {0, 0, 1});
      m.jnt_range.insert(m.jnt_range.end(), {0, 0});
      m.jnt_limited.push_back(0);
      m.jnt_stiffness.push_back(0);
      m.jnt_springref.push_back(0);
      m.jnt_solref.insert(m.jnt_solref.end(), {0.02, 1});
      m.jnt_solimp.insert(m.jnt_solimp.end(), {0.9, 0.95, 0.001, 0.5, 2});
      m.jnt_margin.push_back(0);
      jnt_damping.push_back(0);
      jnt_armature.push_back(0);
      return true;
    }
    Attrs a = resolve("joint", n, cls);
    std::string t = gets(a, "type", "hinge");
    if (t != "hinge") { err = "unsupported joint type '" + t + "'"; return false; }
    m.jnt_type.push_back(JNT_HINGE);
    auto p = getv(a, "pos", {0, 0, 0});
    auto ax = getv(a, "axis", {0, 0, 1});
    double an = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
    for (int k = 0; k < 3; k++) { m.jnt_pos.push_back(p[k]); m.jnt_axis.push_back(ax[k] / an); }
    auto rg = getv(a, "range", {0, 0});
    double lo = rg[0] * kPi / 180, hi = rg[1] * kPi / 180;   // compiler angle="degree" (default)
    m.jnt_range.push_back(lo);
    m.jnt_range.push_back(hi);
    std::string lim = gets(a, "limited", "auto");
    m.jnt_limited.push_back(lim == "true" || (lim == "auto" && lo < hi));
    m.jnt_stiffness.push_back(getv(a, "stiffness", {0})[0]);
    m.jnt_springref.push_back(getv(a, "springref", {0})[0] * kPi / 180);
    auto sr = getv(a, "solreflimit", {0.02, 1});
    auto si = getv(a, "solimplimit", {0.9, 0.95, 0.001, 0.5, 2});
    for (int k = 0; k < 2; k++) m.jnt_solref.push_back(sr[k]);
    for (int k = 0; k < 5; k++) m.jnt_solimp.push_back(si[k]);
    m.jnt_margin.push_back(getv(a, "margin", {0})[0]);
    jnt_damping.push_back(getv(a, "damping", {0})[0]);
    jnt_armature.push_back(getv(a, "armature", {0})[0]);
    return true;
  }
  std::vector<double> jnt_damping, jnt_armature;

  bool walk(const XNode* n, int parent, const std::string& cls) {
    for (auto& k : n->kids)
      if (k->tag == "geom" && !add_geom(k.get(), parent, cls)) return false;
    for (auto& k : n->kids) {
      if (k->tag != "body") continue;
      int id = (int)m.body_parentid.size();
      if (k->get("name")) body_by_name[k->get("name")] = id;
      m.body_name.push_back(k->get("name") ? k->get("name") : "");
      m.body_parentid.push_back(parent);
      std::vector<double> p, q;
      if (!numsn(k->get("pos") ? k->get("pos") : "0 0 0", 3, "pos", p) ||
          !numsn(k->get("quat") ? k->get("quat") : "1 0 0 0", 4, "quat", q))
        return false;
      if (k->get("euler") || k->get("axisangle") || k->get("xyaxes") || k->get("zaxis")) {
        err = "body orientation specifiers other than quat are not supported";
        return false;
      }
      double qn = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
      if (!(qn > 0)) { err = "zero body quat"; return false; }
      for (int j = 0; j < 3; j++) m.body_pos.push_back(p[j]);
      for (int j = 0; j < 4; j++) m.body_quat.push_back(q[j] / qn);
      std::string ccls = k->get("childclass") ? k->get("childclass") : cls;
      for (auto& j : k->kids) {
        if (j->tag == "freejoint" && !add_joint(j.get(), id, ccls, true)) return false;
        if (j->tag == "joint" && !add_joint(j.get(), id, ccls, false)) return false;
        if (j->tag == "inertial") { err = "<inertial> not supported (inertiafromgeom only)"; return false; }
      }
      if (!walk(k.get(), id, ccls)) return false;
    }
    return true;
  }

  // <option>: timestep, gravity, iterations, tolerance are honoured; anything that changes the
  // dynamics in a way the engine does not implement is rejected (never silently ignored).
  bool parse_option(const XNode* k) {
    if (k->get("timestep") && !num1(k->get("timestep"), "timestep", m.timestep)) return false;
    if (!(m.timestep > 0)) { err = "<option timestep> must be > 0"; return false; }
    if (k->get("gravity")) {
      auto g = nums(k->get("gravity"));
      if (g.size() != 3) { err = "<option gravity> needs 3 numbers"; return false; }
      for (int j = 0; j < 3; j++) m.gravity[j] = g[j];
    }
    double it = m.iterations;
    if (k->get("iterations") && !num1(k->get("iterations"), "iterations", it)) return false;
    if (!(it >= 1 && it <= 1e6)) { err = "<option iterations> must be in [1, 1e6]"; return false; }
    m.iterations = (int)it;
    if (k->get("tolerance") && !num1(k->get("tolerance"), "tolerance", m.tolerance)) return false;
    auto is = [&](const char* a, const char* dflt) { return !k->get(a) || std::string(k->get(a)) == dflt; };
    auto zero = [&](const char* a) {
      if (!k->get(a)) return true;
      for (double x : nums(k->get(a))) if (x != 0) return false;
      return true;
    };
    if (k->get("solver")) {
      const std::string sv = k->get("solver");
      if (sv == "Newton") m.solver = 0;
      else if (sv == "PGS") m.solver = 1;
      else { err = "only solver=\"Newton\" (MuJoCo default) or \"PGS\" is supported"; return false; }
    }
    if (!is("integrator", "Euler")) { err = "only integrator=\"Euler\" is supported (reference: MuJoCo default)"; return false; }
    if (!is("cone", "pyramidal")) { err = "only cone=\"pyramidal\" is supported"; return false; }
    double impratio = 1.0;
    if (k->get("impratio") && !num1(k->get("impratio"), "impratio", impratio)) return false;
    if (impratio != 1.0) { err = "only impratio=1 is supported"; return false; }
    if (!zero("noslip_iterations")) { err = "noslip solver not supported"; return false; }
    if (!zero("density") || !zero("viscosity")) { err = "fluid forces (density/viscosity) not supported"; return false; }
    for (auto& f : k->kids)
      if (f->tag == "flag")
        for (auto& a : f->attrs)
          if (a.first != "energy") { err = "<option><flag " + a.first + "> not supported"; return false; }
    return true;
  }

  bool run(const XNode* root) {
    if (root->tag != "mujoco") { err = "root element must be <mujoco>"; return false; }
    classes["main"] = DefClass();
    for (auto& k : root->kids) {
      if (k->tag == "default") parse_defaults(k.get(), nullptr);
      if (k->tag == "option" && !parse_option(k.get())) return false;
      if (k->tag == "compiler" && k->get("angle") && std::string(k->get("angle")) != "degree") {
        err = "compiler angle other than degree not supported";
        return false;
      }
    }
    m.body_name.push_back("world");
    m.body_parentid.push_back(-1);
    m.body_pos.insert(m.body_pos.end(), {0, 0, 0});
    m.body_quat.insert(m.body_quat.end(), {1, 0, 0, 0});
    body_by_name["world"] = 0;
    const XNode* wb = nullptr;
    for (auto& k : root->kids) if (k->tag == "worldbody") wb = k.get();
    if (!wb) { err = "missing <worldbody>"; return false; }
    if (!walk(wb, 0, "main")) return false;
    m.nbody = (int)m.body_parentid.size();
    m.njnt = (int)m.jnt_type.size();
    m.ngeom = (int)m.geom_type.size();
    return finish(root);
  }

  bool finish(const XNode* root);
};

bool Compiler::finish(const XNode* root) {
  int nb = m.nbody;
  // joint / dof addressing
  m.nq = m.nv = 0;
  for (int j = 0; j < m.njnt; j++) {
    m.jnt_qposadr.push_back(m.nq);
    m.jnt_dofadr.push_back(m.nv);
    int nd = m.jnt_type[j] == JNT_FREE ? 6 : 1;
    m.nq += m.jnt_type[j] == JNT_FREE ? 7 : 1;
    for (int k = 0; k < nd; k++) {
      m.dof_jntid.push_back(j);
      m.dof_bodyid.push_back(m.jnt_bodyid[j]);
      m.dof_damping.push_back(jnt_damping[j]);
      m.dof_armature.push_back(jnt_armature[j]);
    }
    m.nv += nd;
  }
  m.body_jntadr.assign(nb, -1); m.body_jntnum.assign(nb, 0);
  m.body_dofadr.assign(nb, -1); m.body_dofnum.assign(nb, 0);
  for (int j = 0; j < m.njnt; j++) {
    int b = m.jnt_bodyid[j];
    if (m.body_jntadr[b] < 0) m.body_jntadr[b] = j;
    m.body_jntnum[b]++;
  }
  for (int d = 0; d < m.nv; d++) {
    int b = m.dof_bodyid[d];
    if (m.body_dofadr[b] < 0) m.body_dofadr[b] = d;
    m.body_dofnum[b]++;
  }
  for (int b = 1; b < nb; b++)
    if (m.body_jntnum[b] > 1)
      for (int j = m.body_jntadr[b]; j < m.body_jntadr[b] + m.body_jntnum[b]; j++)
        if (m.jnt_type[j] == JNT_FREE) { err = "free joint must be the only joint of its body"; return false; }
  m.body_weldid.assign(nb, 0);
  m.body_rootid.assign(nb, 0);
  for (int b = 1; b < nb; b++) {
    int p = m.body_parentid[b];
    m.body_weldid[b] = m.body_jntnum[b] > 0 ? b : m.body_weldid[p];
    m.body_rootid[b] = p == 0 ? b : m.body_rootid[p];
  }
  m.dof_parentid.assign(m.nv, -1);
  std::vector<int> last(nb, -1);
  for (int b = 1; b < nb; b++) {
    int prev = last[m.body_parentid[b]];
    for (int k = 0; k < m.body_dofnum[b]; k++) {
      int d = m.body_dofadr[b] + k;
      m.dof_parentid[d] = prev;
      prev = d;
    }
    last[b] = prev;
  }
  // qpos0 / qpos_spring
  m.qpos0.assign(m.nq, 0);
  m.qpos_spring.assign(m.nq, 0);
  for (int j = 0; j < m.njnt; j++) {
    int a = m.jnt_qposadr[j], b = m.jnt_bodyid[j];
    if (m.jnt_type[j] == JNT_FREE) {
      for (int k = 0; k < 3; k++) m.qpos0[a + k] = m.body_pos[3 * b + k];
      for (int k = 0; k < 4; k++) m.qpos0[a + 3 + k] = m.body_quat[4 * b + k];
      for (int k = 0; k < 7; k++) m.qpos_spring[a + k] = m.qpos0[a + k];
    } else {
      m.qpos_spring[a] = m.jnt_springref[j];
    }
  }
  // mass properties (inertiafromgeom, exact solid capsule / sphere)
  m.body_mass.assign(nb, 0); m.body_ipos.assign(3 * nb, 0); m.body_iquat.assign(4 * nb, 0);
  m.body_inertia.assign(3 * nb, 0); m.body_inertia_full.assign(9 * nb, 0);
  for (int b = 0; b < nb; b++) m.body_iquat[4 * b] = 1;
  for (int b = 1; b < nb; b++) {
    std::vector<int> gs;
    for (int g = 0; g < m.ngeom; g++) if (m.geom_bodyid[g] == b) gs.push_back(g);
    std::vector<double> gm(gs.size()), gi(3 * gs.size());
    double mt = 0, com[3] = {0, 0, 0};
    for (size_t k = 0; k < gs.size(); k++) {
      int g = gs[k];
      double r = m.geom_size[3 * g], rho = geom_density[g];
      if (m.geom_type[g] == GEOM_SPHERE) {
        gm[k] = rho * 4.0 / 3.0 * kPi * r * r * r;
        gi[3 * k] = gi[3 * k + 1] = gi[3 * k + 2] = 0.4 * gm[k] * r * r;
      } else if (m.geom_type[g] == GEOM_CAPSULE) {
        double h = 2 * m.geom_size[3 * g + 1];
        double ms = rho * 4.0 / 3.0 * kPi * r * r * r, mc = rho * kPi * r * r * h;
        gm[k] = ms + mc;
        gi[3 * k] = gi[3 * k + 1] = mc * (3 * r * r + h * h) / 12 + ms * (0.4 * r * r + h * h / 4 + 3 * h * r / 8);
        gi[3 * k + 2] = mc * r * r / 2 + ms * 0.4 * r * r;
      }
      mt += gm[k];
      for (int c = 0; c < 3; c++) com[c] += gm[k] * m.geom_pos[3 * g + c];
    }
    if (mt < kMinVal) { err = "body '" + m.body_name[b] + "' has no mass"; return false; }
    for (double& c : com) c /= mt;
    double I[9] = {0};
    for (size_t k = 0; k < gs.size(); k++) {
      int g = gs[k];
      double R[9], dd[3];
      quat2mat(R, &m.geom_quat[4 * g]);
      for (int c = 0; c < 3; c++) dd[c] = m.geom_pos[3 * g + c] - com[c];
      double d2 = dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2];
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
          double v = 0;
          for (int k2 = 0; k2 < 3; k2++) v += R[3 * r + k2] * gi[3 * k + k2] * R[3 * c + k2];
          I[3 * r + c] += v + gm[k] * ((r == c ? d2 : 0) - dd[r] * dd[c]);
        }
    }
    double w[3], V[9];
    eig3(I, w, V);
    int ord[3] = {0, 1, 2};
    std::sort(ord, ord + 3, [&](int a, int c) { return w[a] > w[c]; });
    double Vs[9], ws[3];
    for (int c = 0; c < 3; c++) {
      ws[c] = w[ord[c]];
      for (int r = 0; r < 3; r++) Vs[3 * r + c] = V[3 * r + ord[c]];
    }
    double det = Vs[0] * (Vs[4] * Vs[8] - Vs[5] * Vs[7]) - Vs[1] * (Vs[3] * Vs[8] - Vs[5] * Vs[6]) +
                 Vs[2] * (Vs[3] * Vs[7] - Vs[4] * Vs[6]);
    if (det < 0) for (int r = 0; r < 3; r++) Vs[3 * r + 2] = -Vs[3 * r + 2];
    m.body_mass[b] = mt;
    for (int c = 0; c < 3; c++) { m.body_ipos[3 * b + c] = com[c]; m.body_inertia[3 * b + c] = ws[c]; }
    mat2quat(&m.body_iquat[4 * b], Vs);
    for (int k = 0; k < 9; k++) m.body_inertia_full[9 * b + k] = I[k];
  }
  m.body_subtreemass = m.body_mass;
  for (int b = nb - 1; b > 0; b--) m.body_subtreemass[m.body_parentid[b]] += m.body_subtreemass[b];

  // tendons (fixed), actuators (motor), excludes, keyframes
  for (auto& k : root->kids) {
    if (k->tag == "tendon") {
      for (auto& t : k->kids) {
        if (t->tag != "fixed") { err = "only fixed tendons supported"; return false; }
        Attrs a = resolve("tendon", t.get(), "main");
        m.tendon_name.push_back(t->get("name") ? t->get("name") : "");
        m.tendon_adr.push_back((int)m.wrap_jnt.size());
        int nw = 0;
        for (auto& w : t->kids) {
          if (w->tag != "joint") continue;
          auto it = jnt_by_name.find(w->get("joint") ? w->get("joint") : "");
          if (it == jnt_by_name.end()) { err = "tendon joint not found"; return false; }
          m.wrap_jnt.push_back(it->second);
          double coef = 1.0;
          if (w->get("coef") && !num1(w->get("coef"), "coef", coef)) return false;
          m.wrap_coef.push_back(coef);
          nw++;
        }
        m.tendon_num.push_back(nw);
        auto rg = getv(a, "range", {0, 0});
        m.tendon_range.push_back(rg[0]);
        m.tendon_range.push_back(rg[1]);
        std::string lim = gets(a, "limited", "auto");
        m.tendon_limited.push_back(lim == "true" || (lim == "auto" && rg[0] < rg[1]));
        auto sr = getv(a, "solreflimit", {0.02, 1});
        auto si = getv(a, "solimplimit", {0.9, 0.95, 0.001, 0.5, 2});
        for (int j = 0; j < 2; j++) m.tendon_solref.push_back(sr[j]);
        for (int j = 0; j < 5; j++) m.tendon_solimp.push_back(si[j]);
        m.tendon_margin.push_back(getv(a, "margin", {0})[0]);
      }
    }
    if (k->tag == "actuator") {
      for (auto& u : k->kids) {
        if (u->tag != "motor") { err = "only <motor> actuators supported"; return false; }
        Attrs a = resolve("motor", u.get(), "main");
        auto it = jnt_by_name.find(u->get("joint") ? u->get("joint") : "");
        if (it == jnt_by_name.end()) { err = "motor joint not found"; return false; }
        m.actuator_name.push_back(u->get("name") ? u->get("name") : "");
        m.actuator_trnid.push_back(it->second);
        m.actuator_gear.push_back(getv(a, "gear", {1})[0]);
        auto cr = getv(a, "ctrlrange", {0, 0});
        m.actuator_ctrlrange.push_back(cr[0]);
        m.actuator_ctrlrange.push_back(cr[1]);
        std::string lim = gets(a, "ctrllimited", "auto");
        m.actuator_ctrllimited.push_back(lim == "true" || (lim == "auto" && cr[0] < cr[1]));
      }
    }
    if (k->tag == "contact") {
      for (auto& e : k->kids) {
        if (e->tag != "exclude") continue;
        const char* n1 = e->get("body1");
        const char* n2 = e->get("body2");
        int b1 = n1 && body_by_name.count(n1) ? body_by_name[n1] : -1;
        int b2 = n2 && body_by_name.count(n2) ? body_by_name[n2] : -1;
        if (b1 < 0 || b2 < 0) { err = "exclude body not found"; return false; }
        m.exclude.emplace_back(std::min(b1, b2), std::max(b1, b2));
      }
    }
    if (k->tag == "keyframe")
      for (auto& e : k->kids)
        if (e->get("qpos")) {
          std::vector<double> kq;
          if (!numsn(e->get("qpos"), (size_t)m.nq, "key qpos", kq)) return false;
          m.keyframes[e->get("name") ? e->get("name") : ""] = kq;
        }
  }
  m.ntendon = (int)m.tendon_adr.size();
  m.nu = (int)m.actuator_trnid.size();

  // static collision candidates (mj_collision filters), canonical order
  std::set<std::pair<int, int>> excl(m.exclude.begin(), m.exclude.end());
  std::vector<std::tuple<int, int, int, int>> pairs;
  for (int g1 = 0; g1 < m.ngeom; g1++)
    for (int g2 = g1 + 1; g2 < m.ngeom; g2++) {
      int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
      if (!((m.geom_contype[g1] & m.geom_conaffinity[g2]) || (m.geom_contype[g2] & m.geom_conaffinity[g1]))) continue;
      int w1 = m.body_weldid[b1], w2 = m.body_weldid[b2];
      if (w1 == w2) continue;
      int wp1 = w1 ? m.body_weldid[m.body_parentid[w1]] : 0, wp2 = w2 ? m.body_weldid[m.body_parentid[w2]] : 0;
      if (w1 && w2 && (w1 == wp2 || w2 == wp1)) continue;
      if (excl.count({std::min(b1, b2), std::max(b1, b2)})) continue;
      int lo = b1 <= b2 ? g1 : g2, hi = b1 <= b2 ? g2 : g1;
      pairs.emplace_back(std::min(b1, b2), std::max(b1, b2), lo, hi);
    }
  std::sort(pairs.begin(), pairs.end());
  for (auto& p : pairs) m.pair_geom.emplace_back(std::get<2>(p), std::get<3>(p));

  // mj_setConst at qpos0: kinematics, com, cdof, CRB -> M; invweights from M^-1
  int nv = m.nv;
  std::vector<double> xpos(3 * nb, 0), xquat(4 * nb, 0), xmat(9 * nb, 0), xipos(3 * nb, 0);
  std::vector<double> xanc(3 * m.njnt), xax(3 * m.njnt);
  xquat[0] = 1;
  for (int b = 1; b < nb; b++) {
    int ja = m.body_jntadr[b], jn = m.body_jntnum[b], p = m.body_parentid[b];
    double pos[3], q[4];
    if (jn == 1 && m.jnt_type[ja] == JNT_FREE) {
      int qa = m.jnt_qposadr[ja];
      for (int k = 0; k < 3; k++) pos[k] = m.qpos0[qa + k];
      for (int k = 0; k < 4; k++) q[k] = m.qpos0[qa + 3 + k];
      for (int k = 0; k < 3; k++) { xanc[3 * ja + k] = pos[k]; xax[3 * ja + k] = m.jnt_axis[3 * ja + k]; }
    } else {
      double R[9];
      quat2mat(R, &xquat[4 * p]);
      mv3(pos, R, &m.body_pos[3 * b]);
      for (int k = 0; k < 3; k++) pos[k] += xpos[3 * p + k];
      quat_mul(q, &xquat[4 * p], &m.body_quat[4 * b]);
      for (int j = ja; j < ja + jn; j++) {   // qpos == qpos0: no joint rotation
        double Rq[9];
        quat2mat(Rq, q);
        mv3(&xax[3 * j], Rq, &m.jnt_axis[3 * j]);
        mv3(&xanc[3 * j], Rq, &m.jnt_pos[3 * j]);
        for (int k = 0; k < 3; k++) xanc[3 * j + k] += pos[k];
      }
    }
    double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int k = 0; k < 4; k++) xquat[4 * b + k] = q[k] / n;
    for (int k = 0; k < 3; k++) xpos[3 * b + k] = pos[k];
    quat2mat(&xmat[9 * b], &xquat[4 * b]);
    mv3(&xipos[3 * b], &xmat[9 * b], &m.body_ipos[3 * b]);
    for (int k = 0; k < 3; k++) xipos[3 * b + k] += pos[k];
  }
  std::vector<double> sub(3 * nb, 0);
  for (int b = 0; b < nb; b++) for (int k = 0; k < 3; k++) sub[3 * b + k] = m.body_mass[b] * xipos[3 * b + k];
  for (int b = nb - 1; b > 0; b--) for (int k = 0; k < 3; k++) sub[3 * m.body_parentid[b] + k] += sub[3 * b + k];
  for (int b = 0; b < nb; b++)
    for (int k = 0; k < 3; k++)
      sub[3 * b + k] = m.body_subtreemass[b] < kMinVal ? xipos[3 * b + k] : sub[3 * b + k] / m.body_subtreemass[b];
  std::vector<double> cdof(6 * nv, 0);
  for (int j = 0; j < m.njnt; j++) {
    int b = m.jnt_bodyid[j], da = m.jnt_dofadr[j], rt = m.body_rootid[b];
    double off[3];
    for (int k = 0; k < 3; k++) off[k] = sub[3 * rt + k] - xanc[3 * j + k];
    if (m.jnt_type[j] == JNT_FREE) {
      for (int i = 0; i < 3; i++) cdof[6 * (da + i) + 3 + i] = 1;
      for (int i = 0; i < 3; i++) {
        double ax[3] = {xmat[9 * b + i], xmat[9 * b + 3 + i], xmat[9 * b + 6 + i]};
        for (int k = 0; k < 3; k++) cdof[6 * (da + 3 + i) + k] = ax[k];
        cross(&cdof[6 * (da + 3 + i) + 3], ax, off);
      }
    } else {
      for (int k = 0; k < 3; k++) cdof[6 * da + k] = xax[3 * j + k];
      cross(&cdof[6 * da + 3], &xax[3 * j], off);
    }
  }
  // 6x6 spatial inertia per body about root subtree com, composite
  std::vector<double> I6(36 * nb, 0);
  for (int b = 1; b < nb; b++) {
    double R[9], T[9], Ic[9], d[3];
    std::memcpy(R, &xmat[9 * b], sizeof R);
    const double* Ib = &m.body_inertia_full[9 * b];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) T[3 * r + c] = R[3 * r] * Ib[c] + R[3 * r + 1] * Ib[3 + c] + R[3 * r + 2] * Ib[6 + c];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) Ic[3 * r + c] = T[3 * r] * R[3 * c] + T[3 * r + 1] * R[3 * c + 1] + T[3 * r + 2] * R[3 * c + 2];
    for (int k = 0; k < 3; k++) d[k] = xipos[3 * b + k] - sub[3 * m.body_rootid[b] + k];
    double mass = m.body_mass[b], d2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    double cx[9] = {0, -d[2], d[1], d[2], 0, -d[0], -d[1], d[0], 0};
    double* S = &I6[36 * b];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        S[6 * r + c] = Ic[3 * r + c] + mass * ((r == c ? d2 : 0) - d[r] * d[c]);
        S[6 * r + 3 + c] = mass * cx[3 * r + c];
        S[6 * (3 + r) + c] = -mass * cx[3 * r + c];
        S[6 * (3 + r) + 3 + c] = r == c ? mass : 0;
      }
  }
  for (int b = nb - 1; b > 0; b--)
    if (m.body_parentid[b] > 0)
      for (int k = 0; k < 36; k++) I6[36 * m.body_parentid[b] + k] += I6[36 * b + k];
  std::vector<double> M(nv * nv, 0);
  for (int i = 0; i < nv; i++) {
    double buf[6] = {0};
    const double* S = &I6[36 * m.dof_bodyid[i]];
    for (int r = 0; r < 6; r++) for (int c = 0; c < 6; c++) buf[r] += S[6 * r + c] * cdof[6 * i + c];
    for (int j = i; j >= 0; j = m.dof_parentid[j]) {
      double v = 0;
      for (int k = 0; k < 6; k++) v += cdof[6 * j + k] * buf[k];
      M[i * nv + j] = M[j * nv + i] = v;
    }
    M[i * nv + i] += m.dof_armature[i];
  }
  // inverse via Gauss-Jordan
  std::vector<double> A = M, Minv(nv * nv, 0);
  for (int i = 0; i < nv; i++) Minv[i * nv + i] = 1;
  for (int c = 0; c < nv; c++) {
    int piv = c;
    for (int r = c + 1; r < nv; r++) if (std::fabs(A[r * nv + c]) > std::fabs(A[piv * nv + c])) piv = r;
    if (std::fabs(A[piv * nv + c]) < 1e-300) { err = "singular mass matrix at qpos0"; return false; }
    for (int k = 0; k < nv; k++) { std::swap(A[c * nv + k], A[piv * nv + k]); std::swap(Minv[c * nv + k], Minv[piv * nv + k]); }
    double inv = 1 / A[c * nv + c];
    for (int k = 0; k < nv; k++) { A[c * nv + k] *= inv; Minv[c * nv + k] *= inv; }
    for (int r = 0; r < nv; r++) {
      if (r == c) continue;
      double f = A[r * nv + c];
      if (f == 0) continue;
      for (int k = 0; k < nv; k++) { A[r * nv + k] -= f * A[c * nv + k]; Minv[r * nv + k] -= f * Minv[c * nv + k]; }
    }
  }
  m.body_invweight0.assign(2 * nb, 0);
  for (int b = 1; b < nb; b++) {
    std::vector<double> jp(3 * nv, 0), jr(3 * nv, 0);
    double off[3];
    for (int k = 0; k < 3; k++) off[k] = xipos[3 * b + k] - sub[3 * m.body_rootid[b] + k];
    int dof = -1;
    for (int bb = b; bb > 0 && dof < 0; bb = m.body_parentid[bb])
      if (m.body_dofnum[bb]) dof = m.body_dofadr[bb] + m.body_dofnum[bb] - 1;
    for (; dof >= 0; dof = m.dof_parentid[dof]) {
      double t[3];
      cross(t, &cdof[6 * dof], off);
      for (int k = 0; k < 3; k++) { jr[k * nv + dof] = cdof[6 * dof + k]; jp[k * nv + dof] = cdof[6 * dof + 3 + k] + t[k]; }
    }
    double tt = 0, tr = 0;
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < nv; i++)
        for (int j = 0; j < nv; j++) {
          tt += jp[k * nv + i] * Minv[i * nv + j] * jp[k * nv + j];
          tr += jr[k * nv + i] * Minv[i * nv + j] * jr[k * nv + j];
        }
    m.body_invweight0[2 * b] = std::max(kMinVal, tt / 3);
    m.body_invweight0[2 * b + 1] = std::max(kMinVal, tr / 3);
  }
  m.dof_invweight0.assign(nv, 0);
  for (int j = 0; j < m.njnt; j++) {
    int da = m.jnt_dofadr[j];
    if (m.jnt_type[j] == JNT_FREE) {
      double t = (Minv[da * nv + da] + Minv[(da + 1) * nv + da + 1] + Minv[(da + 2) * nv + da + 2]) / 3;
      double r = (Minv[(da + 3) * nv + da + 3] + Minv[(da + 4) * nv + da + 4] + Minv[(da + 5) * nv + da + 5]) / 3;
      for (int k = 0; k < 3; k++) { m.dof_invweight0[da + k] = t; m.dof_invweight0[da + 3 + k] = r; }
    } else {
      m.dof_invweight0[da] = Minv[da * nv + da];
    }
  }
  m.tendon_invweight0.assign(m.ntendon, 0);
  for (int t = 0; t < m.ntendon; t++) {
    std::vector<double> J(nv, 0);
    for (int w = m.tendon_adr[t]; w < m.tendon_adr[t] + m.tendon_num[t]; w++) J[m.jnt_dofadr[m.wrap_jnt[w]]] += m.wrap_coef[w];
    double v = 0;
    for (int i = 0; i < nv; i++) for (int j = 0; j < nv; j++) v += J[i] * Minv[i * nv + j] * J[j];
    m.tendon_invweight0[t] = v;
  }
  double tr = 0;
  for (int i = 0; i < nv; i++) tr += M[i * nv + i];
  m.meaninertia = tr / nv;
  return true;
}

}  // namespace

bool compile_mjcf_file(const std::string& path, HostModel& out, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) { err = "cannot open file '" + path + "'"; return false; }
  std::stringstream ss;
  ss << f.rdbuf();
  std::string src = ss.str();
  XParser p(src);
  auto root = p.element();
  if (!root) { err = "XML parse error: " + p.err; return false; }
  out = HostModel();
  Compiler c(out, err);
  return c.run(root.get());
}

int model_field(const HostModel& m, const std::string& name, double* out, int n) {
  std::vector<double> v;
  auto I = [&](const std::vector<int>& x) { v.assign(x.begin(), x.end()); };
  auto Dv = [&](const std::vector<double>& x) { v = x; };
  if (name == "nq") v = {(double)m.nq};
  else if (name == "nv") v = {(double)m.nv};
  else if (name == "nu") v = {(double)m.nu};
  else if (name == "nbody") v = {(double)m.nbody};
  else if (name == "njnt") v = {(double)m.njnt};
  else if (name == "ngeom") v = {(double)m.ngeom};
  else if (name == "ntendon") v = {(double)m.ntendon};
  else if (name == "opt_timestep") v = {m.timestep};
  else if (name == "opt_gravity") v = {m.gravity[0], m.gravity[1], m.gravity[2]};
  else if (name == "opt_iterations") v = {(double)m.iterations};
  else if (name == "opt_tolerance") v = {m.tolerance};
  else if (name == "opt_solver") v = {(double)m.solver};
  else if (name == "stat_meaninertia") v = {m.meaninertia};
  else if (name == "body_parentid") I(m.body_parentid);
  else if (name == "body_rootid") I(m.body_rootid);
  else if (name == "body_weldid") I(m.body_weldid);
  else if (name == "body_jntadr") I(m.body_jntadr);
  else if (name == "body_jntnum") I(m.body_jntnum);
  else if (name == "body_dofadr") I(m.body_dofadr);
  else if (name == "body_dofnum") I(m.body_dofnum);
  else if (name == "body_pos") Dv(m.body_pos);
  else if (name == "body_quat") Dv(m.body_quat);
  else if (name == "body_ipos") Dv(m.body_ipos);
  else if (name == "body_iquat") Dv(m.body_iquat);
  else if (name == "body_inertia") Dv(m.body_inertia);
  else if (name == "body_inertia_full") Dv(m.body_inertia_full);
  else if (name == "body_mass") Dv(m.body_mass);
  else if (name == "body_subtreemass") Dv(m.body_subtreemass);
  else if (name == "body_invweight0") Dv(m.body_invweight0);
  else if (name == "jnt_type") I(m.jnt_type);
  else if (name == "jnt_qposadr") I(m.jnt_qposadr);
  else if (name == "jnt_dofadr") I(m.jnt_dofadr);
  else if (name == "jnt_bodyid") I(m.jnt_bodyid);
  else if (name == "jnt_limited") I(m.jnt_limited);
  else if (name == "jnt_pos") Dv(m.jnt_pos);
  else if (name == "jnt_axis") Dv(m.jnt_axis);
  else if (name == "jnt_range") Dv(m.jnt_range);
  else if (name == "jnt_stiffness") Dv(m.jnt_stiffness);
  else if (name == "jnt_solref") Dv(m.jnt_solref);
  else if (name == "jnt_solimp") Dv(m.jnt_solimp);
  else if (name == "dof_bodyid") I(m.dof_bodyid);
  else if (name == "dof_jntid") I(m.dof_jntid);
  else if (name == "dof_parentid") I(m.dof_parentid);
  else if (name == "dof_armature") Dv(m.dof_armature);
  else if (name == "dof_damping") Dv(m.dof_damping);
  else if (name == "dof_invweight0") Dv(m.dof_invweight0);
  else if (name == "qpos0") Dv(m.qpos0);
  else if (name == "qpos_spring") Dv(m.qpos_spring);
  else if (name == "geom_type") I(m.geom_type);
  else if (name == "geom_bodyid") I(m.geom_bodyid);
  else if (name == "geom_condim") I(m.geom_condim);
  else if (name == "geom_size") Dv(m.geom_size);
  else if (name == "geom_pos") Dv(m.geom_pos);
  else if (name == "geom_quat") Dv(m.geom_quat);
  else if (name == "geom_friction") Dv(m.geom_friction);
  else if (name == "geom_solref") Dv(m.geom_solref);
  else if (name == "geom_solimp") Dv(m.geom_solimp);
  else if (name == "geom_rbound") Dv(m.geom_rbound);
  else if (name == "tendon_adr") I(m.tendon_adr);
  else if (name == "tendon_num") I(m.tendon_num);
  else if (name == "tendon_range") Dv(m.tendon_range);
  else if (name == "tendon_invweight0") Dv(m.tendon_invweight0);
  else if (name == "wrap_jnt") I(m.wrap_jnt);
  else if (name == "wrap_coef") Dv(m.wrap_coef);
  else if (name == "actuator_trnid") I(m.actuator_trnid);
  else if (name == "actuator_gear") Dv(m.actuator_gear);
  else if (name == "actuator_ctrlrange") Dv(m.actuator_ctrlrange);
  else if (name == "actuator_ctrllimited") I(m.actuator_ctrllimited);
  else if (name == "contact_bound") {
    const ContactBound cb = contact_bound(m);
    v = {(double)cb.con_all, (double)cb.efc_all, (double)cb.con_floor, (double)cb.efc_floor};
  }
  else if (name == "collision_pairs") { for (auto& p : m.pair_geom) { v.push_back(p.first); v.push_back(p.second); } }
  else if (name.rfind("key_", 0) == 0) {
    auto it = m.keyframes.find(name.substr(4));
    if (it == m.keyframes.end()) return -1;
    v = it->second;
  } else return -1;
  int cnt = (int)v.size();
  if (out && n >= cnt) std::copy(v.begin(), v.end(), out);
  return cnt;
}

// device solimp: the 5 MuJoCo values + 1/width, 1/mid^(p-1), 1/(1-mid)^(p-1) (getimpedance's
// constant denominators, mj_makeImpedance)
template <typename T>
void fill_solimp(T (&dst)[SOLIMP], const double* si) {
  for (int k = 0; k < 5; k++) dst[k] = (T)si[k];
  dst[5] = (T)(si[2] > 0 ? 1.0 / si[2] : 0.0);
  dst[6] = (T)(1.0 / std::pow(si[3], si[4] - 1));
  dst[7] = (T)(1.0 / std::pow(1 - si[3], si[4] - 1));
}

ContactBound contact_bound(const HostModel& m) {
  ContactBound b{0, 0, 0, 0};
  int nlim = 0;
  for (int j = 0; j < m.njnt; j++) nlim += (m.jnt_limited[j] && m.jnt_type[j] == JNT_HINGE) ? 1 : 0;
  for (int t = 0; t < m.ntendon; t++) nlim += m.tendon_limited[t] ? 1 : 0;
  for (const auto& pr : m.pair_geom) {
    const int g1 = pr.first, g2 = pr.second, t1 = m.geom_type[g1], t2 = m.geom_type[g2];
    const bool plane = t1 == GEOM_PLANE || t2 == GEOM_PLANE;
    const bool caps = t1 == GEOM_CAPSULE || t2 == GEOM_CAPSULE;
    // narrow phase maxima (collide_pair): plane-capsule and capsule-capsule 2, sphere pairs 1
    const int ncon = (caps && (plane || (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE))) ? 2 : 1;
    int dim;
    if (m.geom_priority[g1] != m.geom_priority[g2])
      dim = m.geom_condim[m.geom_priority[g1] > m.geom_priority[g2] ? g1 : g2];
    else
      dim = std::max(m.geom_condim[g1], m.geom_condim[g2]);
    const int rows = dim == 1 ? 1 : 2 * (dim - 1);       // pyramidal cone: 2 (condim - 1) edges
    b.con_all += ncon;
    b.efc_all += ncon * rows;
    if (plane) {
      b.con_floor += ncon;
      b.efc_floor += ncon * rows;
    }
  }
  b.efc_all += nlim;
  b.efc_floor += nlim;
  return b;
}

template <typename T>
bool build_dev_model(const HostModel& m, DevModel<T>& d, std::string& err) {
  std::memset(&d, 0, sizeof d);
  char buf[256];
  auto cap = [&](const char* what, int n, int mx) {
    if (n > mx) { std::snprintf(buf, sizeof buf, "model exceeds engine capacity: %s = %d > %d", what, n, mx); err = buf; return false; }
    return true;
  };
  if (!cap("nbody", m.nbody, MAXBODY) || !cap("nv", m.nv, MAXDOF) || !cap("nq", m.nq, MAXQ) ||
      !cap("njnt", m.njnt, MAXJNT) || !cap("ngeom", m.ngeom, MAXGEOM) || !cap("ntendon", m.ntendon, MAXTEN) ||
      !cap("nu", m.nu, MAXU) || !cap("npair", (int)m.pair_geom.size(), MAXPAIR))
    return false;
  {   // every geom resting on the floor at once must fit the wide tier (contacts are dropped only
      // past it, and only in body-body pile-ups on top of a flat-lying body)
    const ContactBound cb = contact_bound(m);
    if (!cap("contacts with every geom on the floor", cb.con_floor, MAXCON_WIDE) ||
        !cap("constraint rows with every geom on the floor", cb.efc_floor, MAXEFC_WIDE))
      return false;
  }
  for (int b = 1; b < m.nbody; b++)
    if (m.body_rootid[b] != m.body_rootid[1]) { err = "engine supports a single kinematic tree under world"; return false; }
  for (int b = 1; b < m.nbody; b++) {   // kernel keeps a body's joint rotations in registers
    int ja = m.body_jntadr[b], jn = m.body_jntnum[b];
    bool has_free = false;
    for (int j = ja; j < ja + jn; j++) has_free |= m.jnt_type[j] == JNT_FREE;
    if (has_free && jn != 1) { err = "a free joint must be its body's only joint"; return false; }
    if (!has_free && !cap("hinge joints per body", jn, MAXJPB)) return false;
  }
  d.nq = m.nq; d.nv = m.nv; d.nu = m.nu; d.nbody = m.nbody; d.njnt = m.njnt; d.ngeom = m.ngeom;
  d.ntendon = m.ntendon; d.npair = (int)m.pair_geom.size();
  d.timestep = (T)m.timestep;
  for (int k = 0; k < 3; k++) d.gravity[k] = (T)m.gravity[k];
  d.newton_scale = (T)(1.0 / (m.meaninertia * std::max(1, m.nv)));
  d.pgs_tol = (T)m.tolerance;
  d.total_mass = (T)m.body_subtreemass[0];
  // levels by depth
  std::vector<int> depth(m.nbody, 0);
  int maxd = 0;
  for (int b = 1; b < m.nbody; b++) { depth[b] = depth[m.body_parentid[b]] + 1; maxd = std::max(maxd, depth[b]); }
  if (!cap("tree depth", maxd, MAXLEVEL)) return false;
  d.nlevel = maxd;
  int n = 0;
  for (int L = 1; L <= maxd; L++) {
    d.level_adr[L - 1] = n;
    for (int b = 1; b < m.nbody; b++) if (depth[b] == L) d.level_body[n++] = b;
  }
  d.level_adr[maxd] = n;
  for (int b = 0; b < m.nbody; b++) {
    d.body_parentid[b] = m.body_parentid[b];
    d.body_depth[b] = depth[b];
    d.body_jntadr[b] = m.body_jntadr[b];
    d.body_jntnum[b] = m.body_jntnum[b];
    d.body_dofadr[b] = m.body_dofadr[b];
    d.body_dofnum[b] = m.body_dofnum[b];
    for (int k = 0; k < 3; k++) { d.body_pos[b][k] = (T)m.body_pos[3 * b + k]; d.body_ipos[b][k] = (T)m.body_ipos[3 * b + k]; }
    for (int k = 0; k < 4; k++) d.body_quat[b][k] = (T)m.body_quat[4 * b + k];
    const double* I = &m.body_inertia_full[9 * b];
    d.body_inert[b][0] = (T)I[0]; d.body_inert[b][1] = (T)I[4]; d.body_inert[b][2] = (T)I[8];
    d.body_inert[b][3] = (T)I[1]; d.body_inert[b][4] = (T)I[2]; d.body_inert[b][5] = (T)I[5];
    d.body_mass[b] = (T)m.body_mass[b];
    d.body_invweight_tran[b] = (T)m.body_invweight0[2 * b];
    uint32_t chain = 0;
    for (int bb = b; bb > 0; bb = m.body_parentid[bb])
      for (int k = 0; k < m.body_dofnum[bb]; k++) chain |= 1u << (m.body_dofadr[bb] + k);
    d.body_chainmask[b] = chain;
    uint32_t desc = 0;
    for (int c = 0; c < m.nbody; c++)
      for (int bb = c; bb >= 0; bb = bb ? m.body_parentid[bb] : -1)
        if (bb == b) { desc |= 1u << c; break; }
    d.body_descmask[b] = desc;
  }
  for (int j = 0; j < m.njnt; j++) {
    d.jnt_type[j] = m.jnt_type[j];
    d.jnt_qposadr[j] = m.jnt_qposadr[j];
    d.jnt_dofadr[j] = m.jnt_dofadr[j];
    d.jnt_bodyid[j] = m.jnt_bodyid[j];
    d.jnt_limited[j] = m.jnt_limited[j] && m.jnt_type[j] == JNT_HINGE;
    for (int k = 0; k < 3; k++) { d.jnt_pos[j][k] = (T)m.jnt_pos[3 * j + k]; d.jnt_axis[j][k] = (T)m.jnt_axis[3 * j + k]; }
    for (int k = 0; k < 2; k++) { d.jnt_range[j][k] = (T)m.jnt_range[2 * j + k]; d.jnt_solref[j][k] = (T)m.jnt_solref[2 * j + k]; }
    fill_solimp(d.jnt_solimp[j], &m.jnt_solimp[5 * j]);
    d.jnt_margin[j] = (T)m.jnt_margin[j];
  }
  for (int i = 0; i < m.nv; i++) {
    int j = m.dof_jntid[i];
    d.dof_bodyid[i] = m.dof_bodyid[i];
    d.dof_jntid[i] = j;
    d.dof_qposadr[i] = m.jnt_type[j] == JNT_HINGE ? m.jnt_qposadr[j] : -1;
    uint32_t anc = 0;
    for (int k = i; k >= 0; k = m.dof_parentid[k]) anc |= 1u << k;
    d.dof_ancmask[i] = anc;
    d.dof_relmask[i] = anc;
    for (int k = 0; k < i; k++)      // i is a descendant of each of its ancestors k
      if ((anc >> k) & 1u) d.dof_relmask[k] |= 1u << i;
    // mj_comVel: a hinge sees the velocity of all its dof ancestors; the 3 rotational dofs of
    // a free joint all see the velocity after its 3 translational dofs; translations see none.
    uint32_t dot = 0;
    if (m.jnt_type[j] == JNT_HINGE) {
      dot = anc & ~(1u << i);
    } else if (i - m.jnt_dofadr[j] >= 3) {           // free rotation: parent chain + 3 translations
      int da = m.jnt_dofadr[j];
      for (int k = m.dof_parentid[da]; k >= 0; k = m.dof_parentid[k]) dot |= 1u << k;
      dot |= 7u << da;
    }                                                 // free translation: cdof_dot == 0
    d.dof_dotmask[i] = dot;
    d.dof_armature[i] = (T)m.dof_armature[i];
    d.dof_damping[i] = (T)m.dof_damping[i];
    d.dof_invweight0[i] = (T)m.dof_invweight0[i];
    d.dof_stiffness[i] = m.jnt_type[j] == JNT_HINGE ? (T)m.jnt_stiffness[j] : T(0);
    d.dof_springref[i] = m.jnt_type[j] == JNT_HINGE ? (T)m.qpos_spring[m.jnt_qposadr[j]] : T(0);
    d.dof_actuator[i] = -1;
  }
  for (int u = 0; u < m.nu; u++) {
    int dof = m.jnt_dofadr[m.actuator_trnid[u]];
    if (m.jnt_type[m.actuator_trnid[u]] != JNT_HINGE) { err = "motors must drive hinge joints"; return false; }
    if (d.dof_actuator[dof] >= 0) { err = "at most one motor per joint supported"; return false; }
    d.dof_actuator[dof] = u;
    d.act_dof[u] = dof;
    d.act_gear[u] = (T)m.actuator_gear[u];
    d.act_ctrllimited[u] = m.actuator_ctrllimited[u];
    d.act_ctrlrange[u][0] = (T)m.actuator_ctrlrange[2 * u];
    d.act_ctrlrange[u][1] = (T)m.actuator_ctrlrange[2 * u + 1];
  }
  for (int g = 0; g < m.ngeom; g++) {
    d.geom_type[g] = m.geom_type[g];
    d.geom_bodyid[g] = m.geom_bodyid[g];
    double R[9];
    quat2mat(R, &m.geom_quat[4 * g]);
    for (int k = 0; k < 3; k++) { d.geom_pos[g][k] = (T)m.geom_pos[3 * g + k]; d.geom_zaxis[g][k] = (T)R[3 * k + 2]; }
    d.geom_size[g][0] = (T)m.geom_size[3 * g];
    d.geom_size[g][1] = (T)m.geom_size[3 * g + 1];
  }
  for (size_t p = 0; p < m.pair_geom.size(); p++) {
    int g1 = m.pair_geom[p].first, g2 = m.pair_geom[p].second;
    if (m.geom_type[g1] > m.geom_type[g2]) std::swap(g1, g2);
    int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
    int fn = -1;
    if (t1 == GEOM_PLANE && t2 == GEOM_SPHERE) fn = PAIR_PLANE_SPHERE;
    else if (t1 == GEOM_PLANE && t2 == GEOM_CAPSULE) fn = PAIR_PLANE_CAPSULE;
    else if (t1 == GEOM_SPHERE && t2 == GEOM_SPHERE) fn = PAIR_SPHERE_SPHERE;
    else if (t1 == GEOM_SPHERE && t2 == GEOM_CAPSULE) fn = PAIR_SPHERE_CAPSULE;
    else if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) fn = PAIR_CAPSULE_CAPSULE;
    if (fn < 0) { err = "unsupported collision pair (plane-plane)"; return false; }
    d.pair_g1[p] = g1; d.pair_g2[p] = g2; d.pair_fn[p] = fn;
    d.pair_b1[p] = m.geom_bodyid[g1]; d.pair_b2[p] = m.geom_bodyid[g2];
    // mj_contactParam (equal priority: max condim/friction, solmix-weighted solref/solimp)
    double mu, sr[2], si[5];
    int dim;
    if (m.geom_priority[g1] != m.geom_priority[g2]) {
      int g = m.geom_priority[g1] > m.geom_priority[g2] ? g1 : g2;
      dim = m.geom_condim[g]; mu = m.geom_friction[3 * g];
      for (int k = 0; k < 2; k++) sr[k] = m.geom_solref[2 * g + k];
      for (int k = 0; k < 5; k++) si[k] = m.geom_solimp[5 * g + k];
    } else {
      dim = std::max(m.geom_condim[g1], m.geom_condim[g2]);
      mu = std::max(m.geom_friction[3 * g1], m.geom_friction[3 * g2]);
      double s1 = m.geom_solmix[g1], s2 = m.geom_solmix[g2], mix;
      if (s1 >= kMinVal && s2 >= kMinVal) mix = s1 / (s1 + s2);
      else if (s1 < kMinVal && s2 < kMinVal) mix = 0.5;
      else mix = s1 < kMinVal ? 0.0 : 1.0;
      for (int k = 0; k < 2; k++)
        sr[k] = (m.geom_solref[2 * g1] > 0 && m.geom_solref[2 * g2] > 0)
                    ? mix * m.geom_solref[2 * g1 + k] + (1 - mix) * m.geom_solref[2 * g2 + k]
                    : std::min(m.geom_solref[2 * g1 + k], m.geom_solref[2 * g2 + k]);
      for (int k = 0; k < 5; k++) si[k] = mix * m.geom_solimp[5 * g1 + k] + (1 - mix) * m.geom_solimp[5 * g2 + k];
    }
    if (dim != 1 && dim != 3) { err = "only condim 1 and 3 supported"; return false; }
    d.pair_dim[p] = dim;
    d.pair_info[p][0] = g1; d.pair_info[p][1] = g2; d.pair_info[p][2] = fn; d.pair_info[p][3] = dim;
    d.pair_size[p][0] = (T)m.geom_size[3 * g1]; d.pair_size[p][1] = (T)m.geom_size[3 * g1 + 1];
    d.pair_size[p][2] = (T)m.geom_size[3 * g2]; d.pair_size[p][3] = (T)m.geom_size[3 * g2 + 1];
    d.pair_mu[p] = (T)mu;
    d.pair_margin[p] = (T)(std::max(m.geom_margin[g1], m.geom_margin[g2]) - std::max(m.geom_gap[g1], m.geom_gap[g2]));
    if (std::max(m.geom_margin[g1], m.geom_margin[g2]) != 0) { err = "nonzero geom margin not supported"; return false; }
    for (int k = 0; k < 2; k++) d.pair_solref[p][k] = (T)sr[k];
    fill_solimp(d.pair_solimp[p], si);
  }
  for (int t = 0; t < m.ntendon; t++) {
    if (m.tendon_num[t] > MAXWRAP) { err = "tendon has too many joints"; return false; }
    d.ten_nwrap[t] = m.tendon_num[t];
    for (int w = 0; w < m.tendon_num[t]; w++) {
      int j = m.wrap_jnt[m.tendon_adr[t] + w];
      d.ten_wrapdof[t][w] = m.jnt_dofadr[j];
      d.ten_wrapqadr[t][w] = m.jnt_qposadr[j];
      d.ten_wrapcoef[t][w] = (T)m.wrap_coef[m.tendon_adr[t] + w];
    }
    d.ten_limited[t] = m.tendon_limited[t];
    for (int k = 0; k < 2; k++) { d.ten_range[t][k] = (T)m.tendon_range[2 * t + k]; d.ten_solref[t][k] = (T)m.tendon_solref[2 * t + k]; }
    fill_solimp(d.ten_solimp[t], &m.tendon_solimp[5 * t]);
    d.ten_margin[t] = (T)m.tendon_margin[t];
    d.ten_invweight0[t] = (T)m.tendon_invweight0[t];
  }
  int nlim = 0;
  for (int j = 0; j < m.njnt; j++) nlim += d.jnt_limited[j];
  for (int t = 0; t < m.ntendon; t++) nlim += d.ten_limited[t];
  d.nhinge_limited = nlim;
  for (int k = 0; k < m.nq; k++) d.qpos0[k] = (T)m.qpos0[k];
  return true;
}

template bool build_dev_model<float>(const HostModel&, DevModel<float>&, std::string&);
template bool build_dev_model<double>(const HostModel&, DevModel<double>&, std::string&);

}  // namespace hs
