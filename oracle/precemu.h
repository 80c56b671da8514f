/* ORACLE (test infrastructure only): fp32-EMULATING build of the fp64 restatement, per stage.
 *
 * Force-included (g++ -x c++ -include oracle/precemu.h oracle/hsim_oracle.c), like flopcount.h:
 * every `double` of the oracle becomes `pdouble`, a layout-identical wrapper (one double), whose
 * arithmetic results are rounded to float when bit k of orc_prec_mask is set for the current stage k
 * (ORC_STAGE in orc_forward / step_impl).  + - * / sqrt computed in double and rounded once to float
 * are exactly the correctly rounded float results, so a stage with its bit set computes as an fp32
 * engine would (oracle/precision.py; DESIGN.md 4: where the fp32 engine's divergence comes from).
 * Model data and the state stay doubles; the caller rounds them to float for a full fp32 run.
 */
#ifndef ORC_PRECEMU_H
#define ORC_PRECEMU_H
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#define ORC_NSTAGE 32
#define ORC_PREC_SUBSTAGES 1
extern "C" {
int orc_prec_stage;
unsigned orc_prec_mask;
}
#define ORC_STAGE(k) (orc_prec_stage = (k))

struct pdouble {
  double v;
  pdouble() = default;
  constexpr pdouble(double x) : v(x) {}   // NOLINT: implicit, like the builtin it replaces
  explicit operator double() const { return v; }
  explicit operator int() const { return (int)v; }
  static double r(double x) { return ((orc_prec_mask >> orc_prec_stage) & 1u) ? (double)(float)x : x; }
  pdouble& operator+=(pdouble o) { v = r(v + o.v); return *this; }
  pdouble& operator-=(pdouble o) { v = r(v - o.v); return *this; }
  pdouble& operator*=(pdouble o) { v = r(v * o.v); return *this; }
  pdouble& operator/=(pdouble o) { v = r(v / o.v); return *this; }
  pdouble operator-() const { return pdouble(-v); }
  pdouble operator+() const { return *this; }
};
static_assert(sizeof(pdouble) == sizeof(double) && alignof(pdouble) == alignof(double), "layout");
static_assert(std::is_trivially_copyable<pdouble>::value, "memcpy-able");

template <typename T>
using orc_arith = std::enable_if_t<std::is_arithmetic<T>::value, int>;
#define ORC_BINOP(op)                                                                              \
  inline pdouble operator op(pdouble a, pdouble b) { return pdouble(pdouble::r(a.v op b.v)); } \
  template <typename T, orc_arith<T> = 0>                                                          \
  inline pdouble operator op(pdouble a, T b) { return pdouble(pdouble::r(a.v op (double)b)); } \
  template <typename T, orc_arith<T> = 0>                                                          \
  inline pdouble operator op(T a, pdouble b) { return pdouble(pdouble::r((double)a op b.v)); }
ORC_BINOP(+)
ORC_BINOP(-)
ORC_BINOP(*)
ORC_BINOP(/)
#undef ORC_BINOP
#define ORC_CMP(op)                                                                       \
  inline bool operator op(pdouble a, pdouble b) { return a.v op b.v; }                    \
  template <typename T, orc_arith<T> = 0>                                                 \
  inline bool operator op(pdouble a, T b) { return a.v op (double)b; }                    \
  template <typename T, orc_arith<T> = 0>                                                 \
  inline bool operator op(T a, pdouble b) { return (double)a op b.v; }
ORC_CMP(<)
ORC_CMP(>)
ORC_CMP(<=)
ORC_CMP(>=)
ORC_CMP(==)
ORC_CMP(!=)
#undef ORC_CMP
#define ORC_FN1(f) \
  inline pdouble f(pdouble a) { return pdouble(pdouble::r(std::f(a.v))); }
ORC_FN1(sqrt)
ORC_FN1(sin)
ORC_FN1(cos)
ORC_FN1(asin)
ORC_FN1(exp)
ORC_FN1(fabs)
ORC_FN1(floor)
#undef ORC_FN1
#define ORC_FN2(f)                                                                                  \
  inline pdouble f(pdouble a, pdouble b) { return pdouble(pdouble::r(std::f(a.v, b.v))); }     \
  template <typename T, orc_arith<T> = 0>                                                           \
  inline pdouble f(pdouble a, T b) { return pdouble(pdouble::r(std::f(a.v, (double)b))); }     \
  template <typename T, orc_arith<T> = 0>                                                           \
  inline pdouble f(T a, pdouble b) { return pdouble(pdouble::r(std::f((double)a, b.v))); }
ORC_FN2(atan2)
ORC_FN2(pow)
ORC_FN2(fmin)
ORC_FN2(fmax)
#undef ORC_FN2

#define double pdouble
#endif
