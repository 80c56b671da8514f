/* ORACLE (test infrastructure only): FLOP-counting build of the fp64 restatement (SURVEY.md 8d,
 * "Algorithmic FLOPs: count in the CPU restatement with an instrumented op counter per stage").
 *
 * Force-included (g++ -x c++ -include oracle/flopcount.h oracle/hsim_oracle.c): every `double`
 * of the oracle becomes `fdouble`, a layout-identical wrapper (one double, trivially copyable, so
 * OrcModel / OrcData keep the ctypes layout of oracle/oracle.py) whose arithmetic operators and
 * math functions add to a per-stage counter.  Counted as 1 FLOP each: + - * / (incl. compound
 * assignments) and sqrt / sin / cos / atan2 / asin / exp / pow / fabs / fmin / fmax; not counted:
 * comparisons, negation, copies.  Stages are set by ORC_STAGE(k) in orc_forward / step_impl.
 * orc_flops(out, n) copies the counters (n <= ORC_NSTAGE) and zeroes them.
 */
#ifndef ORC_FLOPCOUNT_H
#define ORC_FLOPCOUNT_H
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#define ORC_NSTAGE 16
/* force-included into the one translation unit (hsim_oracle.c): the counters live here */
extern "C" {
double orc_flop_counter[ORC_NSTAGE];
int orc_flop_stage;
void orc_flops(double* out, int n) {
  for (int k = 0; k < n && k < ORC_NSTAGE; k++) { out[k] = orc_flop_counter[k]; orc_flop_counter[k] = 0; }
}
}
#define ORC_STAGE(k) (orc_flop_stage = (k))

struct fdouble {
  double v;
  fdouble() = default;
  constexpr fdouble(double x) : v(x) {}   // NOLINT: implicit, like the builtin it replaces
  explicit operator double() const { return v; }
  explicit operator int() const { return (int)v; }
  static void tick() { orc_flop_counter[orc_flop_stage] += 1.0; }
  fdouble& operator+=(fdouble o) { tick(); v += o.v; return *this; }
  fdouble& operator-=(fdouble o) { tick(); v -= o.v; return *this; }
  fdouble& operator*=(fdouble o) { tick(); v *= o.v; return *this; }
  fdouble& operator/=(fdouble o) { tick(); v /= o.v; return *this; }
  fdouble operator-() const { return fdouble(-v); }
  fdouble operator+() const { return *this; }
};
static_assert(sizeof(fdouble) == sizeof(double) && alignof(fdouble) == alignof(double), "layout");
static_assert(std::is_trivially_copyable<fdouble>::value, "memcpy-able");

template <typename T>
using orc_arith = std::enable_if_t<std::is_arithmetic<T>::value, int>;
#define ORC_BINOP(op)                                                                              \
  inline fdouble operator op(fdouble a, fdouble b) { fdouble::tick(); return fdouble(a.v op b.v); } \
  template <typename T, orc_arith<T> = 0>                                                          \
  inline fdouble operator op(fdouble a, T b) { fdouble::tick(); return fdouble(a.v op (double)b); } \
  template <typename T, orc_arith<T> = 0>                                                          \
  inline fdouble operator op(T a, fdouble b) { fdouble::tick(); return fdouble((double)a op b.v); }
ORC_BINOP(+)
ORC_BINOP(-)
ORC_BINOP(*)
ORC_BINOP(/)
#undef ORC_BINOP
#define ORC_CMP(op)                                                                       \
  inline bool operator op(fdouble a, fdouble b) { return a.v op b.v; }                    \
  template <typename T, orc_arith<T> = 0>                                                 \
  inline bool operator op(fdouble a, T b) { return a.v op (double)b; }                    \
  template <typename T, orc_arith<T> = 0>                                                 \
  inline bool operator op(T a, fdouble b) { return (double)a op b.v; }
ORC_CMP(<)
ORC_CMP(>)
ORC_CMP(<=)
ORC_CMP(>=)
ORC_CMP(==)
ORC_CMP(!=)
#undef ORC_CMP
#define ORC_FN1(f) \
  inline fdouble f(fdouble a) { fdouble::tick(); return fdouble(std::f(a.v)); }
ORC_FN1(sqrt)
ORC_FN1(sin)
ORC_FN1(cos)
ORC_FN1(asin)
ORC_FN1(exp)
ORC_FN1(fabs)
ORC_FN1(floor)
#undef ORC_FN1
#define ORC_FN2(f)                                                                                  \
  inline fdouble f(fdouble a, fdouble b) { fdouble::tick(); return fdouble(std::f(a.v, b.v)); }     \
  template <typename T, orc_arith<T> = 0>                                                           \
  inline fdouble f(fdouble a, T b) { fdouble::tick(); return fdouble(std::f(a.v, (double)b)); }     \
  template <typename T, orc_arith<T> = 0>                                                           \
  inline fdouble f(T a, fdouble b) { fdouble::tick(); return fdouble(std::f((double)a, b.v)); }
ORC_FN2(atan2)
ORC_FN2(pow)
ORC_FN2(fmin)
ORC_FN2(fmax)
#undef ORC_FN2

#define double fdouble
#endif
