/* SB3 VecEnv info dicts of one HumanoidVecEnv.step_wait, built in C (CPython extension _hsinfo).
 *
 * SubprocVecEnv returns one dict per env per step (custom_env.py:216-230 keys; SB3 adds
 * terminal_observation and TimeLimit.truncated for envs that finished, train_sb3.py:203).  At 4096
 * envs building them in Python costs ~5 ms per step, several times the physics; here each dict is a
 * handful of PyDict_SetItem calls with interned keys.  vec_env.StepInfos calls build() lazily: for
 * one env on indexed access, for all of them when a consumer iterates (SB3's collect_rollouts does).
 *
 * build(height, step_count, truncated, terminated, total_reward, done_pos, term_obs, start, stop)
 *   height / step_count / truncated / terminated / total_reward: lists (per env, Python scalars;
 *   truncated / terminated of bool)
 *   done_pos: dict env -> row of term_obs (the envs that finished), term_obs: 2-D array or None
 *   returns [dict for env in range(start, stop)], equal to the eager Python construction. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

static PyObject *k_height, *k_step_count, *k_truncated, *k_truncation_info, *k_terminated, *k_total_reward,
    *k_reward_components, *k_terminal_observation, *k_timelimit, *k_reason, *v_timeout;

static int set_new(PyObject* d, PyObject* k, PyObject* v) {   /* steals v */
  if (!v) return -1;
  int rc = PyDict_SetItem(d, k, v);
  Py_DECREF(v);
  return rc;
}

static PyObject* build_one(PyObject* h, PyObject* sc, PyObject* tr, PyObject* te, PyObject* tot, PyObject* done_pos,
                           PyObject* tobs, Py_ssize_t i) {
  PyObject* d = _PyDict_NewPresized(9);   /* 7 keys, 9 for a finished env: no resize on the way */
  if (!d) return NULL;
  PyObject* trunc = PyList_GET_ITEM(tr, i);
  PyObject* term = PyList_GET_ITEM(te, i);
  const int is_trunc = trunc == Py_True, is_term = term == Py_True;
  PyObject* tinfo = PyDict_New();
  if (!tinfo) goto fail;
  if (is_trunc && PyDict_SetItem(tinfo, k_reason, v_timeout) < 0) { Py_DECREF(tinfo); goto fail; }
  if (set_new(d, k_reward_components, PyDict_New()) < 0) { Py_DECREF(tinfo); goto fail; }
  /* keys in custom_env.py:216-224's order */
  if (PyDict_SetItem(d, k_height, PyList_GET_ITEM(h, i)) < 0 ||
      PyDict_SetItem(d, k_step_count, PyList_GET_ITEM(sc, i)) < 0 ||
      PyDict_SetItem(d, k_truncated, trunc) < 0 ||
      set_new(d, k_truncation_info, tinfo) < 0 ||
      PyDict_SetItem(d, k_terminated, term) < 0 ||
      PyDict_SetItem(d, k_total_reward, PyList_GET_ITEM(tot, i)) < 0)
    goto fail;
  if ((is_trunc || is_term) && done_pos != Py_None) {
    PyObject* key = PyLong_FromSsize_t(i);
    if (!key) goto fail;
    PyObject* row = PyDict_GetItemWithError(done_pos, key);   /* borrowed */
    Py_DECREF(key);
    if (!row && PyErr_Occurred()) goto fail;
    if (row) {
      if (set_new(d, k_terminal_observation, PyObject_GetItem(tobs, row)) < 0) goto fail;
      PyObject* tl = (is_trunc && !is_term) ? Py_True : Py_False;
      if (PyDict_SetItem(d, k_timelimit, tl) < 0) goto fail;
    }
  }
  return d;
fail:
  Py_DECREF(d);
  return NULL;
}

static PyObject* build(PyObject* self, PyObject* args) {
  PyObject *h, *sc, *tr, *te, *tot, *done_pos, *tobs;
  Py_ssize_t start, stop;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!O!O!O!OOnn", &PyList_Type, &h, &PyList_Type, &sc, &PyList_Type, &tr, &PyList_Type,
                        &te, &PyList_Type, &tot, &done_pos, &tobs, &start, &stop))
    return NULL;
  const Py_ssize_t n = PyList_GET_SIZE(h);
  if (PyList_GET_SIZE(sc) != n || PyList_GET_SIZE(tr) != n || PyList_GET_SIZE(te) != n || PyList_GET_SIZE(tot) != n) {
    PyErr_SetString(PyExc_ValueError, "_hsinfo.build: column lengths differ");
    return NULL;
  }
  if (start < 0 || stop > n || start > stop) {
    PyErr_SetString(PyExc_IndexError, "_hsinfo.build: range out of bounds");
    return NULL;
  }
  if (done_pos != Py_None && !PyDict_Check(done_pos)) {
    PyErr_SetString(PyExc_TypeError, "_hsinfo.build: done_pos must be a dict or None");
    return NULL;
  }
  PyObject* out = PyList_New(stop - start);
  if (!out) return NULL;
  /* the cyclic GC off while the (acyclic) dicts are made: otherwise every ~700 new containers run a
   * young-generation collection, which triples the cost at 4096 envs */
  const int gc_was = PyGC_Disable();
  for (Py_ssize_t i = start; i < stop; i++) {
    PyObject* d = build_one(h, sc, tr, te, tot, done_pos, tobs, i);
    if (!d) {
      if (gc_was) PyGC_Enable();
      Py_DECREF(out);
      return NULL;
    }
    PyList_SET_ITEM(out, i - start, d);   /* steals d */
  }
  if (gc_was) PyGC_Enable();
  return out;
}

static PyMethodDef methods[] = {
    {"build", build, METH_VARARGS, "SB3 info dicts of envs [start, stop) of one step (see hs_infos.c)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_hsinfo", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__hsinfo(void) {
#define INTERN(var, s) if (!(var = PyUnicode_InternFromString(s))) return NULL
  INTERN(k_height, "height");
  INTERN(k_step_count, "step_count");
  INTERN(k_truncated, "truncated");
  INTERN(k_truncation_info, "truncation_info");
  INTERN(k_terminated, "terminated");
  INTERN(k_total_reward, "total_reward");
  INTERN(k_reward_components, "reward_components");
  INTERN(k_terminal_observation, "terminal_observation");
  INTERN(k_timelimit, "TimeLimit.truncated");
  INTERN(k_reason, "reason");
  INTERN(v_timeout, "timeout");
#undef INTERN
  return PyModule_Create(&module);
}
