/* hostbook.c — the host side of one dict-facade turn (EnvStateManager._book), as a CPython
 * extension.
 *
 * EnvStateManager.step with the reference's list-of-dict inputs (es_manager.py:105-171) runs the
 * turn on the device, then has to leave per env exactly what the reference's loop leaves: the
 * EnvStatus counters and rewards, the penalty, the finished history entry (actions, reward,
 * info, llm_response, llm_raw_response) and the next one (state, actions_left), and the set of
 * envs still active.  In Python that loop was 65 % of a dict-facade turn (cProfile,
 * profiles/r03_prof_api.log); here it is the same object operations without the interpreter.
 * The Python version (_book_py) stays the definition: tests/test_hostbook.py checks this one
 * against it on every branch (Countdown's int rewards, info present / absent, penalties, done
 * flags, a note callback, rendered and pre-rendered observations).
 *
 * book(t, inputs, gids, rows, acts_l, m_l, flags, num_actions, info, n_exec, rw, pen, obs,
 *      envs, rcache, lo0, is_cd, note, render, consts) -> set of the gids still active
 *   inputs / gids / rows / acts_l / m_l: per stepped env (lists); flags / num_actions / info /
 *   n_exec / rw / pen: per tag-local row (lists); obs: list of str or None (render(i) then);
 *   note: callable(t, i, executed) or None; consts: (F_TERM, F_TRUNC, F_DONE, I_PRES, I_EFF,
 *   I_VAL, I_SUCC).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

static PyObject *k_status, *k_history, *k_penalty, *k_actions, *k_reward, *k_info, *k_llm_response,
    *k_llm_raw_response, *k_state, *k_actions_left, *k_max_actions, *k_eff, *k_valid, *k_success, *k_num_actions,
    *k_rewards, *k_terminated, *k_truncated;

static PyObject* item(PyObject* mapping, PyObject* key) {  /* new reference */
  if (PyDict_CheckExact(mapping)) {
    PyObject* v = PyDict_GetItemWithError(mapping, key);
    if (v) Py_INCREF(v);
    else if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, key);
    return v;
  }
  return PyObject_GetItem(mapping, key);
}

static int set_item(PyObject* mapping, PyObject* key, PyObject* v) {
  return PyDict_CheckExact(mapping) ? PyDict_SetItem(mapping, key, v) : PyObject_SetItem(mapping, key, v);
}

static int append(PyObject* seq, PyObject* v) {  /* list.append or seq.append(v) */
  if (PyList_Check(seq)) return PyList_Append(seq, v);
  PyObject* r = PyObject_CallMethod(seq, "append", "O", v);
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}

static PyObject* book(PyObject* self, PyObject* args) {
  long t, lo0;
  int is_cd;
  PyObject *inputs, *gids, *rows, *acts_l, *m_l, *flags, *num_actions, *info, *n_exec, *rw, *pen, *obs, *envs, *rcache,
      *note, *render;
  long F_TERM, F_TRUNC, F_DONE, I_PRES, I_EFF, I_VAL, I_SUCC;
  if (!PyArg_ParseTuple(args, "lO!O!O!O!O!O!O!O!O!O!O!OO!O!lpOO(lllllll)", &t, &PyList_Type, &inputs, &PyList_Type,
                        &gids, &PyList_Type, &rows, &PyList_Type, &acts_l, &PyList_Type, &m_l, &PyList_Type, &flags,
                        &PyList_Type, &num_actions, &PyList_Type, &info, &PyList_Type, &n_exec, &PyList_Type, &rw,
                        &PyList_Type, &pen, &obs, &PyList_Type, &envs, &PyList_Type, &rcache, &lo0, &is_cd, &note,
                        &render, &F_TERM, &F_TRUNC, &F_DONE, &I_PRES, &I_EFF, &I_VAL, &I_SUCC))
    return NULL;
  const Py_ssize_t n = PyList_GET_SIZE(inputs);
  if (PyList_GET_SIZE(gids) != n || PyList_GET_SIZE(rows) != n || PyList_GET_SIZE(acts_l) != n ||
      PyList_GET_SIZE(m_l) != n) {
    PyErr_SetString(PyExc_ValueError, "book: per-env lists differ in length");
    return NULL;
  }
  const Py_ssize_t B = PyList_GET_SIZE(flags);
  if (PyList_GET_SIZE(num_actions) != B || PyList_GET_SIZE(info) != B || PyList_GET_SIZE(n_exec) != B ||
      PyList_GET_SIZE(rw) != B || PyList_GET_SIZE(pen) != B || (obs != Py_None && (!PyList_Check(obs) ||
                                                                                   PyList_GET_SIZE(obs) != B))) {
    PyErr_SetString(PyExc_ValueError, "book: per-row lists differ in length");
    return NULL;
  }
  PyObject* still = PySet_New(NULL);
  if (!still) return NULL;
  PyObject* zero = PyLong_FromLong(0);
  for (Py_ssize_t k = 0; k < n; ++k) {
    PyObject *inp = PyList_GET_ITEM(inputs, k), *gid = PyList_GET_ITEM(gids, k);
    PyObject *acts = PyList_GET_ITEM(acts_l, k), *m = PyList_GET_ITEM(m_l, k);
    const long g = PyLong_AsLong(gid), i = PyLong_AsLong(PyList_GET_ITEM(rows, k));
    if (PyErr_Occurred()) goto fail;
    if (i < 0 || i >= B || g - lo0 < 0 || g - lo0 >= PyList_GET_SIZE(envs) || g - lo0 >= PyList_GET_SIZE(rcache)) {
      PyErr_SetString(PyExc_IndexError, "book: env row out of range");
      goto fail;
    }
    PyObject *entry = PyList_GET_ITEM(envs, g - lo0), *cache = PyList_GET_ITEM(rcache, g - lo0);
    const long ne = PyLong_AsLong(PyList_GET_ITEM(n_exec, i));
    if (PyErr_Occurred()) goto fail;
    /* executed = (acts if is_cd else [a for a in m if a != 0])[:ne] */
    PyObject* executed;
    if (is_cd) {
      executed = PySequence_GetSlice(acts, 0, ne);
    } else {
      executed = PyList_New(0);
      PyObject* ms = executed ? PySequence_Fast(m, "book: m_l entry") : NULL;
      if (ms) {
        const Py_ssize_t L = PySequence_Fast_GET_SIZE(ms);
        for (Py_ssize_t q = 0; q < L && PyList_GET_SIZE(executed) < ne; ++q) {
          PyObject* a = PySequence_Fast_GET_ITEM(ms, q);
          const int nz = PyObject_RichCompareBool(a, zero, Py_NE);
          if (nz < 0 || (nz && PyList_Append(executed, a) < 0)) {
            Py_CLEAR(executed);
            break;
          }
        }
        Py_DECREF(ms);
      } else {
        Py_CLEAR(executed);
      }
    }
    if (!executed) goto fail;
    if (note != Py_None) {
      PyObject* r = PyObject_CallFunction(note, "llO", t, i, executed);
      if (!r) {
        Py_DECREF(executed);
        goto fail;
      }
      Py_DECREF(r);
    }
    /* acc = rw[i] if ne else 0; Countdown: int(acc) for 0.0 / 1.0 */
    PyObject* acc;
    if (ne) {
      acc = PyList_GET_ITEM(rw, i);
      Py_INCREF(acc);
      if (is_cd) {
        const double v = PyFloat_AsDouble(acc);
        if (v == -1.0 && PyErr_Occurred()) {
          Py_DECREF(executed);
          Py_DECREF(acc);
          goto fail;
        }
        if (v == 0.0 || v == 1.0) {
          Py_DECREF(acc);
          acc = PyLong_FromLong((long)v);
        }
      }
    } else {
      acc = PyLong_FromLong(0);
    }
    const long inf = PyLong_AsLong(PyList_GET_ITEM(info, i));
    PyObject* turn_info = PyDict_New();
    int bad = !acc || !turn_info || (inf == -1 && PyErr_Occurred());
    if (!bad && (inf & I_PRES)) {
      bad = PyDict_SetItem(turn_info, k_eff, (inf & I_EFF) ? Py_True : Py_False) < 0 ||
            PyDict_SetItem(turn_info, k_valid, (inf & I_VAL) ? Py_True : Py_False) < 0 ||
            PyDict_SetItem(turn_info, k_success, (inf & I_SUCC) ? Py_True : Py_False) < 0;
    }
    /* EnvStatus: num_actions, rewards.append(acc), terminated, truncated */
    PyObject* na = PyList_GET_ITEM(num_actions, i);
    const long fl = PyLong_AsLong(PyList_GET_ITEM(flags, i));
    PyObject *st = NULL, *rews = NULL, *hist = NULL, *h = NULL, *maxa = NULL, *left = NULL, *nxt = NULL, *state = NULL,
             *resp = NULL, *raw = NULL;
    if (!bad) bad = (fl == -1 && PyErr_Occurred());
    if (!bad) bad = !(st = item(entry, k_status));
    if (!bad) bad = PyObject_SetAttr(st, k_num_actions, na) < 0;
    if (!bad) bad = !(rews = PyObject_GetAttr(st, k_rewards));
    if (!bad) bad = append(rews, acc) < 0;
    if (!bad) bad = PyObject_SetAttr(st, k_terminated, (fl & F_TERM) ? Py_True : Py_False) < 0;
    if (!bad) bad = PyObject_SetAttr(st, k_truncated, (fl & F_TRUNC) ? Py_True : Py_False) < 0;
    if (!bad) {  /* if pen[i] != 0: cache["penalty"] = pen[i] */
      PyObject* p = PyList_GET_ITEM(pen, i);
      const int nz = PyObject_RichCompareBool(p, zero, Py_NE);
      bad = nz < 0 || (nz && set_item(cache, k_penalty, p) < 0);
    }
    /* the finished entry and the next one */
    if (!bad) bad = !(hist = item(cache, k_history));
    if (!bad) bad = !(h = PySequence_GetItem(hist, -1));
    if (!bad) bad = !(resp = item(inp, k_llm_response)) || !(raw = item(inp, k_llm_raw_response));
    if (!bad)
      bad = set_item(h, k_actions, executed) < 0 || set_item(h, k_reward, acc) < 0 || set_item(h, k_info, turn_info) < 0 ||
            set_item(h, k_llm_response, resp) < 0 || set_item(h, k_llm_raw_response, raw) < 0;
    if (!bad) {
      if (obs != Py_None) {
        state = PyList_GET_ITEM(obs, i);
        Py_INCREF(state);
      } else {
        state = PyObject_CallFunction(render, "l", i);
      }
      bad = !state;
    }
    if (!bad) bad = !(maxa = item(entry, k_max_actions)) || !(left = PyNumber_Subtract(maxa, na));
    if (!bad) {
      nxt = PyDict_New();
      bad = !nxt || PyDict_SetItem(nxt, k_state, state) < 0 || PyDict_SetItem(nxt, k_actions_left, left) < 0 ||
            append(hist, nxt) < 0;
    }
    if (!bad && !(fl & F_DONE)) bad = PySet_Add(still, gid) < 0;
    Py_XDECREF(st);
    Py_XDECREF(rews);
    Py_XDECREF(hist);
    Py_XDECREF(h);
    Py_XDECREF(resp);
    Py_XDECREF(raw);
    Py_XDECREF(state);
    Py_XDECREF(maxa);
    Py_XDECREF(left);
    Py_XDECREF(nxt);
    Py_XDECREF(turn_info);
    Py_XDECREF(acc);
    Py_DECREF(executed);
    if (bad) goto fail;
  }
  Py_DECREF(zero);
  return still;
fail:
  Py_XDECREF(zero);
  Py_DECREF(still);
  return NULL;
}

static PyMethodDef methods[] = {
    {"book", book, METH_VARARGS, "The host side of one dict-facade turn (EnvStateManager._book)."},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_hostbook", NULL, -1, methods};

PyMODINIT_FUNC PyInit__hostbook(void) {
  struct {
    PyObject** dst;
    const char* s;
  } keys[] = {{&k_status, "status"},
              {&k_history, "history"},
              {&k_penalty, "penalty"},
              {&k_actions, "actions"},
              {&k_reward, "reward"},
              {&k_info, "info"},
              {&k_llm_response, "llm_response"},
              {&k_llm_raw_response, "llm_raw_response"},
              {&k_state, "state"},
              {&k_actions_left, "actions_left"},
              {&k_max_actions, "max_actions_per_traj"},
              {&k_eff, "action_is_effective"},
              {&k_valid, "action_is_valid"},
              {&k_success, "success"},
              {&k_num_actions, "num_actions"},
              {&k_rewards, "rewards"},
              {&k_terminated, "terminated"},
              {&k_truncated, "truncated"}};
  for (size_t j = 0; j < sizeof(keys) / sizeof(keys[0]); ++j)
    if (!(*keys[j].dst = PyUnicode_InternFromString(keys[j].s))) return NULL;
  return PyModule_Create(&module);
}
