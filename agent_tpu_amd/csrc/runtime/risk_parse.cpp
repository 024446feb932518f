// risk_accumulate over a JSON-decoded Python list, natively.
//
// The reference converts every element with a Python helper (`_to_float`: int/float/bool
// as float(), numeric strings via float(s.strip()), anything else ValueError("value must
// be numeric"), ref ops/risk_accumulate.py:10-15) and accumulates count/sum/min/max in a
// Python loop (:65-68), ~8 M values/s. This walks the list with the CPython API: the same
// conversions (strings go through float() itself, so its accepted forms and error
// messages are unchanged), the same sequential float64 sum and the same `<` / `>`
// comparisons, so results are bit-identical to the reference, at C speed.
#include <Python.h>

#include <cstdint>
#include <stdexcept>
#include <vector>

#include "atpu/runtime.h"

namespace atpu {
namespace {

struct PyErrorAlreadySet {};

// float(value) with the reference's type gate; throws PyErrorAlreadySet with the Python error set
inline double to_float(PyObject* v) {
  if (PyFloat_CheckExact(v)) return PyFloat_AS_DOUBLE(v);
  if (PyLong_Check(v)) {  // bool is an int subclass: True -> 1.0 (as the reference)
    const double d = PyLong_AsDouble(v);
    if (d == -1.0 && PyErr_Occurred()) throw PyErrorAlreadySet{};
    return d;
  }
  if (PyFloat_Check(v)) return PyFloat_AsDouble(v);
  if (PyUnicode_Check(v)) {
    PyObject* stripped = PyObject_CallMethod(v, "strip", nullptr);
    if (!stripped) throw PyErrorAlreadySet{};
    PyObject* f = PyFloat_FromString(stripped);
    Py_DECREF(stripped);
    if (!f) throw PyErrorAlreadySet{};
    const double d = PyFloat_AS_DOUBLE(f);
    Py_DECREF(f);
    return d;
  }
  PyErr_SetString(PyExc_ValueError, "value must be numeric");
  throw PyErrorAlreadySet{};
}

}  // namespace

// mode 0: `values` list; mode 1: `items` list of dicts, reading key `field` (items without
// it are skipped; a non-dict item raises ValueError("payload.items must contain dict
// objects")). Returns false with a Python exception set on error. `out` (optional)
// receives the converted values.
bool risk_stats_pylist(PyObject* list, int mode, PyObject* field, RiskStats* st, std::vector<double>* out) {
  st->count = 0;
  st->sum = 0.0;
  st->min = st->max = 0.0;
  const Py_ssize_t n = PyList_GET_SIZE(list);
  if (out) out->reserve(static_cast<size_t>(n));
  try {
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* v = PyList_GET_ITEM(list, i);  // borrowed
      if (mode == 1) {
        if (!PyDict_Check(v)) {
          PyErr_SetString(PyExc_ValueError, "payload.items must contain dict objects");
          throw PyErrorAlreadySet{};
        }
        v = PyDict_GetItemWithError(v, field);  // borrowed
        if (!v) {
          if (PyErr_Occurred()) throw PyErrorAlreadySet{};
          continue;
        }
      }
      const double d = to_float(v);
      if (st->count == 0) {
        st->min = st->max = d;
      } else {
        if (d < st->min) st->min = d;
        if (d > st->max) st->max = d;
      }
      st->sum += d;
      st->count += 1;
      if (out) out->push_back(d);
    }
  } catch (const PyErrorAlreadySet&) {
    return false;
  }
  return true;
}

}  // namespace atpu
