#!/usr/bin/env python3
"""Generate ``_ncffast.c``: a CPython extension that calls the C-ABI entry points of
libncf_hip.so with one PyArg_ParseTuple per call instead of ctypes' per-argument conversion.

ctypes stays the loader (``_lib.load()`` resolves every symbol and checks the signatures); the
extension receives the resolved function addresses once (``bind(index, address)``) and then
only forwards arguments.  One wrapper per signature of ``_lib.SIGNATURES`` whose result is an
integer; the argument kinds map to format units: pointer -> ``O&`` (None -> NULL, or an int
address), int64 -> ``L``, int32 -> ``i``, uint64 -> ``K``, float -> ``f``, double -> ``d``.
Measured reason (tools/dropin_host.py): a 25-argument ctypes call costs ~7 us of host time, and
a training step makes ~13 of them on the reference call pattern's critical host path.

Launch tapes.  While a tape records (``tape_begin``), every wrapper that returns 0 also appends
its call -- the entry point and its converted arguments, packed in a per-signature struct -- to
the tape; ``tape_replay`` later makes the same calls in the same order from C, with no Python
in between.  Pointer arguments that fall inside one of the ranges given to ``tape_begin``
(the step's id lists, the loss gradient, the stream) are patched at replay with the new base
addresses passed to ``tape_replay`` (same offsets).  A call that fails, or an entry point
reached through ctypes instead of this module (``tape_invalidate``), invalidates the tape;
``tape_hold(1)`` suspends recording (size queries).  ``tape_tag(arg, slot)`` marks a scalar
argument of the next call as a replay slot (a per-step size or counter), replayed with the value
passed for that slot.

    python gen_fastcall.py OUT.c
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def load_signatures():
    """Read SIGNATURES from _lib.py without importing torch (exec of the table only)."""
    src = open(os.path.join(HERE, "..", "_lib.py")).read()
    start = src.index("P = ctypes.c_void_p")
    end = src.index("\nclass ReduceDesc")
    ns = {"ctypes": ctypes}
    exec(src[start:end], ns)     # the type aliases + the SIGNATURES literal
    return ns["SIGNATURES"], ns


TAPE_RUNTIME = r"""
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
typedef int (*replay_fn)(const void*);
typedef struct { int idx; int size; char* blob; } TapeOp;
typedef struct { int op; int off; int slot; int width; unsigned long long delta; } TapePatch;
typedef struct { TapeOp* ops; int n, cap; TapePatch* pt; int np, pcap; int valid; } Tape;
#define NCF_TAPE_SLOTS 16
static Tape* g_rec = NULL;        /* the tape being recorded, if any */
static int g_hold = 0;            /* recording suspended (size queries) */
static unsigned long long g_lo[NCF_TAPE_SLOTS], g_hi[NCF_TAPE_SLOTS];
static int g_nslots = 0;
/* scalar slots: tape_tag(arg, slot) marks argument `arg` of the NEXT recorded call as slot
   `slot` (replayed with the value passed for that slot) */
#define NCF_TAPE_TAGS 8
static int g_tag_arg[NCF_TAPE_TAGS], g_tag_slot[NCF_TAPE_TAGS];
static int g_ntags = 0;

static int tape_add_patch(Tape* t, int op, int off, int slot, int width, unsigned long long delta) {
  if (t->np == t->pcap) {
    int cap = t->pcap ? 2 * t->pcap : 32;
    TapePatch* p = (TapePatch*)realloc(t->pt, sizeof(TapePatch) * cap);
    if (!p) { t->valid = 0; return 0; }
    t->pt = p; t->pcap = cap;
  }
  TapePatch* p = &t->pt[t->np++];
  p->op = op; p->off = off; p->slot = slot; p->width = width; p->delta = delta;
  return 1;
}

static void tape_clear(Tape* t) {
  for (int i = 0; i < t->n; ++i) free(t->ops[i].blob);
  t->n = 0; t->np = 0; t->valid = 1;
}

static void tape_push(int idx, const void* args, int size, const int* poff, const int* aoff,
                      const int* awid, int nargs) {
  Tape* t = g_rec;
  int ntags = g_ntags;
  g_ntags = 0;
  if (!t->valid) return;
  if (t->n == t->cap) {
    int cap = t->cap ? 2 * t->cap : 32;
    TapeOp* o = (TapeOp*)realloc(t->ops, sizeof(TapeOp) * cap);
    if (!o) { t->valid = 0; return; }
    t->ops = o; t->cap = cap;
  }
  char* blob = (char*)malloc(size);
  if (!blob) { t->valid = 0; return; }
  memcpy(blob, args, size);
  int op = t->n;
  t->ops[op].idx = idx; t->ops[op].size = size; t->ops[op].blob = blob;
  t->n++;
  for (int k = 0; k < ntags; ++k) {
    const int a = g_tag_arg[k];
    if (a < 0 || a >= nargs || (awid[a] != 4 && awid[a] != 8)) { t->valid = 0; return; }
    if (!tape_add_patch(t, op, aoff[a], g_tag_slot[k], awid[a], 0)) return;
  }
  for (int k = 0; poff[k] >= 0; ++k) {
    unsigned long long v;
    memcpy(&v, blob + poff[k], sizeof v);
    for (int s = 0; s < g_nslots; ++s) {
      if (v >= g_lo[s] && v < g_hi[s]) {
        if (!tape_add_patch(t, op, poff[k], s, 8, v - g_lo[s])) return;
        break;
      }
    }
  }
}
"""

TAPE_API = r"""
static void tape_free_capsule(PyObject* cap) {
  Tape* t = (Tape*)PyCapsule_GetPointer(cap, "ncf_tape");
  if (!t) return;
  if (g_rec == t) g_rec = NULL;
  tape_clear(t);
  free(t->ops); free(t->pt); free(t);
}

static Tape* tape_of(PyObject* cap) { return (Tape*)PyCapsule_GetPointer(cap, "ncf_tape"); }

static PyObject* py_tape_new(PyObject* self, PyObject* a) {
  Tape* t = (Tape*)calloc(1, sizeof(Tape));
  if (!t) return PyErr_NoMemory();
  t->valid = 1;
  return PyCapsule_New(t, "ncf_tape", tape_free_capsule);
}

/* tape_begin(tape, (lo0, size0, lo1, size1, ...)): record into tape (cleared first); pointer
   arguments inside [lo_s, lo_s + size_s) become patch slot s */
static PyObject* py_tape_begin(PyObject* self, PyObject* a) {
  PyObject *cap, *ranges;
  if (!PyArg_ParseTuple(a, "OO!:tape_begin", &cap, &PyTuple_Type, &ranges)) return NULL;
  Tape* t = tape_of(cap);
  if (!t) return NULL;
  Py_ssize_t m = PyTuple_GET_SIZE(ranges);
  if (m % 2 || m / 2 > NCF_TAPE_SLOTS) {
    PyErr_SetString(PyExc_ValueError, "tape_begin: (base, size) pairs, at most 16");
    return NULL;
  }
  if (g_rec) { PyErr_SetString(PyExc_RuntimeError, "tape_begin: a tape is already recording"); return NULL; }
  for (Py_ssize_t s = 0; s < m / 2; ++s) {
    unsigned long long lo = PyLong_AsUnsignedLongLongMask(PyTuple_GET_ITEM(ranges, 2 * s));
    unsigned long long sz = PyLong_AsUnsignedLongLongMask(PyTuple_GET_ITEM(ranges, 2 * s + 1));
    if (PyErr_Occurred()) return NULL;
    g_lo[s] = lo; g_hi[s] = lo + sz;
  }
  g_nslots = (int)(m / 2);
  tape_clear(t);
  g_rec = t; g_hold = 0; g_ntags = 0;
  Py_RETURN_NONE;
}

/* tape_end() -> (calls recorded, valid) */
static PyObject* py_tape_end(PyObject* self, PyObject* a) {
  Tape* t = g_rec;
  g_rec = NULL; g_hold = 0; g_nslots = 0; g_ntags = 0;
  if (!t) return Py_BuildValue("(ii)", 0, 0);
  return Py_BuildValue("(ii)", t->n, t->valid);
}

static PyObject* py_tape_hold(PyObject* self, PyObject* a) {
  int h;
  if (!PyArg_ParseTuple(a, "i:tape_hold", &h)) return NULL;
  int prev = g_hold;
  g_hold = h;
  return PyLong_FromLong(prev);
}

/* tape_tag(arg, slot): argument `arg` (0-based) of the next recorded call is scalar slot `slot` */
static PyObject* py_tape_tag(PyObject* self, PyObject* a) {
  int arg, slot;
  if (!PyArg_ParseTuple(a, "ii:tape_tag", &arg, &slot)) return NULL;
  if (slot < 0 || slot >= NCF_TAPE_SLOTS || g_ntags >= NCF_TAPE_TAGS) {
    PyErr_SetString(PyExc_ValueError, "tape_tag: slot out of range or too many tags");
    return NULL;
  }
  if (g_rec) { g_tag_arg[g_ntags] = arg; g_tag_slot[g_ntags] = slot; g_ntags++; }
  Py_RETURN_NONE;
}

static PyObject* py_tape_invalidate(PyObject* self, PyObject* a) {
  if (g_rec) g_rec->valid = 0;
  g_ntags = 0;
  Py_RETURN_NONE;
}

static PyObject* py_tape_size(PyObject* self, PyObject* a) {
  PyObject* cap;
  if (!PyArg_ParseTuple(a, "O:tape_size", &cap)) return NULL;
  Tape* t = tape_of(cap);
  if (!t) return NULL;
  return Py_BuildValue("(iii)", t->n, t->np, t->valid);
}

/* tape_replay(tape, (base0, base1, ...)) -> 0, or (index of the failing call, its code) */
static PyObject* py_tape_replay(PyObject* self, PyObject* a) {
  PyObject *cap, *bases;
  if (!PyArg_ParseTuple(a, "OO!:tape_replay", &cap, &PyTuple_Type, &bases)) return NULL;
  Tape* t = tape_of(cap);
  if (!t) return NULL;
  if (!t->valid) { PyErr_SetString(PyExc_RuntimeError, "tape_replay: invalid tape"); return NULL; }
  if (g_rec) { PyErr_SetString(PyExc_RuntimeError, "tape_replay while recording"); return NULL; }
  unsigned long long v[NCF_TAPE_SLOTS];
  Py_ssize_t m = PyTuple_GET_SIZE(bases);
  if (m > NCF_TAPE_SLOTS) { PyErr_SetString(PyExc_ValueError, "tape_replay: at most 16 bases"); return NULL; }
  for (Py_ssize_t s = 0; s < m; ++s) {
    v[s] = PyLong_AsUnsignedLongLongMask(PyTuple_GET_ITEM(bases, s));
    if (PyErr_Occurred()) return NULL;
  }
  for (int i = 0; i < t->np; ++i) {
    const TapePatch* p = &t->pt[i];
    if (p->slot >= m) { PyErr_SetString(PyExc_ValueError, "tape_replay: missing base"); return NULL; }
    unsigned long long x = v[p->slot] + p->delta;
    if (p->width == 8) {
      memcpy(t->ops[p->op].blob + p->off, &x, 8);
    } else {
      unsigned int y = (unsigned int)x;
      memcpy(t->ops[p->op].blob + p->off, &y, 4);
    }
  }
  int fail = -1, rc = 0;
  Py_BEGIN_ALLOW_THREADS
  for (int i = 0; i < t->n; ++i) {
    int idx = t->ops[i].idx;
    rc = (idx >= 0 && idx < NREPLAY) ? REPLAY[idx](t->ops[i].blob) : -1;
    if (rc != 0) { fail = i; break; }
  }
  Py_END_ALLOW_THREADS
  if (fail < 0) return PyLong_FromLong(0);
  return Py_BuildValue("(ii)", fail, rc);
}
"""


def main(out):
    sigs, ns = load_signatures()
    kinds = {id(ns["P"]): ("O&", "void*", "ncf_ptr_conv"),
             id(ns["I64"]): ("L", "long long", None),
             id(ns["I32"]): ("i", "int", None),
             id(ctypes.c_int32): ("i", "int", None),
             id(ns["F32"]): ("f", "float", None),
             id(ns["F64"]): ("d", "double", None),
             id(ns["U64"]): ("K", "unsigned long long", None)}
    rets = {id(ns["I32"]): ("int", "PyLong_FromLong"), id(ns["I64"]): ("long long", "PyLong_FromLongLong")}
    lines = ["/* generated by gen_fastcall.py from _lib.SIGNATURES -- do not edit */",
             "#define PY_SSIZE_T_CLEAN", "#include <Python.h>", "",
             "static int ncf_ptr_conv(PyObject* o, void** out) {",
             "  if (o == Py_None) { *out = NULL; return 1; }",
             "  if (PyLong_Check(o)) { *out = PyLong_AsVoidPtr(o); return !PyErr_Occurred(); }",
             "  PyErr_SetString(PyExc_TypeError, \"pointer argument must be an int address or None\");",
             "  return 0;", "}", "",
             TAPE_RUNTIME]
    names = []
    for name, (res, args) in sigs.items():
        if id(res) not in rets or any(id(a) not in kinds for a in args):
            continue
        rtype, rconv = rets[id(res)]
        idx = len(names)
        names.append(name)
        fmt = "".join(kinds[id(a)][0] for a in args)
        decl = ", ".join(kinds[id(a)][1] for a in args) or "void"
        lines.append(f"typedef {rtype} (*fn_{idx})({decl});")
        lines.append(f"static fn_{idx} p_{idx} = NULL;")
        fields = " ".join(f"{kinds[id(t)][1]} a{j};" for j, t in enumerate(args)) or "char unused;"
        lines.append(f"typedef struct {{ {fields} }} A_{idx};")
        offs = [f"(int)offsetof(A_{idx}, a{j})" for j, t in enumerate(args) if kinds[id(t)][2]]
        lines.append(f"static const int po_{idx}[] = {{" + ", ".join(offs + ["-1"]) + "};")
        aoffs = [f"(int)offsetof(A_{idx}, a{j})" for j in range(len(args))] or ["0"]
        awids = [f"(int)sizeof(((A_{idx}*)0)->a{j})" for j in range(len(args))] or ["0"]
        lines.append(f"static const int ao_{idx}[] = {{" + ", ".join(aoffs) + "};")
        lines.append(f"static const int aw_{idx}[] = {{" + ", ".join(awids) + "};")
        lines.append(f"static PyObject* w_{idx}(PyObject* self, PyObject* a) {{  /* {name} */")
        for j, t in enumerate(args):
            lines.append(f"  {kinds[id(t)][1]} a{j} = 0;")
        refs = []
        for j, t in enumerate(args):
            if kinds[id(t)][2]:
                refs.append(f"{kinds[id(t)][2]}, &a{j}")
            else:
                refs.append(f"&a{j}")
        argsref = (", " + ", ".join(refs)) if refs else ""
        lines.append(f"  if (!PyArg_ParseTuple(a, \"{fmt}:{name}\"{argsref})) return NULL;")
        lines.append(f"  if (!p_{idx}) {{ PyErr_SetString(PyExc_RuntimeError, \"{name} not bound\"); return NULL; }}")
        call = ", ".join(f"a{j}" for j in range(len(args)))
        lines.append(f"  {rtype} r;")
        lines.append("  Py_BEGIN_ALLOW_THREADS")
        lines.append(f"  r = p_{idx}({call});")
        lines.append("  Py_END_ALLOW_THREADS")
        lines.append("  if (g_rec && !g_hold) {")
        lines.append("    if (r != 0) { g_rec->valid = 0; g_ntags = 0; }")
        if args:
            lines.append(f"    else {{ A_{idx} s; memset(&s, 0, sizeof s); " +
                         " ".join(f"s.a{j} = a{j};" for j in range(len(args))) +
                         f" tape_push({idx}, &s, (int)sizeof s, po_{idx}, ao_{idx}, aw_{idx}, {len(args)}); }}")
        else:
            lines.append(f"    else {{ A_{idx} s; memset(&s, 0, sizeof s); tape_push({idx}, &s, (int)sizeof s, po_{idx}, ao_{idx}, aw_{idx}, 0); }}")
        lines.append("  }")
        lines.append(f"  return {rconv}(r);")
        lines.append("}")
        # replay: the packed arguments -> the same call
        lines.append(f"static int r_{idx}(const void* b) {{")
        lines.append(f"  const A_{idx}* s = (const A_{idx}*)b; (void)s;")
        lines.append(f"  return (int)p_{idx}(" + ", ".join(f"s->a{j}" for j in range(len(args))) + ");")
        lines.append("}")
    lines.append("")
    lines.append("static PyObject* ncf_bind(PyObject* self, PyObject* a) {")
    lines.append("  int i; void* p;")
    lines.append("  if (!PyArg_ParseTuple(a, \"iO&:bind\", &i, ncf_ptr_conv, &p)) return NULL;")
    lines.append("  switch (i) {")
    for idx in range(len(names)):
        lines.append(f"    case {idx}: p_{idx} = (fn_{idx})p; break;")
    lines.append("    default: PyErr_SetString(PyExc_IndexError, \"bad index\"); return NULL;")
    lines.append("  }")
    lines.append("  Py_RETURN_NONE;")
    lines.append("}")
    lines.append("")
    lines.append("static const replay_fn REPLAY[] = {" +
                 ", ".join(f"r_{i}" for i in range(len(names))) + "};")
    lines.append(f"static const int NREPLAY = {len(names)};")
    lines.append(TAPE_API)
    lines.append("static PyMethodDef methods[] = {")
    lines.append("  {\"bind\", ncf_bind, METH_VARARGS, \"bind(index, address)\"},")
    for fn in ("tape_new", "tape_begin", "tape_end", "tape_hold", "tape_invalidate", "tape_replay",
               "tape_size", "tape_tag"):
        lines.append(f"  {{\"{fn}\", py_{fn}, METH_VARARGS, NULL}},")
    for idx, name in enumerate(names):
        lines.append(f"  {{\"{name}\", w_{idx}, METH_VARARGS, NULL}},")
    lines.append("  {NULL, NULL, 0, NULL}};")
    lines.append("")
    lines.append("static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, \"_ncffast\", NULL, -1, methods};")
    lines.append("PyMODINIT_FUNC PyInit__ncffast(void) {")
    lines.append("  PyObject* m = PyModule_Create(&mod);")
    lines.append("  if (!m) return NULL;")
    lines.append("  PyObject* names = PyTuple_New(%d);" % len(names))
    for idx, name in enumerate(names):
        lines.append(f"  PyTuple_SET_ITEM(names, {idx}, PyUnicode_FromString(\"{name}\"));")
    lines.append("  PyModule_AddObject(m, \"NAMES\", names);")
    lines.append("  return m;")
    lines.append("}")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(sys.argv[1])
