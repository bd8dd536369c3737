/*
 * info_rows.c -- the host side of the SB3 info contract: the per-env info rows of one
 * HedgingVecEnv step, served from the step's pinned host columns without building a dict
 * per row.
 *
 * SB3 reads every row of `infos` on every step: collect_rollouts' _update_info_buffer calls
 * info.get("episode") / info.get("is_success") for each env, and the reference evaluation
 * loop (src/agents/train_ppo_v2.py:481-501) reads 9 keys per env.  A row there is a dict of
 * the env's info keys (hedging_env_v2.py:268-293) plus SB3's "TimeLimit.truncated", and on a
 * done row "terminal_observation" and Monitor's "episode" (train_ppo_v2.py:119,127-141).  A
 * dict per row costs ~0.3 us to build (20 ms per step at 65,536 envs, C or Python alike:
 * the allocation is the cost), so here:
 *
 *   Rows   the list: len(), rows[i], rows[a:b], iteration (subclassable: InfoView,
 *          cantorrl_amd/vec_env.py, is one; its _load() is called on the first row access
 *          and must call _attach()).  Row objects are made on first access and cached, so
 *          rows[i] is rows[i] and an item stored into a row stays.
 *   Row    one env's info: a read-only window on the columns (row[k], row.get(k, d), k in
 *          row) until something needs the whole mapping (keys / items / values / iteration /
 *          len / copy / repr / ==, an assignment or a deletion); it then becomes a plain dict
 *          it forwards to.  A done row's extra items ("terminal_observation", "episode") come
 *          from ends(i) at that moment, so a step in which no row is done reads only columns.
 *
 *   rows._attach(keys, cols, kinds, n, extra_key, extra_value, done, done_keys, ends)
 *     keys        tuple of str: the column keys, in row order
 *     cols        tuple of C-contiguous buffers, one per key, each >= n elements
 *     kinds       bytes, a type code per key: 'd' f64 -> float, 'f' f32 -> float, 'i' i32 -> int
 *     extra_key   a key every row holds with extra_value ("TimeLimit.truncated"), or None
 *     done        None, or a buffer of n bytes (nonzero: the row is done)
 *     done_keys   tuple of the keys only done rows hold (looked up through ends)
 *     ends        callable ends(i) -> dict of done row i's extra items (called once per row)
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

#define MAX_KEYS 64

/* ------------------------------------------------------------------ the columns (shared) */
typedef struct {
    PyObject_HEAD
    Py_ssize_t n, nk, held;
    PyObject* keys;
    PyObject* extra_key;
    PyObject* extra_val;
    PyObject* done_keys;
    PyObject* ends;
    int has_done;
    Py_buffer done;
    char kinds[MAX_KEYS];
    Py_hash_t hash[MAX_KEYS];      /* the column keys' hashes: a miss costs no string compare */
    Py_hash_t extra_hash;
    Py_ssize_t n_done_keys;
    Py_hash_t done_hash[MAX_KEYS];
    Py_buffer buf[MAX_KEYS];
} Cols;

static void cols_dealloc(Cols* c) {
    PyObject_GC_UnTrack(c);
    for (Py_ssize_t k = 0; k < c->held; ++k) PyBuffer_Release(&c->buf[k]);
    if (c->has_done) PyBuffer_Release(&c->done);
    Py_XDECREF(c->keys);
    Py_XDECREF(c->extra_key);
    Py_XDECREF(c->extra_val);
    Py_XDECREF(c->done_keys);
    Py_XDECREF(c->ends);
    PyObject_GC_Del(c);
}

static int cols_traverse(Cols* c, visitproc visit, void* arg) {
    Py_VISIT(c->extra_val);
    Py_VISIT(c->ends);
    return 0;
}

static PyTypeObject ColsType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "cantorrl_amd._info_rows._Cols",
    .tp_basicsize = sizeof(Cols),
    .tp_dealloc = (destructor)cols_dealloc,
    .tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC,
    .tp_traverse = (traverseproc)cols_traverse,
};

static inline PyObject* col_value(const Cols* c, Py_ssize_t k, Py_ssize_t i) {
    switch (c->kinds[k]) {
        case 'd': return PyFloat_FromDouble(((const double*)c->buf[k].buf)[i]);
        case 'f': return PyFloat_FromDouble((double)((const float*)c->buf[k].buf)[i]);
        default: return PyLong_FromLong((long)((const int32_t*)c->buf[k].buf)[i]);
    }
}

static inline int row_done(const Cols* c, Py_ssize_t i) {
    return c->has_done && ((const uint8_t*)c->done.buf)[i] != 0;
}

/* index of `key` (hash h) among keys (-1 none, -2 error): the hash first (a str caches its
 * own), then identity (the keys are interned literals on both sides in practice), then
 * equality -- as a dict lookup does */
static Py_ssize_t key_index(PyObject* keys, const Py_hash_t* hashes, Py_ssize_t nk, PyObject* key, Py_hash_t h) {
    for (Py_ssize_t k = 0; k < nk; ++k) {
        if (hashes[k] != h) continue;
        PyObject* kk = PyTuple_GET_ITEM(keys, k);
        if (kk == key) return k;
        const int eq = PyObject_RichCompareBool(kk, key, Py_EQ);
        if (eq < 0) return -2;
        if (eq) return k;
    }
    return -1;
}

static int key_eq(PyObject* a, Py_hash_t ha, PyObject* key, Py_hash_t h) {
    if (a == Py_None || ha != h) return 0;
    if (a == key) return 1;
    return PyObject_RichCompareBool(a, key, Py_EQ);
}

/* ------------------------------------------------------------------ one row */
typedef struct {
    PyObject_HEAD
    Cols* c;
    Py_ssize_t i;
    PyObject* d;   /* the row as a dict once materialized, else NULL */
} Row;

static PyTypeObject RowType;

/* A Row is not a GC object: 65,536 of them per step at SB3's loop would trigger the cyclic
 * collector's generation-0 pass every 700 and, through the long-lived count, full passes over
 * every object of the process (torch's included): 90 ms per step measured, against 25 ms.
 * A Row refers to its Cols (no cycle: a Cols never refers to a Row) and, once materialized,
 * to its dict; a cycle through that dict (a row stored into itself) is not collected. */
static PyObject* row_new(Cols* c, Py_ssize_t i) {
    Row* r = PyObject_New(Row, &RowType);
    if (!r) return NULL;
    Py_INCREF(c);
    r->c = c;
    r->i = i;
    r->d = NULL;
    return (PyObject*)r;
}

static void row_dealloc(Row* r) {
    Py_XDECREF(r->c);
    Py_XDECREF(r->d);
    PyObject_Del(r);
}

/* the whole row as a dict (made once; the row then forwards to it) */
static PyObject* row_dict(Row* r) {
    if (r->d) return r->d;
    const Cols* c = r->c;
    PyObject* d = PyDict_New();
    if (!d) return NULL;
    for (Py_ssize_t k = 0; k < c->nk; ++k) {
        PyObject* v = col_value(c, k, r->i);
        if (!v || PyDict_SetItem(d, PyTuple_GET_ITEM(c->keys, k), v) < 0) {
            Py_XDECREF(v);
            Py_DECREF(d);
            return NULL;
        }
        Py_DECREF(v);
    }
    if (c->extra_key != Py_None && PyDict_SetItem(d, c->extra_key, c->extra_val) < 0) {
        Py_DECREF(d);
        return NULL;
    }
    if (row_done(c, r->i) && c->ends != Py_None) {
        PyObject* e = PyObject_CallFunction(c->ends, "n", r->i);
        if (!e || PyDict_Update(d, e) < 0) {
            Py_XDECREF(e);
            Py_DECREF(d);
            return NULL;
        }
        Py_DECREF(e);
    }
    r->d = d;
    return d;
}

/* 1 found (*out a new reference), 0 missing, -1 error */
static int row_find(Row* r, PyObject* key, PyObject** out) {
    if (r->d) {
        PyObject* v = PyDict_GetItemWithError(r->d, key);
        if (v) {
            Py_INCREF(v);
            *out = v;
            return 1;
        }
        return PyErr_Occurred() ? -1 : 0;
    }
    const Cols* c = r->c;
    const Py_hash_t h = PyObject_Hash(key);
    if (h == -1) return -1;
    const Py_ssize_t k = key_index(c->keys, c->hash, c->nk, key, h);
    if (k == -2) return -1;
    if (k >= 0) {
        *out = col_value(c, k, r->i);
        return *out ? 1 : -1;
    }
    int eq = key_eq(c->extra_key, c->extra_hash, key, h);
    if (eq < 0) return -1;
    if (eq) {
        Py_INCREF(c->extra_val);
        *out = c->extra_val;
        return 1;
    }
    if (row_done(c, r->i)) {
        const Py_ssize_t m = key_index(c->done_keys, c->done_hash, c->n_done_keys, key, h);
        if (m == -2) return -1;
        if (m >= 0) {
            if (!row_dict(r)) return -1;
            return row_find(r, key, out);
        }
    }
    return 0;
}

static PyObject* row_subscript(Row* r, PyObject* key) {
    PyObject* v = NULL;
    const int f = row_find(r, key, &v);
    if (f > 0) return v;
    if (f == 0) PyErr_SetObject(PyExc_KeyError, key);
    return NULL;
}

static int row_ass_subscript(Row* r, PyObject* key, PyObject* v) {
    PyObject* d = row_dict(r);
    if (!d) return -1;
    return v ? PyDict_SetItem(d, key, v) : PyDict_DelItem(d, key);
}

static Py_ssize_t row_length(Row* r) {
    PyObject* d = row_dict(r);
    return d ? PyDict_GET_SIZE(d) : -1;
}

static int row_contains(Row* r, PyObject* key) {
    PyObject* v = NULL;
    const int f = row_find(r, key, &v);
    Py_XDECREF(v);
    return f;
}

static PyObject* row_get(Row* r, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs < 1 || nargs > 2) {
        PyErr_SetString(PyExc_TypeError, "get expected 1 or 2 arguments");
        return NULL;
    }
    PyObject* v = NULL;
    const int f = row_find(r, args[0], &v);
    if (f > 0) return v;
    if (f < 0) return NULL;
    PyObject* dflt = nargs == 2 ? args[1] : Py_None;
    Py_INCREF(dflt);
    return dflt;
}

static PyObject* row_forward(Row* r, const char* name) {
    PyObject* d = row_dict(r);
    return d ? PyObject_CallMethod(d, name, NULL) : NULL;
}
static PyObject* row_keys(Row* r, PyObject* u) { return row_forward(r, "keys"); }
static PyObject* row_values(Row* r, PyObject* u) { return row_forward(r, "values"); }
static PyObject* row_items(Row* r, PyObject* u) { return row_forward(r, "items"); }
static PyObject* row_copy(Row* r, PyObject* u) { return row_forward(r, "copy"); }

static PyObject* row_pop(Row* r, PyObject* const* args, Py_ssize_t nargs) {
    PyObject* d = row_dict(r);
    if (!d) return NULL;
    PyObject* m = PyObject_GetAttrString(d, "pop");
    if (!m) return NULL;
    PyObject* out = PyObject_Vectorcall(m, args, nargs, NULL);
    Py_DECREF(m);
    return out;
}

static PyObject* row_setdefault(Row* r, PyObject* const* args, Py_ssize_t nargs) {
    PyObject* d = row_dict(r);
    if (!d) return NULL;
    PyObject* m = PyObject_GetAttrString(d, "setdefault");
    if (!m) return NULL;
    PyObject* out = PyObject_Vectorcall(m, args, nargs, NULL);
    Py_DECREF(m);
    return out;
}

static PyObject* row_update(Row* r, PyObject* args, PyObject* kw) {
    PyObject* d = row_dict(r);
    if (!d) return NULL;
    PyObject* m = PyObject_GetAttrString(d, "update");
    if (!m) return NULL;
    PyObject* out = PyObject_Call(m, args, kw);
    Py_DECREF(m);
    return out;
}

static PyObject* row_iter(Row* r) {
    PyObject* d = row_dict(r);
    return d ? PyObject_GetIter(d) : NULL;
}

static PyObject* row_repr(Row* r) {
    PyObject* d = row_dict(r);
    return d ? PyObject_Repr(d) : NULL;
}

static PyObject* row_richcompare(Row* r, PyObject* other, int op) {
    if (op != Py_EQ && op != Py_NE) Py_RETURN_NOTIMPLEMENTED;
    PyObject* d = row_dict(r);
    if (!d) return NULL;
    PyObject* o = other;
    if (Py_TYPE(other) == &RowType) {
        o = row_dict((Row*)other);
        if (!o) return NULL;
    } else if (!PyDict_Check(other)) {
        Py_RETURN_NOTIMPLEMENTED;
    }
    return PyObject_RichCompare(d, o, op);
}

static PyMethodDef row_methods[] = {
    {"get", (PyCFunction)(void (*)(void))row_get, METH_FASTCALL, "get(key, default=None)"},
    {"keys", (PyCFunction)row_keys, METH_NOARGS, NULL},
    {"values", (PyCFunction)row_values, METH_NOARGS, NULL},
    {"items", (PyCFunction)row_items, METH_NOARGS, NULL},
    {"copy", (PyCFunction)row_copy, METH_NOARGS, "the row as a new dict"},
    {"pop", (PyCFunction)(void (*)(void))row_pop, METH_FASTCALL, NULL},
    {"setdefault", (PyCFunction)(void (*)(void))row_setdefault, METH_FASTCALL, NULL},
    {"update", (PyCFunction)(void (*)(void))row_update, METH_VARARGS | METH_KEYWORDS, NULL},
    {NULL, NULL, 0, NULL},
};

static PyMappingMethods row_as_mapping = {
    .mp_length = (lenfunc)row_length,
    .mp_subscript = (binaryfunc)row_subscript,
    .mp_ass_subscript = (objobjargproc)row_ass_subscript,
};

static PySequenceMethods row_as_sequence = {
    .sq_contains = (objobjproc)row_contains,
};

static PyTypeObject RowType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "cantorrl_amd._info_rows.Row",
    .tp_basicsize = sizeof(Row),
    .tp_dealloc = (destructor)row_dealloc,
    .tp_repr = (reprfunc)row_repr,
    .tp_as_sequence = &row_as_sequence,
    .tp_as_mapping = &row_as_mapping,
    .tp_hash = PyObject_HashNotImplemented,
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "One env's info of one step (a dict once anything needs the whole mapping).",
    .tp_richcompare = (richcmpfunc)row_richcompare,
    .tp_iter = (getiterfunc)row_iter,
    .tp_methods = row_methods,
};

/* ------------------------------------------------------------------ the list of rows */
typedef struct {
    PyObject_HEAD
    Cols* c;          /* NULL until _attach */
    PyObject* cache;  /* list of n rows (None until made) */
} Rows;

static int rows_traverse(Rows* s, visitproc visit, void* arg) {
    Py_VISIT(s->c);
    Py_VISIT(s->cache);
    return 0;
}

static int rows_clear(Rows* s) {
    Py_CLEAR(s->cache);
    Py_CLEAR(s->c);
    return 0;
}

static void rows_dealloc(Rows* s) {
    PyObject_GC_UnTrack(s);
    rows_clear(s);
    Py_TYPE(s)->tp_free((PyObject*)s);
}

static int rows_ready(Rows* s) {
    if (s->c) return 0;
    PyObject* r = PyObject_CallMethod((PyObject*)s, "_load", NULL);
    if (!r) return -1;
    Py_DECREF(r);
    if (!s->c) {
        PyErr_SetString(PyExc_RuntimeError, "Rows._load() did not call _attach()");
        return -1;
    }
    return 0;
}

static PyObject* rows_attach(Rows* s, PyObject* args) {
    PyObject *keys, *cols, *extra_key, *extra_val, *done, *done_keys, *ends;
    const char* kinds;
    Py_ssize_t nkinds, n;
    if (!PyArg_ParseTuple(args, "O!O!y#nOOOO!O", &PyTuple_Type, &keys, &PyTuple_Type, &cols, &kinds, &nkinds, &n,
                          &extra_key, &extra_val, &done, &PyTuple_Type, &done_keys, &ends))
        return NULL;
    const Py_ssize_t nk = PyTuple_GET_SIZE(keys);
    if (PyTuple_GET_SIZE(cols) != nk || nkinds != nk || nk > MAX_KEYS || n < 0) {
        PyErr_SetString(PyExc_ValueError, "_attach: keys, cols and kinds must have one length (<= 64); n >= 0");
        return NULL;
    }
    if (ends != Py_None && !PyCallable_Check(ends)) {
        PyErr_SetString(PyExc_TypeError, "_attach: ends must be callable or None");
        return NULL;
    }
    Cols* c = PyObject_GC_New(Cols, &ColsType);
    if (!c) return NULL;
    c->n = n;
    c->nk = nk;
    c->held = 0;
    c->has_done = 0;
    Py_INCREF(keys);
    c->keys = keys;
    Py_INCREF(extra_key);
    c->extra_key = extra_key;
    Py_INCREF(extra_val);
    c->extra_val = extra_val;
    Py_INCREF(done_keys);
    c->done_keys = done_keys;
    Py_INCREF(ends);
    c->ends = ends;
    c->extra_hash = 0;
    c->n_done_keys = 0;
    PyObject_GC_Track(c);
    if (extra_key != Py_None && (c->extra_hash = PyObject_Hash(extra_key)) == -1) goto fail;
    if (PyTuple_GET_SIZE(done_keys) > MAX_KEYS) {
        PyErr_SetString(PyExc_ValueError, "_attach: at most 64 done keys");
        goto fail;
    }
    for (Py_ssize_t k = 0; k < PyTuple_GET_SIZE(done_keys); ++k)
        if ((c->done_hash[k] = PyObject_Hash(PyTuple_GET_ITEM(done_keys, k))) == -1) goto fail;
    c->n_done_keys = PyTuple_GET_SIZE(done_keys);
    for (Py_ssize_t k = 0; k < nk; ++k)
        if ((c->hash[k] = PyObject_Hash(PyTuple_GET_ITEM(keys, k))) == -1) goto fail;
    for (Py_ssize_t k = 0; k < nk; ++k) {
        const char t = kinds[k];
        const Py_ssize_t isz = (t == 'd') ? 8 : (t == 'f' || t == 'i') ? 4 : 0;
        if (!isz) {
            PyErr_Format(PyExc_ValueError, "_attach: unknown type code %c", t);
            goto fail;
        }
        c->kinds[k] = t;
        if (PyObject_GetBuffer(PyTuple_GET_ITEM(cols, k), &c->buf[k], PyBUF_C_CONTIGUOUS) < 0) goto fail;
        ++c->held;
        if (c->buf[k].len < n * isz) {
            PyErr_Format(PyExc_ValueError, "_attach: column %zd holds %zd bytes, %zd needed", k, c->buf[k].len,
                         n * isz);
            goto fail;
        }
    }
    if (done != Py_None) {
        if (PyObject_GetBuffer(done, &c->done, PyBUF_C_CONTIGUOUS) < 0) goto fail;
        c->has_done = 1;
        if (c->done.len < n) {
            PyErr_Format(PyExc_ValueError, "_attach: done holds %zd bytes, %zd needed", c->done.len, n);
            goto fail;
        }
    }
    PyObject* cache = PyList_New(n);
    if (!cache) goto fail;
    for (Py_ssize_t i = 0; i < n; ++i) {
        Py_INCREF(Py_None);
        PyList_SET_ITEM(cache, i, Py_None);
    }
    Py_XSETREF(s->cache, cache);
    Py_XSETREF(s->c, c);
    Py_RETURN_NONE;
fail:
    Py_DECREF(c);
    return NULL;
}

static PyObject* rows_item(Rows* s, Py_ssize_t i) {
    if (rows_ready(s) < 0) return NULL;
    if (i < 0 || i >= s->c->n) {
        PyErr_SetString(PyExc_IndexError, "info index out of range");
        return NULL;
    }
    PyObject* r = PyList_GET_ITEM(s->cache, i);
    if (r == Py_None) {
        r = row_new(s->c, i);
        if (!r) return NULL;
        PyList_SET_ITEM(s->cache, i, r);   /* steals; the None it replaces is released */
        Py_DECREF(Py_None);
    }
    Py_INCREF(r);
    return r;
}

static PyObject* rows_subscript(Rows* s, PyObject* key) {
    if (PyIndex_Check(key)) {
        Py_ssize_t i = PyNumber_AsSsize_t(key, PyExc_IndexError);
        if (i == -1 && PyErr_Occurred()) return NULL;
        if (rows_ready(s) < 0) return NULL;
        if (i < 0) i += s->c->n;
        return rows_item(s, i);
    }
    if (PySlice_Check(key)) {
        if (rows_ready(s) < 0) return NULL;
        Py_ssize_t start, stop, step;
        if (PySlice_Unpack(key, &start, &stop, &step) < 0) return NULL;
        const Py_ssize_t len = PySlice_AdjustIndices(s->c->n, &start, &stop, step);
        PyObject* out = PyList_New(len);
        if (!out) return NULL;
        for (Py_ssize_t j = 0, i = start; j < len; ++j, i += step) {
            PyObject* r = rows_item(s, i);
            if (!r) {
                Py_DECREF(out);
                return NULL;
            }
            PyList_SET_ITEM(out, j, r);
        }
        return out;
    }
    PyErr_Format(PyExc_TypeError, "info indices must be integers or slices, not %.200s", Py_TYPE(key)->tp_name);
    return NULL;
}

static Py_ssize_t rows_length(Rows* s) {
    if (rows_ready(s) < 0) return -1;
    return s->c->n;
}

/* the rows' iterator: rows_item in index order */
typedef struct {
    PyObject_HEAD
    Rows* s;
    Py_ssize_t i;
} RowsIter;

static void rowsiter_dealloc(RowsIter* it) {
    Py_XDECREF(it->s);
    PyObject_Del(it);
}

static PyObject* rowsiter_next(RowsIter* it) {
    if (!it->s || it->i >= it->s->c->n) return NULL;
    return rows_item(it->s, it->i++);
}

static PyTypeObject RowsIterType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "cantorrl_amd._info_rows._RowsIter",
    .tp_basicsize = sizeof(RowsIter),
    .tp_dealloc = (destructor)rowsiter_dealloc,
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_iter = PyObject_SelfIter,
    .tp_iternext = (iternextfunc)rowsiter_next,
};

static PyObject* rows_iter(Rows* s) {
    if (rows_ready(s) < 0) return NULL;
    RowsIter* it = PyObject_New(RowsIter, &RowsIterType);
    if (!it) return NULL;
    Py_INCREF(s);
    it->s = s;
    it->i = 0;
    return (PyObject*)it;
}

static PyObject* rows_attached(Rows* s, void* u) { return PyBool_FromLong(s->c != NULL); }

static PyMethodDef rows_methods[] = {
    {"_attach", (PyCFunction)rows_attach, METH_VARARGS,
     "_attach(keys, cols, kinds, n, extra_key, extra_value, done, done_keys, ends)"},
    {NULL, NULL, 0, NULL},
};

static PyGetSetDef rows_getset[] = {
    {"_attached", (getter)rows_attached, NULL, "the columns are attached", NULL},
    {NULL, NULL, NULL, NULL, NULL},
};

static PyMappingMethods rows_as_mapping = {
    .mp_length = (lenfunc)rows_length,
    .mp_subscript = (binaryfunc)rows_subscript,
};

static PySequenceMethods rows_as_sequence = {
    .sq_length = (lenfunc)rows_length,
    .sq_item = (ssizeargfunc)rows_item,
};

static PyTypeObject RowsType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "cantorrl_amd._info_rows.Rows",
    .tp_basicsize = sizeof(Rows),
    .tp_dealloc = (destructor)rows_dealloc,
    .tp_as_sequence = &rows_as_sequence,
    .tp_as_mapping = &rows_as_mapping,
    .tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE | Py_TPFLAGS_HAVE_GC,
    .tp_doc = "A step's info rows (list-like); subclasses define _load(), which calls _attach().",
    .tp_traverse = (traverseproc)rows_traverse,
    .tp_clear = (inquiry)rows_clear,
    .tp_iter = (getiterfunc)rows_iter,
    .tp_methods = rows_methods,
    .tp_getset = rows_getset,
    .tp_new = PyType_GenericNew,
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_info_rows", NULL, -1, NULL, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__info_rows(void) {
    if (PyType_Ready(&ColsType) < 0 || PyType_Ready(&RowType) < 0 || PyType_Ready(&RowsType) < 0 ||
        PyType_Ready(&RowsIterType) < 0)
        return NULL;
    PyObject* m = PyModule_Create(&module);
    if (!m) return NULL;
    Py_INCREF(&RowType);
    Py_INCREF(&RowsType);
    if (PyModule_AddObject(m, "Row", (PyObject*)&RowType) < 0 || PyModule_AddObject(m, "Rows", (PyObject*)&RowsType) < 0) {
        Py_DECREF(m);
        return NULL;
    }
    return m;
}
