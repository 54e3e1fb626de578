/* sedhost.c — host-side C for the edit-script half of the path, as a
 * CPython extension module `_sedhost`.
 *
 * Once the DP and the traceback run on the GPU, a 4096 x 4096 pair spends more time in
 * Python building the edit-script dicts, patching and writing JSON than on the device.
 * These functions reproduce the reference's results exactly:
 *
 *   es_from_ops(ops, str1, str2)  generate_es over the canonical path given as op codes
 *                                 (StringEditDistance.py:274-334, index -1 quirk included)
 *   rev_es(es)                    generate_rev_es (:338-369), sharing the same dict objects
 *   seq_from_es(es)               generate_sequence_from_es (:371-377)
 *   patching(es, str1)            patching (:380-457), Python slicing semantics
 *   es_json(es, indent)           json.dumps({'edit_script': es}, indent=indent) (gui.py:629-638)
 *
 * Each function returns NotImplemented for inputs outside its fast path (non-dict records,
 * multi-character 'character' values, indices that do not fit a C long, non-ASCII text in
 * JSON ...); the Python wrappers then run the Python restatement, so results never differ.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static PyObject *K_OPERATION, *K_SOURCE, *K_DESTINATION, *K_CHARACTER, *K_INDEX;
static PyObject *S_INSERT, *S_DELETE, *S_UPDATE;

/* ------------------------------------------------------------------ es_from_ops */
/* Leaves shared by every record (immutable objects, so sharing is invisible to callers): the one-character strings
 * of code points < 256 (CPython's own singletons, looked up without a call) and the index ints 0 .. G_INTS_MAX - 1,
 * created once and kept, so a 4096^2 script's ~8500 index ints are neither allocated nor freed per call. */
#define G_INTS_MAX (1 << 20)
static PyObject *g_chars[256];
static PyObject **g_ints;
static Py_ssize_t g_nints;

static int ints_reserve(Py_ssize_t want) {
    if (want <= g_nints) return 0;
    if (want > G_INTS_MAX) want = G_INTS_MAX;
    if (want <= g_nints) return 0;
    PyObject **p = (PyObject **)PyMem_Realloc(g_ints, sizeof(PyObject *) * (size_t)want);
    if (!p) {
        PyErr_NoMemory();
        return -1;
    }
    g_ints = p;
    for (Py_ssize_t k = g_nints; k < want; ++k) {
        if (!(g_ints[k] = PyLong_FromSsize_t(k))) {
            g_nints = k;
            return -1;
        }
    }
    g_nints = want;
    return 0;
}

static PyObject *int_of(Py_ssize_t i) {
    if (i >= 0 && i < g_nints) {
        Py_INCREF(g_ints[i]);
        return g_ints[i];
    }
    return PyLong_FromSsize_t(i);
}

static PyObject *char_at(PyObject *s, Py_ssize_t len, Py_ssize_t i) {
    if (i < 0) i += len;
    if (i < 0 || i >= len) {
        PyErr_SetString(PyExc_IndexError, "string index out of range");
        return NULL;
    }
    if (PyUnicode_KIND(s) == PyUnicode_1BYTE_KIND) {
        PyObject *ch = g_chars[((const unsigned char *)PyUnicode_DATA(s))[i]];
        Py_INCREF(ch);
        return ch;
    }
    return PyUnicode_Substring(s, i, i + 1);
}

static PyObject *side(PyObject *s, Py_ssize_t len, Py_ssize_t i) {
    PyObject *ch = char_at(s, len, i);
    if (!ch) return NULL;
    PyObject *idx = int_of(i);
    PyObject *d = PyDict_New();
    if (!idx || !d || PyDict_SetItem(d, K_CHARACTER, ch) || PyDict_SetItem(d, K_INDEX, idx)) {
        Py_XDECREF(d);
        d = NULL;
    }
    Py_DECREF(ch);
    Py_XDECREF(idx);
    return d;
}

static PyObject *es_from_ops_impl(PyObject *self, PyObject *args) {
    Py_buffer ops;
    PyObject *s1, *s2;
    if (!PyArg_ParseTuple(args, "y*UU", &ops, &s1, &s2)) return NULL;
    const unsigned char *op = (const unsigned char *)ops.buf;
    const Py_ssize_t n = ops.len, l1 = PyUnicode_GET_LENGTH(s1), l2 = PyUnicode_GET_LENGTH(s2);
    PyObject *out = NULL;
    if (PyUnicode_READY(s1) < 0 || PyUnicode_READY(s2) < 0 || ints_reserve((l1 > l2 ? l1 : l2) + 1) < 0) goto fail;
    out = PyList_New(n);
    if (!out) goto fail;
    Py_ssize_t r = 0, c = 0;
    for (Py_ssize_t k = 0; k < n; ++k) {
        if (op[k] > 2) {
            PyErr_SetString(PyExc_ValueError, "op code > 2");
            goto fail;
        }
        if (op[k] != 1) ++c;
        if (op[k] != 0) ++r;
        PyObject *src = side(s1, l1, r - 1);
        if (!src) goto fail;
        PyObject *dst = side(s2, l2, c - 1);
        if (!dst) {
            Py_DECREF(src);
            goto fail;
        }
        PyObject *rec = PyDict_New();
        PyObject *name = op[k] == 0 ? S_INSERT : (op[k] == 1 ? S_DELETE : S_UPDATE);
        if (!rec || PyDict_SetItem(rec, K_OPERATION, name) || PyDict_SetItem(rec, K_SOURCE, src) ||
            PyDict_SetItem(rec, K_DESTINATION, dst)) {
            Py_XDECREF(rec);
            Py_DECREF(src);
            Py_DECREF(dst);
            goto fail;
        }
        Py_DECREF(src);
        Py_DECREF(dst);
        PyList_SET_ITEM(out, k, rec);
    }
    PyBuffer_Release(&ops);
    return out;
fail:
    Py_XDECREF(out);
    PyBuffer_Release(&ops);
    return NULL;
}

/* ------------------------------------------------------------------ helpers on records */
/* str equality with the interned-pointer shortcut (generated records share the interned names) */
static int eq(PyObject *a, PyObject *b) {
    if (a == b) return 1;
    if (!PyUnicode_Check(a)) return 0;
    return PyUnicode_GET_LENGTH(a) == PyUnicode_GET_LENGTH(b) && PyUnicode_Compare(a, b) == 0;
}

/* borrowed rec[key] when rec is a dict holding it, else NULL without an exception set */
static PyObject *get(PyObject *rec, PyObject *key) {
    if (!PyDict_CheckExact(rec)) return NULL;
    return PyDict_GetItemWithError(rec, key);
}

#define NOT_IMPL() \
    do {           \
        Py_RETURN_NOTIMPLEMENTED; \
    } while (0)

/* ------------------------------------------------------------------ rev_es */
static PyObject *rev_es_impl(PyObject *self, PyObject *es) {
    if (!PyList_CheckExact(es)) NOT_IMPL();
    const Py_ssize_t n = PyList_GET_SIZE(es);
    /* validate first: any record outside the fast path -> Python restatement */
    for (Py_ssize_t k = 0; k < n; ++k) {
        PyObject *rec = PyList_GET_ITEM(es, k), *op, *src, *dst;
        if (!(op = get(rec, K_OPERATION)) || !(src = get(rec, K_SOURCE)) || !(dst = get(rec, K_DESTINATION))) {
            if (PyErr_Occurred()) return NULL;
            NOT_IMPL();
        }
        if (!PyUnicode_CheckExact(op)) NOT_IMPL();
        const int isd = eq(op, S_DELETE);
        if (!isd && !eq(op, S_INSERT) && !eq(op, S_UPDATE)) NOT_IMPL();
        if (isd) {
            PyObject *i = get(dst, K_INDEX), *ch = get(dst, K_CHARACTER);
            if (!i || !ch || !PyLong_CheckExact(i)) {
                if (PyErr_Occurred()) return NULL;
                NOT_IMPL();
            }
        }
    }
    PyObject *out = PyList_New(n);
    if (!out) return NULL;
    for (Py_ssize_t k = 0; k < n; ++k) {
        PyObject *rec = PyList_GET_ITEM(es, k);
        PyObject *op = get(rec, K_OPERATION), *src = get(rec, K_SOURCE), *dst = get(rec, K_DESTINATION);
        PyObject *nop, *nsrc, *ndst = src;
        if (eq(op, S_INSERT)) {
            nop = S_DELETE;
            nsrc = dst;
            Py_INCREF(nsrc);
        } else if (eq(op, S_DELETE)) {
            nop = S_INSERT;
            PyObject *one = PyLong_FromLong(1);
            PyObject *i = one ? PyNumber_Subtract(get(dst, K_INDEX), one) : NULL;
            Py_XDECREF(one);
            nsrc = PyDict_New();
            if (!i || !nsrc || PyDict_SetItem(nsrc, K_INDEX, i) ||
                PyDict_SetItem(nsrc, K_CHARACTER, get(dst, K_CHARACTER))) {
                Py_XDECREF(i);
                Py_XDECREF(nsrc);
                Py_DECREF(out);
                return NULL;
            }
            Py_DECREF(i);
        } else {
            nop = S_UPDATE;
            nsrc = dst;
            Py_INCREF(nsrc);
        }
        PyObject *r = PyDict_New();
        if (!r || PyDict_SetItem(r, K_OPERATION, nop) || PyDict_SetItem(r, K_SOURCE, nsrc) ||
            PyDict_SetItem(r, K_DESTINATION, ndst)) {
            Py_XDECREF(r);
            Py_DECREF(nsrc);
            Py_DECREF(out);
            return NULL;
        }
        Py_DECREF(nsrc);
        PyList_SET_ITEM(out, k, r);
    }
    return out;
}

/* ------------------------------------------------------------------ seq_from_es */
/* fast path: every record a dict with a str operation; non-inserts have a 1-char str source char */
static int source_chars(PyObject *es, Py_UCS4 **buf, Py_ssize_t *len) {
    const Py_ssize_t n = PyList_GET_SIZE(es);
    Py_UCS4 *b = PyMem_Malloc(sizeof(Py_UCS4) * (n ? n : 1));
    if (!b) {
        PyErr_NoMemory();
        return -1;
    }
    Py_ssize_t m = 0;
    for (Py_ssize_t k = 0; k < n; ++k) {
        PyObject *rec = PyList_GET_ITEM(es, k), *op = get(rec, K_OPERATION), *src, *ch;
        if (!op || !PyUnicode_CheckExact(op)) goto bail;
        if (eq(op, S_INSERT)) continue;
        if (!(src = get(rec, K_SOURCE)) || !(ch = get(src, K_CHARACTER))) goto bail;
        if (!PyUnicode_CheckExact(ch) || PyUnicode_GET_LENGTH(ch) != 1) goto bail;
        b[m++] = PyUnicode_READ_CHAR(ch, 0);
    }
    *buf = b;
    *len = m;
    return 0;
bail:
    PyMem_Free(b);
    return PyErr_Occurred() ? -1 : 1;
}

static PyObject *seq_from_es(PyObject *self, PyObject *es) {
    if (!PyList_CheckExact(es)) NOT_IMPL();
    Py_UCS4 *b;
    Py_ssize_t m;
    const int rc = source_chars(es, &b, &m);
    if (rc < 0) return NULL;
    if (rc > 0) NOT_IMPL();
    PyObject *s = PyUnicode_FromKindAndData(PyUnicode_4BYTE_KIND, b, m);
    PyMem_Free(b);
    return s;
}

/* ------------------------------------------------------------------ patching */
typedef struct {
    Py_UCS4 *p;
    Py_ssize_t len, cap;
} ubuf;

static int ub_reserve(ubuf *u, Py_ssize_t want) {
    if (want <= u->cap) return 0;
    Py_ssize_t cap = u->cap ? u->cap : 64;
    while (cap < want) cap *= 2;
    Py_UCS4 *q = PyMem_Realloc(u->p, sizeof(Py_UCS4) * cap);
    if (!q) {
        PyErr_NoMemory();
        return -1;
    }
    u->p = q;
    u->cap = cap;
    return 0;
}

/* Python slice bound: s[:k] / s[k:] with k possibly negative or past the end */
static Py_ssize_t norm(long long k, Py_ssize_t len) {
    if (k < 0) k += len;
    if (k < 0) k = 0;
    if (k > len) k = len;
    return (Py_ssize_t)k;
}

/* out = s[:a] + (ch or nothing) + s[b:], with a = norm(k), b = norm(k2) (b may be < a) */
static int splice(ubuf *u, long long k, long long k2, int have_ch, Py_UCS4 ch) {
    const Py_ssize_t a = norm(k, u->len), b = norm(k2, u->len);
    const Py_ssize_t tail = u->len - b, nlen = a + (have_ch ? 1 : 0) + tail;
    if (b >= a) {  /* in place: shift the tail */
        if (ub_reserve(u, nlen)) return -1;
        memmove(u->p + a + (have_ch ? 1 : 0), u->p + b, sizeof(Py_UCS4) * tail);
        if (have_ch) u->p[a] = ch;
        u->len = nlen;
        return 0;
    }
    /* overlapping slices (negative index quirks): build a fresh buffer */
    Py_UCS4 *q = PyMem_Malloc(sizeof(Py_UCS4) * (nlen ? nlen : 1));
    if (!q) {
        PyErr_NoMemory();
        return -1;
    }
    memcpy(q, u->p, sizeof(Py_UCS4) * a);
    if (have_ch) q[a] = ch;
    memcpy(q + a + (have_ch ? 1 : 0), u->p + b, sizeof(Py_UCS4) * tail);
    PyMem_Free(u->p);
    u->p = q;
    u->len = u->cap = nlen;
    if (!nlen) u->cap = 1;
    return 0;
}

static int long_of(PyObject *o, long long *v) {
    if (!o || !PyLong_CheckExact(o)) return 1;
    int ovf = 0;
    *v = PyLong_AsLongLongAndOverflow(o, &ovf);
    if (ovf || *v > (1LL << 40) || *v < -(1LL << 40)) return 1;
    return 0;
}

typedef struct {
    long long si, di;
    Py_UCS4 sch, dch;  /* source char (non-inserts), destination char (updates / inserts) */
    signed char op;    /* 0 insert, 1 delete, 2 update, -1 other (reads indices, applies nothing) */
} prec;

static PyObject *patching(PyObject *self, PyObject *args) {
    PyObject *es, *s1;
    if (!PyArg_ParseTuple(args, "OO", &es, &s1)) return NULL;
    if (!PyList_CheckExact(es) || !PyUnicode_CheckExact(s1)) NOT_IMPL();
    const Py_ssize_t n = PyList_GET_SIZE(es);
    prec *pr = PyMem_Malloc(sizeof(prec) * (n ? n : 1));
    if (!pr) return PyErr_NoMemory();
    /* one pass: validate every record (the reference reads both indices of every record, the
     * source character of every non-insert and the destination character of updates/inserts) */
    Py_ssize_t olen = 0;
    for (Py_ssize_t k = 0; k < n; ++k) {
        PyObject *rec = PyList_GET_ITEM(es, k), *op = get(rec, K_OPERATION), *src, *dst, *ch;
        if (!op || !PyUnicode_CheckExact(op) || !(src = get(rec, K_SOURCE)) || !(dst = get(rec, K_DESTINATION)) ||
            long_of(get(src, K_INDEX), &pr[k].si) || long_of(get(dst, K_INDEX), &pr[k].di))
            goto notimpl;
        pr[k].op = eq(op, S_INSERT) ? 0 : eq(op, S_DELETE) ? 1 : eq(op, S_UPDATE) ? 2 : -1;
        if (pr[k].op != 0) {
            ch = get(src, K_CHARACTER);
            if (!ch || !PyUnicode_CheckExact(ch) || PyUnicode_GET_LENGTH(ch) != 1) goto notimpl;
            pr[k].sch = PyUnicode_READ_CHAR(ch, 0);
            ++olen;
        }
        if (pr[k].op == 0 || pr[k].op == 2) {
            ch = get(dst, K_CHARACTER);
            if (!ch || !PyUnicode_CheckExact(ch) || PyUnicode_GET_LENGTH(ch) != 1) goto notimpl;
            pr[k].dch = PyUnicode_READ_CHAR(ch, 0);
        }
    }
    /* error code: str1 == generate_sequence_from_es(es) ? 0 : (len(str1) >= its length ? 1 : -1) */
    const Py_ssize_t l1 = PyUnicode_GET_LENGTH(s1);
    int err = 0;
    if (l1 == olen) {
        const int kind = PyUnicode_KIND(s1);
        const void *data = PyUnicode_DATA(s1);
        Py_ssize_t i = 0;
        for (Py_ssize_t k = 0; k < n && !err; ++k)
            if (pr[k].op != 0 && PyUnicode_READ(kind, data, i++) != pr[k].sch) err = 1;
    } else {
        err = l1 >= olen ? 1 : -1;
    }
    if (err == -1) {
        PyMem_Free(pr);
        return Py_BuildValue("(is)", -1, "");
    }
    ubuf u = {0, 0, 0};
    if (ub_reserve(&u, l1 + n + 1) || !PyUnicode_AsUCS4(s1, u.p, u.cap, 0)) {
        PyMem_Free(u.p);
        PyMem_Free(pr);
        return NULL;
    }
    u.len = l1;
    long long removed = 0, inserted = 0;
    for (Py_ssize_t k = 0; k < n; ++k) {
        const long long at = pr[k].op == 0 ? pr[k].di : pr[k].si + removed + inserted;
        int e = 0;
        if (pr[k].op == 2) {
            if (at >= 0 && at < u.len) u.p[at] = pr[k].dch; /* s[:at] + ch + s[at+1:] */
            else e = splice(&u, at, at + 1, 1, pr[k].dch);
        } else if (pr[k].op == 1) {
            e = splice(&u, at, at + 1, 0, 0);
            removed -= 1;
        } else if (pr[k].op == 0) {
            e = splice(&u, at, at, 1, pr[k].dch);
            inserted += 1;
        }
        if (e) {
            PyMem_Free(u.p);
            PyMem_Free(pr);
            return NULL;
        }
    }
    PyMem_Free(pr);
    PyObject *res = PyUnicode_FromKindAndData(PyUnicode_4BYTE_KIND, u.p, u.len);
    PyMem_Free(u.p);
    if (!res) return NULL;
    return Py_BuildValue("(iN)", err, res);
notimpl:
    PyMem_Free(pr);
    if (PyErr_Occurred()) return NULL;
    Py_RETURN_NOTIMPLEMENTED;
}

/* ------------------------------------------------------------------ es_json */
typedef struct {
    char *p;
    size_t len, cap;
} cbuf;

static int cb_put(cbuf *b, const char *s, size_t n) {
    if (b->len + n > b->cap) {
        size_t cap = b->cap ? b->cap : 4096;
        while (cap < b->len + n) cap *= 2;
        char *q = PyMem_Realloc(b->p, cap);
        if (!q) {
            PyErr_NoMemory();
            return -1;
        }
        b->p = q;
        b->cap = cap;
    }
    memcpy(b->p + b->len, s, n);
    b->len += n;
    return 0;
}
static int cb_str(cbuf *b, const char *s) { return cb_put(b, s, strlen(s)); }
static int cb_nl(cbuf *b, int depth, int indent) {
    static const char nl[] = "\n                                                                ";  /* 64 spaces */
    const int n = depth * indent;  /* depth <= 4, indent <= 16 */
    return cb_put(b, nl, (size_t)(1 + n));
}

/* a JSON string for a 1-char printable-ASCII str (json.dumps escapes '"' and '\\') */
static int json_char(cbuf *b, PyObject *ch) {
    if (!ch || !PyUnicode_CheckExact(ch) || PyUnicode_GET_LENGTH(ch) != 1) return 1;
    const Py_UCS4 c = PyUnicode_READ_CHAR(ch, 0);
    if (c < 0x20 || c > 0x7e) return 1;
    char tmp[5] = {'"', 0, 0, 0, 0};
    int k = 1;
    if (c == '"' || c == '\\') tmp[k++] = '\\';
    tmp[k++] = (char)c;
    tmp[k++] = '"';
    return cb_put(b, tmp, k) ? -1 : 0;
}

static int json_side(cbuf *b, PyObject *d, int depth, int indent) {
    if (!d || !PyDict_CheckExact(d) || PyDict_GET_SIZE(d) != 2) return 1;
    /* key order as stored: {'character', 'index'} (generate_es) or {'index', 'character'} (rev of a delete) */
    PyObject *key, *val;
    Py_ssize_t pos = 0;
    if (cb_put(b, "{", 1)) return -1;
    int first = 1;
    while (PyDict_Next(d, &pos, &key, &val)) {
        if (!first && cb_put(b, ",", 1)) return -1;
        first = 0;
        if (cb_nl(b, depth + 1, indent)) return -1;
        if (eq(key, K_CHARACTER)) {
            if (cb_str(b, "\"character\": ")) return -1;
            const int r = json_char(b, val);
            if (r) return r;
        } else if (eq(key, K_INDEX)) {
            long long v;
            if (long_of(val, &v)) return 1;
            char num[32];
            snprintf(num, sizeof num, "\"index\": %lld", v);
            if (cb_str(b, num)) return -1;
        } else {
            return 1;
        }
    }
    if (cb_nl(b, depth, indent) || cb_put(b, "}", 1)) return -1;
    return 0;
}

static PyObject *es_json(PyObject *self, PyObject *args) {
    PyObject *es;
    int indent = 4;
    if (!PyArg_ParseTuple(args, "O|i", &es, &indent)) return NULL;
    if (!PyList_CheckExact(es) || indent < 0 || indent > 16) NOT_IMPL();
    cbuf b = {0, 0, 0};
    int r = 0;
    const Py_ssize_t n = PyList_GET_SIZE(es);
    if ((r = cb_put(&b, "{", 1)) || (r = cb_nl(&b, 1, indent)) || (r = cb_str(&b, "\"edit_script\": ["))) goto done;
    if (n == 0) {
        if ((r = cb_str(&b, "]"))) goto done;
    }
    for (Py_ssize_t k = 0; k < n && !r; ++k) {
        PyObject *rec = PyList_GET_ITEM(es, k);
        if (!PyDict_CheckExact(rec) || PyDict_GET_SIZE(rec) != 3) {
            r = 1;
            break;
        }
        PyObject *op = get(rec, K_OPERATION), *src = get(rec, K_SOURCE), *dst = get(rec, K_DESTINATION);
        if (!op || !src || !dst || !PyUnicode_CheckExact(op)) {
            r = 1;
            break;
        }
        const char *name = eq(op, S_INSERT)   ? "insert"
                           : eq(op, S_DELETE) ? "delete"
                           : eq(op, S_UPDATE) ? "update"
                                                                  : NULL;
        if (!name) {
            r = 1;
            break;
        }
        /* keys must be stored in the order operation, source, destination */
        PyObject *key, *val;
        Py_ssize_t pos = 0, i = 0;
        PyObject *order[3] = {K_OPERATION, K_SOURCE, K_DESTINATION};
        while (PyDict_Next(rec, &pos, &key, &val))
            if (!eq(key, order[i++])) r = 1;
        if (r) break;
        if (k && (r = cb_put(&b, ",", 1))) break;
        if ((r = cb_nl(&b, 2, indent)) || (r = cb_put(&b, "{", 1)) || (r = cb_nl(&b, 3, indent)) ||
            (r = cb_str(&b, "\"operation\": \"")) || (r = cb_str(&b, name)) || (r = cb_str(&b, "\",")) ||
            (r = cb_nl(&b, 3, indent)) || (r = cb_str(&b, "\"source\": ")) || (r = json_side(&b, src, 3, indent)) ||
            (r = cb_put(&b, ",", 1)) || (r = cb_nl(&b, 3, indent)) || (r = cb_str(&b, "\"destination\": ")) ||
            (r = json_side(&b, dst, 3, indent)) || (r = cb_nl(&b, 2, indent)) || (r = cb_put(&b, "}", 1)))
            break;
    }
    if (!r && n && ((r = cb_nl(&b, 1, indent)) || (r = cb_put(&b, "]", 1)))) goto done;
    if (!r) {
        if ((r = cb_nl(&b, 0, indent)) || (r = cb_put(&b, "}", 1))) goto done;
    }
done:;
    PyObject *res = NULL;
    if (r == 0) res = PyUnicode_DecodeASCII(b.p, (Py_ssize_t)b.len, NULL);
    PyMem_Free(b.p);
    if (r < 0 || (r == 0 && !res)) return NULL;
    if (r > 0) {
        if (PyErr_Occurred()) return NULL;
        Py_RETURN_NOTIMPLEMENTED;
    }
    return res;
}

/* ------------------------------------------------------------------ module */
/* ------------------------------------------------------------------ GC pause
 * A 4096^2 script is ~5000 records = 15000 new dicts.  Every 700 container allocations the
 * cyclic GC runs a collection, which for this build loop is pure overhead: the records hold
 * only str/int leaves and cannot form cycles.  Pausing the collector for the build halves
 * es_from_ops' time; the objects stay visible to the next regular collection. */
static PyObject *es_from_ops(PyObject *self, PyObject *args) {
    const int was = PyGC_Disable();
    PyObject *r = es_from_ops_impl(self, args);
    if (was) PyGC_Enable();
    return r;
}

/* ------------------------------------------------------------------ ES skeletons
 * es_skeleton(count) -> (records, sides): `count` generate_es records whose values are still None, built ahead of the
 * op codes (the drop-in module builds them while the device computes the script), and a bytes object holding each
 * record's source and destination dict (borrowed pointers into the records) for es_fill.
 * es_fill(records, sides, ops, str1, str2) -> records: es_from_ops' values written into the first len(ops) records
 * (records past len(ops) are dropped; if there are fewer, the rest are built here).  The result equals
 * es_from_ops(ops, str1, str2). */
static int fill_side(PyObject *d, PyObject *s, Py_ssize_t len, Py_ssize_t i) {
    PyObject *ch = char_at(s, len, i);
    if (!ch) return -1;
    PyObject *idx = int_of(i);
    const int rc = (!idx || PyDict_SetItem(d, K_CHARACTER, ch) || PyDict_SetItem(d, K_INDEX, idx)) ? -1 : 0;
    Py_DECREF(ch);
    Py_XDECREF(idx);
    return rc;
}

static PyObject *es_skeleton_impl(PyObject *self, PyObject *args) {
    Py_ssize_t count;
    if (!PyArg_ParseTuple(args, "n", &count)) return NULL;
    if (count < 0) count = 0;
    PyObject *list = PyList_New(count), *sides = PyBytes_FromStringAndSize(NULL, 2 * count * (Py_ssize_t)sizeof(PyObject *));
    if (!list || !sides) goto fail;
    PyObject **sp = (PyObject **)PyBytes_AS_STRING(sides);
    for (Py_ssize_t k = 0; k < count; ++k) {
        PyObject *src = PyDict_New(), *dst = PyDict_New(), *rec = PyDict_New();
        if (!src || !dst || !rec || PyDict_SetItem(src, K_CHARACTER, Py_None) || PyDict_SetItem(src, K_INDEX, Py_None) ||
            PyDict_SetItem(dst, K_CHARACTER, Py_None) || PyDict_SetItem(dst, K_INDEX, Py_None) ||
            PyDict_SetItem(rec, K_OPERATION, Py_None) || PyDict_SetItem(rec, K_SOURCE, src) ||
            PyDict_SetItem(rec, K_DESTINATION, dst)) {
            Py_XDECREF(src);
            Py_XDECREF(dst);
            Py_XDECREF(rec);
            goto fail;
        }
        sp[2 * k] = src;  /* (borrowed: the record holds them) */
        sp[2 * k + 1] = dst;
        Py_DECREF(src);
        Py_DECREF(dst);
        PyList_SET_ITEM(list, k, rec);
    }
    PyObject *ret = PyTuple_Pack(2, list, sides);
    Py_DECREF(list);
    Py_DECREF(sides);
    return ret;
fail:
    Py_XDECREF(list);
    Py_XDECREF(sides);
    return NULL;
}

static PyObject *es_fill_impl(PyObject *self, PyObject *args) {
    PyObject *list, *sides, *s1, *s2;
    Py_buffer ops;
    if (!PyArg_ParseTuple(args, "O!O!y*UU", &PyList_Type, &list, &PyBytes_Type, &sides, &ops, &s1, &s2)) return NULL;
    const unsigned char *op = (const unsigned char *)ops.buf;
    const Py_ssize_t n = ops.len, l1 = PyUnicode_GET_LENGTH(s1), l2 = PyUnicode_GET_LENGTH(s2);
    Py_ssize_t have = PyList_GET_SIZE(list);
    if (PyBytes_GET_SIZE(sides) != 2 * have * (Py_ssize_t)sizeof(PyObject *)) {
        PyErr_SetString(PyExc_ValueError, "es_fill: records and sides differ");
        goto fail;
    }
    if (PyUnicode_READY(s1) < 0 || PyUnicode_READY(s2) < 0 || ints_reserve((l1 > l2 ? l1 : l2) + 1) < 0) goto fail;
    if (have > n) {  /* drop the records past the script */
        if (PyList_SetSlice(list, n, have, NULL) < 0) goto fail;
        have = n;
    }
    PyObject *const *sp = (PyObject *const *)PyBytes_AS_STRING(sides);
    Py_ssize_t r = 0, c = 0;
    for (Py_ssize_t k = 0; k < n; ++k) {
        if (op[k] > 2) {
            PyErr_SetString(PyExc_ValueError, "op code > 2");
            goto fail;
        }
        if (op[k] != 1) ++c;
        if (op[k] != 0) ++r;
        PyObject *name = op[k] == 0 ? S_INSERT : (op[k] == 1 ? S_DELETE : S_UPDATE);
        if (k < have) {
            if (PyDict_SetItem(PyList_GET_ITEM(list, k), K_OPERATION, name) || fill_side(sp[2 * k], s1, l1, r - 1) ||
                fill_side(sp[2 * k + 1], s2, l2, c - 1))
                goto fail;
        } else {  /* more ops than skeleton records: build the rest */
            PyObject *src = side(s1, l1, r - 1);
            if (!src) goto fail;
            PyObject *dst = side(s2, l2, c - 1);
            PyObject *rec = dst ? PyDict_New() : NULL;
            const int bad = !rec || PyDict_SetItem(rec, K_OPERATION, name) || PyDict_SetItem(rec, K_SOURCE, src) ||
                            PyDict_SetItem(rec, K_DESTINATION, dst) || PyList_Append(list, rec);
            Py_DECREF(src);
            Py_XDECREF(dst);
            Py_XDECREF(rec);
            if (bad) goto fail;
        }
    }
    PyBuffer_Release(&ops);
    Py_INCREF(list);
    return list;
fail:
    PyBuffer_Release(&ops);
    return NULL;
}

/* es_recycle(records, count) -> (records, sides) | None: a previous generate_es list, which the caller has checked no
 * one else holds, reused as the next call's skeleton: every record an exact dict held only by the list, with exactly
 * the keys operation, source, destination in that order, each side an exact dict held only by its record with exactly
 * character, index in that order (rev_es' records share side dicts: those lists are refused).  Records are appended up
 * to `count`.  The values stay until es_fill overwrites them.  None when any record does not qualify. */
static int side_reusable(PyObject *d) {
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    if (!PyDict_CheckExact(d) || Py_REFCNT(d) != 1 || PyDict_GET_SIZE(d) != 2) return 0;
    if (!PyDict_Next(d, &pos, &k, &v) || k != K_CHARACTER) return 0;
    if (!PyDict_Next(d, &pos, &k, &v) || k != K_INDEX) return 0;
    return 1;
}
static PyObject *es_recycle_impl(PyObject *self, PyObject *args) {
    PyObject *list;
    Py_ssize_t count;
    if (!PyArg_ParseTuple(args, "O!n", &PyList_Type, &list, &count)) return NULL;
    const Py_ssize_t have = PyList_GET_SIZE(list), total = have > count ? have : count;
    PyObject *sides = PyBytes_FromStringAndSize(NULL, 2 * total * (Py_ssize_t)sizeof(PyObject *));
    if (!sides) return NULL;
    PyObject **sp = (PyObject **)PyBytes_AS_STRING(sides);
    for (Py_ssize_t i = 0; i < have; ++i) {
        PyObject *rec = PyList_GET_ITEM(list, i), *k, *op, *src, *dst;
        Py_ssize_t pos = 0;
        if (!PyDict_CheckExact(rec) || Py_REFCNT(rec) != 1 || PyDict_GET_SIZE(rec) != 3 ||
            !PyDict_Next(rec, &pos, &k, &op) || k != K_OPERATION || !PyDict_Next(rec, &pos, &k, &src) ||
            k != K_SOURCE || !PyDict_Next(rec, &pos, &k, &dst) || k != K_DESTINATION || src == dst ||
            !side_reusable(src) || !side_reusable(dst)) {
            Py_DECREF(sides);
            Py_RETURN_NONE;
        }
        sp[2 * i] = src;
        sp[2 * i + 1] = dst;
    }
    for (Py_ssize_t i = have; i < total; ++i) {  /* (as es_skeleton) */
        PyObject *src = PyDict_New(), *dst = PyDict_New(), *rec = PyDict_New();
        if (!src || !dst || !rec || PyDict_SetItem(src, K_CHARACTER, Py_None) || PyDict_SetItem(src, K_INDEX, Py_None) ||
            PyDict_SetItem(dst, K_CHARACTER, Py_None) || PyDict_SetItem(dst, K_INDEX, Py_None) ||
            PyDict_SetItem(rec, K_OPERATION, Py_None) || PyDict_SetItem(rec, K_SOURCE, src) ||
            PyDict_SetItem(rec, K_DESTINATION, dst) || PyList_Append(list, rec)) {
            Py_XDECREF(src);
            Py_XDECREF(dst);
            Py_XDECREF(rec);
            Py_DECREF(sides);
            return NULL;
        }
        sp[2 * i] = src;
        sp[2 * i + 1] = dst;
        Py_DECREF(src);
        Py_DECREF(dst);
        Py_DECREF(rec);
    }
    return PyTuple_Pack(2, list, sides);
}

static PyObject *es_recycle(PyObject *self, PyObject *args) {
    const int was = PyGC_Disable();
    PyObject *r = es_recycle_impl(self, args);
    if (was) PyGC_Enable();
    return r;
}

static PyObject *es_skeleton(PyObject *self, PyObject *args) {
    const int was = PyGC_Disable();
    PyObject *r = es_skeleton_impl(self, args);
    if (was) PyGC_Enable();
    return r;
}

static PyObject *es_fill(PyObject *self, PyObject *args) {
    const int was = PyGC_Disable();
    PyObject *r = es_fill_impl(self, args);
    if (was) PyGC_Enable();
    return r;
}

static PyObject *rev_es(PyObject *self, PyObject *es) {
    const int was = PyGC_Disable();
    PyObject *r = rev_es_impl(self, es);
    if (was) PyGC_Enable();
    return r;
}

/* ------------------------------------------------------------------ co-optimal path lengths and count
 * Over the edge mask M of the full matrix ((n+1) x (m+1) bytes, bit 1 insert from the left, 2 delete
 * from above, 4 update from the diagonal; sed_full_matrix), for copaths.py.
 *
 * length_windows(M, n, m, words) -> (lmin, lmax, win) as bytes: per cell the shortest and longest
 * co-optimal origin->cell path (int32) and a window of 64*words bits, bit b set when a co-optimal path of
 * length lmin + b exists.  Exact for every path of total length <= lmin(sink) + 64*words - 1: a prefix
 * of such a path ends at a cell c with length <= lmin(c) + 64*words - 1, since lmin(c) plus the shortest
 * c->sink suffix is at least lmin(sink).  4097 x 4097 with words = 1: 268 MB instead of a Python bitset
 * of up to n+m bits per cell.
 *
 * count_paths(M, n, m) -> int: the number of co-optimal origin->sink paths, a row-by-row sum over the
 * optimal edges in multi-limb integers (two rows live), returned as a Python int. */
static PyObject *length_windows(PyObject *self, PyObject *args) {
    Py_buffer mb;
    Py_ssize_t n, m;
    int W;
    if (!PyArg_ParseTuple(args, "y*nni", &mb, &n, &m, &W)) return NULL;
    PyObject *ret = NULL, *bl = NULL, *bh = NULL, *bw = NULL;
    const Py_ssize_t cols = m + 1, cells = (n + 1) * cols;
    if (n < 0 || m < 0 || W < 1 || W > 1024 || mb.len < cells) {
        PyErr_SetString(PyExc_ValueError, "length_windows: bad shape");
        goto done;
    }
    bl = PyBytes_FromStringAndSize(NULL, 4 * cells);
    bh = PyBytes_FromStringAndSize(NULL, 4 * cells);
    bw = PyBytes_FromStringAndSize(NULL, 8 * (Py_ssize_t)W * cells);
    if (!bl || !bh || !bw) goto done;
    {
        const unsigned char *M = (const unsigned char *)mb.buf;
        int32_t *lo = (int32_t *)PyBytes_AS_STRING(bl), *hi = (int32_t *)PyBytes_AS_STRING(bh);
        uint64_t *win = (uint64_t *)PyBytes_AS_STRING(bw);
        Py_BEGIN_ALLOW_THREADS
        memset(win, 0, 8 * (size_t)W * (size_t)cells);
        lo[0] = hi[0] = 0;
        win[0] = 1;
        for (Py_ssize_t i = 0; i <= n; ++i) {
            for (Py_ssize_t j = 0; j <= m; ++j) {
                if (!i && !j) continue;
                const Py_ssize_t c = i * cols + j;
                const int mk = M[c] & 7;
                Py_ssize_t pr[3];
                int np_ = 0;
                if ((mk & 1) && j > 0) pr[np_++] = c - 1;
                if ((mk & 2) && i > 0) pr[np_++] = c - cols;
                if ((mk & 4) && i > 0 && j > 0) pr[np_++] = c - cols - 1;
                if (!np_) {  /* unreachable (not in a valid mask): no paths */
                    lo[c] = hi[c] = -1;
                    continue;
                }
                int32_t a = INT32_MAX, b = -1;
                for (int k = 0; k < np_; ++k) {
                    if (lo[pr[k]] < 0) continue;
                    if (lo[pr[k]] + 1 < a) a = lo[pr[k]] + 1;
                    if (hi[pr[k]] + 1 > b) b = hi[pr[k]] + 1;
                }
                if (b < 0) {
                    lo[c] = hi[c] = -1;
                    continue;
                }
                lo[c] = a;
                hi[c] = b;
                uint64_t *out = win + (size_t)W * (size_t)c;
                for (int k = 0; k < np_; ++k) {
                    if (lo[pr[k]] < 0) continue;
                    const uint64_t *in = win + (size_t)W * (size_t)pr[k];
                    const int sh = lo[pr[k]] + 1 - a, ws = sh >> 6, bs = sh & 63;
                    for (int t = W - 1; t >= ws; --t) {
                        uint64_t v = in[t - ws] << bs;
                        if (bs && t - ws - 1 >= 0) v |= in[t - ws - 1] >> (64 - bs);
                        out[t] |= v;
                    }
                }
            }
        }
        Py_END_ALLOW_THREADS
    }
    ret = PyTuple_Pack(3, bl, bh, bw);
done:
    Py_XDECREF(bl);
    Py_XDECREF(bh);
    Py_XDECREF(bw);
    PyBuffer_Release(&mb);
    return ret;
}

static PyObject *count_paths(PyObject *self, PyObject *args) {
    Py_buffer mb;
    Py_ssize_t n, m;
    if (!PyArg_ParseTuple(args, "y*nn", &mb, &n, &m)) return NULL;
    PyObject *ret = NULL;
    const Py_ssize_t cols = m + 1;
    uint64_t *prev = NULL, *cur = NULL;
    size_t cap = 1;  /* limbs per cell, both rows */
    if (n < 0 || m < 0 || mb.len < (n + 1) * cols) {
        PyErr_SetString(PyExc_ValueError, "count_paths: bad shape");
        goto done;
    }
    prev = calloc((size_t)cols * cap, 8);
    cur = calloc((size_t)cols * cap, 8);
    if (!prev || !cur) {
        PyErr_NoMemory();
        goto done;
    }
    {
        const unsigned char *M = (const unsigned char *)mb.buf;
        int oom = 0;
        Py_BEGIN_ALLOW_THREADS
        for (Py_ssize_t i = 0; i <= n && !oom; ++i) {
            for (Py_ssize_t j = 0; j <= m; ++j) {
                uint64_t *o = cur + (size_t)j * cap;
                memset(o, 0, 8 * cap);
                if (!i && !j) {
                    o[0] = 1;
                    continue;
                }
                const int mk = M[i * cols + j] & 7;
                const uint64_t *src[3];
                int ns = 0;
                if ((mk & 1) && j > 0) src[ns++] = cur + (size_t)(j - 1) * cap;
                if ((mk & 2) && i > 0) src[ns++] = prev + (size_t)j * cap;
                if ((mk & 4) && i > 0 && j > 0) src[ns++] = prev + (size_t)(j - 1) * cap;
                uint64_t carry_out = 0;
                for (int k = 0; k < ns; ++k) {
                    uint64_t carry = 0;
                    for (size_t t = 0; t < cap; ++t) {
                        uint64_t s1 = o[t] + src[k][t];
                        uint64_t c1 = s1 < o[t];
                        uint64_t s2 = s1 + carry;
                        c1 += s2 < s1;
                        o[t] = s2;
                        carry = c1;
                    }
                    carry_out += carry;
                }
                if (carry_out) {  /* grow every cell of both rows by one limb, then redo this cell */
                    const size_t nc = cap + 1;
                    uint64_t *np2 = calloc((size_t)cols * nc, 8), *nc2 = calloc((size_t)cols * nc, 8);
                    if (!np2 || !nc2) {
                        free(np2);
                        free(nc2);
                        oom = 1;
                        break;
                    }
                    for (Py_ssize_t x = 0; x <= m; ++x) {
                        memcpy(np2 + (size_t)x * nc, prev + (size_t)x * cap, 8 * cap);
                        memcpy(nc2 + (size_t)x * nc, cur + (size_t)x * cap, 8 * cap);
                    }
                    free(prev);
                    free(cur);
                    prev = np2;
                    cur = nc2;
                    cap = nc;
                    --j;  /* recompute cell j with the wider limbs */
                    continue;
                }
            }
            uint64_t *t = prev;
            prev = cur;
            cur = t;
        }
        Py_END_ALLOW_THREADS
        if (oom) {
            PyErr_NoMemory();
            goto done;
        }
        /* the last row finished is in prev */
        ret = _PyLong_FromByteArray((const unsigned char *)(prev + (size_t)m * cap), 8 * cap, 1, 0);
    }
done:
    free(prev);
    free(cur);
    PyBuffer_Release(&mb);
    return ret;
}

static PyMethodDef methods[] = {
    {"length_windows", length_windows, METH_VARARGS, "co-optimal path length windows per cell"},
    {"count_paths", count_paths, METH_VARARGS, "number of co-optimal paths (Python int)"},
    {"es_from_ops", es_from_ops, METH_VARARGS, "generate_es over a canonical op sequence"},
    {"es_skeleton", es_skeleton, METH_VARARGS, "generate_es records with their values still None, and their side dicts"},
    {"es_fill", es_fill, METH_VARARGS, "es_from_ops' values written into es_skeleton records"},
    {"es_recycle", es_recycle, METH_VARARGS, "a previous generate_es list no one else holds, as an es_skeleton"},
    {"rev_es", rev_es, METH_O, "generate_rev_es"},
    {"seq_from_es", seq_from_es, METH_O, "generate_sequence_from_es"},
    {"patching", patching, METH_VARARGS, "patching(es, str1) -> (error_code, str)"},
    {"es_json", es_json, METH_VARARGS, "json.dumps({'edit_script': es}, indent=indent)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_sedhost", NULL, -1, methods};

PyMODINIT_FUNC PyInit__sedhost(void) {
    K_OPERATION = PyUnicode_InternFromString("operation");
    K_SOURCE = PyUnicode_InternFromString("source");
    K_DESTINATION = PyUnicode_InternFromString("destination");
    K_CHARACTER = PyUnicode_InternFromString("character");
    K_INDEX = PyUnicode_InternFromString("index");
    S_INSERT = PyUnicode_InternFromString("insert");
    S_DELETE = PyUnicode_InternFromString("delete");
    S_UPDATE = PyUnicode_InternFromString("update");
    if (!K_OPERATION || !K_SOURCE || !K_DESTINATION || !K_CHARACTER || !K_INDEX || !S_INSERT || !S_DELETE ||
        !S_UPDATE)
        return NULL;
    for (int k = 0; k < 256; ++k)
        if (!(g_chars[k] = PyUnicode_FromOrdinal(k))) return NULL;
    return PyModule_Create(&moddef);
}
