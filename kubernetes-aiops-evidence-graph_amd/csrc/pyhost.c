/* _egr_pyhost: the host side of the drop-in rules boundary in native code.
 *
 * encode_rows  -- evidence dicts -> the row columns egr_rules_eval consumes (egraph/encode.py
 *                 is the same encoder in Python; both follow RulesEngine._process_*_evidence,
 *                 src/services/rca/rules_engine.py:294-376 of the reference).
 * assemble     -- kernel outputs -> the reference's hypothesis dicts
 *                 (rules_engine.py:235-262 / :457-478, hypothesis_ranker.py:63-71).
 *
 * Exactness rule for encode_rows: a row is taken here only when every value the reference
 * would read from it is of a plain built-in type (exact dict / list / str / int / bool / float
 * / None), where the row's Python expressions cannot run user code and cannot raise.  Any
 * other row -- a dict subclass, an unhashable reason, a None where a number is compared, a
 * string where a list is iterated -- is handed to the Python row encoder (`slow_row`), which
 * evaluates the reference's expressions in the reference's order and raises what they raise.
 * The fast path never raises on input data; it only decides "plain" or "hand over".
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

/* include/egraph.h EGR_F_* (kept in sync by tests/test_native_host.py) */
#define F_RECENT_DEPLOY  (1u << 0)
#define F_IMAGE_CHANGED  (1u << 1)
#define F_MEMORY_HIGH    (1u << 2)
#define F_HPA_AT_MAX     (1u << 3)
#define F_LATENCY_HIGH   (1u << 4)
#define F_NODE_ISSUE     (1u << 5)
#define F_NOT_READY      (1u << 6)
#define F_READINESS_FAIL (1u << 7)
#define F_ERR_FLOAT      (1u << 8)
#define NO_NODE 0xFFFFFFFFu
#define INT_LIMIT 2147483648.0   /* egraph/encode.py _INT_LIMIT */

enum { T_NONE, T_POD, T_DEPLOY, T_IMAGE, T_LOG, T_METRIC, T_NODE };

/* interned keys and constants */
static PyObject *k_id, *k_type, *k_data, *k_waiting, *k_terminated, *k_restart, *k_node_name,
    *k_conditions, *k_ctype, *k_status, *k_phase, *k_reason, *k_recent, *k_image_changed,
    *k_patterns, *k_error_count, *k_query, *k_anomalous, *k_current, *k_name, *k_ready_key;
static PyObject *s_ready, *s_true, *s_running, *s_cnr, *s_memory, *s_hpa, *s_max, *s_latency;
static PyObject *s_type_names[7];
static PyObject *i_zero, *i_one, *i_ninety;
static PyObject* type_map;   /* evidence_type name -> T_* (a dict lookup, like processors.get) */
/* hypothesis dict keys */
static PyObject *h_id, *h_incident, *h_category, *h_title, *h_description, *h_confidence,
    *h_rank, *h_support_ids, *h_actions, *h_generated_by, *h_rule_id, *h_support_count,
    *h_strength, *h_final;

static int intern_all(void) {
#define S(var, text) if (!(var = PyUnicode_InternFromString(text))) return -1
  S(k_id, "id"); S(k_type, "evidence_type"); S(k_data, "data");
  S(k_waiting, "waiting_reason"); S(k_terminated, "terminated_reason");
  S(k_restart, "restart_count"); S(k_node_name, "node_name"); S(k_conditions, "conditions");
  S(k_ctype, "type"); S(k_status, "status"); S(k_phase, "phase"); S(k_reason, "reason");
  S(k_recent, "is_recent_change"); S(k_image_changed, "image_changed");
  S(k_patterns, "patterns_found"); S(k_error_count, "error_count"); S(k_query, "query_name");
  S(k_anomalous, "is_anomalous"); S(k_current, "current_value"); S(k_name, "name");
  S(k_ready_key, "Ready");
  S(s_ready, "Ready"); S(s_true, "True"); S(s_running, "Running");
  S(s_cnr, "ContainersNotReady"); S(s_memory, "memory"); S(s_hpa, "hpa"); S(s_max, "max");
  S(s_latency, "latency");
  s_type_names[T_NONE] = NULL;
  S(s_type_names[T_POD], "kubernetes_pod"); S(s_type_names[T_DEPLOY], "deploy_change");
  S(s_type_names[T_IMAGE], "image_change"); S(s_type_names[T_LOG], "log_signal");
  S(s_type_names[T_METRIC], "metric_signal"); S(s_type_names[T_NODE], "kubernetes_node");
  S(h_id, "id"); S(h_incident, "incident_id"); S(h_category, "category"); S(h_title, "title");
  S(h_description, "description"); S(h_confidence, "confidence"); S(h_rank, "rank");
  S(h_support_ids, "supporting_evidence_ids"); S(h_actions, "recommended_actions");
  S(h_generated_by, "generated_by"); S(h_rule_id, "rule_id");
  S(h_support_count, "support_count"); S(h_strength, "signal_strength");
  S(h_final, "final_score");
#undef S
  if (!(type_map = PyDict_New())) return -1;
  for (int i = T_POD; i <= T_NODE; ++i) {
    PyObject* v = PyLong_FromLong(i);
    if (!v || PyDict_SetItem(type_map, s_type_names[i], v) < 0) return -1;
    Py_DECREF(v);
  }
  if (!(i_zero = PyLong_FromLong(0)) || !(i_one = PyLong_FromLong(1)) ||
      !(i_ninety = PyLong_FromLong(90)))
    return -1;
  return 0;
}

/* ---- plain-value helpers (no user code runs, nothing raises) ------------------------------ */

/* 1: value is of a plain built-in type (NULL = key missing counts as plain) */
static inline int plain(PyObject* o) {
  return o == NULL || o == Py_None || PyUnicode_CheckExact(o) || PyLong_CheckExact(o) ||
         PyBool_Check(o) || PyFloat_CheckExact(o) || PyList_CheckExact(o) ||
         PyDict_CheckExact(o);
}
static inline int is_num(PyObject* o) {
  return PyLong_CheckExact(o) || PyBool_Check(o) || PyFloat_CheckExact(o);
}
static inline int hashable_plain(PyObject* o) {
  return o == Py_None || PyUnicode_CheckExact(o) || PyLong_CheckExact(o) || PyBool_Check(o) ||
         PyFloat_CheckExact(o);
}
/* truthiness of a plain value (missing = None = falsy) */
static inline int truthy(PyObject* o) {
  if (o == NULL || o == Py_None) return 0;
  return PyObject_IsTrue(o);   /* built-in types: no user code, cannot fail */
}
/* `o == <str constant>` for a plain value: only an equal str compares equal */
static inline int eq_str(PyObject* o, PyObject* s) {
  return o != NULL && PyUnicode_CheckExact(o) && PyUnicode_Compare(o, s) == 0;
}
/* dict.get on an exact dict with an interned str key: borrowed or NULL (missing).  Returns -1
 * only if the lookup itself raised (a key whose __eq__ raises on a hash collision): hand over. */
static inline int dget(PyObject* d, PyObject* key, PyObject** out) {
  *out = PyDict_GetItemWithError(d, key);
  if (*out == NULL && PyErr_Occurred()) { PyErr_Clear(); return -1; }
  return 0;
}
/* number > / == constant for plain numbers (int, bool, float); cannot fail on these types */
static inline int num_cmp(PyObject* o, PyObject* c, int op) {
  return PyObject_RichCompareBool(o, c, op);
}
/* vocab lookup: bits of a hashable plain key, 0 when absent; -1 = hand over */
static inline int64_t vocab_bits(PyObject* vocab, PyObject* key) {
  if (!hashable_plain(key)) return -1;
  PyObject* v = PyDict_GetItemWithError(vocab, key);
  if (v == NULL) {
    if (PyErr_Occurred()) { PyErr_Clear(); return -1; }
    return 0;
  }
  unsigned long b = PyLong_AsUnsignedLong(v);
  if (b == (unsigned long)-1 && PyErr_Occurred()) { PyErr_Clear(); return -1; }
  return (int64_t)(b & 0xFFFFFFFFu);
}

typedef struct {
  PyObject *waiting, *terminated, *patterns, *node_keys;
} Vocab;

typedef struct {
  uint32_t flags, vocab, node;
  double err;
  PyObject* pending_node;   /* node_keys.setdefault(name) to apply when the row is accepted */
} Row;

/* Each returns 0 = encoded, 1 = hand the row to the Python encoder. */

static int enc_pod(PyObject* d, const Vocab* V, Row* r) {
  PyObject *wr, *tr, *rc, *nn, *conds;
  if (dget(d, k_waiting, &wr) || dget(d, k_terminated, &tr) || dget(d, k_restart, &rc) ||
      dget(d, k_node_name, &nn) || dget(d, k_conditions, &conds))
    return 1;
  if (!plain(wr) || !plain(tr) || !plain(nn)) return 1;
  if (rc != NULL && !is_num(rc)) return 1;              /* max(int, rc) needs a number */
  int wr_t = truthy(wr), tr_t = truthy(tr);
  if (wr_t) {                                            /* waiting_reasons.add (:318) */
    int64_t b = vocab_bits(V->waiting, wr);
    if (b < 0) return 1;
    r->vocab |= (uint32_t)b;
  }
  if (tr_t) {                                            /* terminated_reasons.add (:320) */
    int64_t b = vocab_bits(V->terminated, tr);
    if (b < 0) return 1;
    r->vocab |= (uint32_t)b;
  }
  int has_issue = wr_t || tr_t || (rc != NULL && num_cmp(rc, i_zero, Py_GT) == 1);
  if (truthy(nn) && has_issue) {                        /* pods_by_node[node_name] (:330) */
    if (!hashable_plain(nn)) return 1;
    r->pending_node = nn;
  }
  /* next(c for c in conditions if c.get("type") == "Ready") (:333-335) */
  PyObject* ready = NULL;
  if (conds != NULL) {
    if (!PyList_CheckExact(conds)) return 1;
    Py_ssize_t n = PyList_GET_SIZE(conds);
    for (Py_ssize_t i = 0; i < n && ready == NULL; ++i) {
      PyObject* c = PyList_GET_ITEM(conds, i);
      if (!PyDict_CheckExact(c)) return 1;
      PyObject* t;
      if (dget(c, k_ctype, &t) || !plain(t)) return 1;
      if (eq_str(t, s_ready)) ready = c;
    }
  }
  if (ready != NULL && PyDict_GET_SIZE(ready) > 0) {
    PyObject *st, *ph, *rs;
    if (dget(ready, k_status, &st) || !plain(st)) return 1;
    if (!eq_str(st, s_true)) {
      if (dget(d, k_phase, &ph) || !plain(ph)) return 1;
      if (eq_str(ph, s_running)) {
        r->flags |= F_NOT_READY;
        if (dget(ready, k_reason, &rs) || !plain(rs)) return 1;
        if (eq_str(rs, s_cnr)) r->flags |= F_READINESS_FAIL;
      }
    }
  }
  return 0;
}

static int enc_flag(PyObject* d, PyObject* key, uint32_t bit, Row* r) {
  PyObject* v;
  if (dget(d, key, &v) || !plain(v)) return 1;
  if (truthy(v)) r->flags |= bit;
  return 0;
}

static int enc_log(PyObject* d, const Vocab* V, Row* r) {
  PyObject *pf, *ec;
  if (dget(d, k_patterns, &pf) || dget(d, k_error_count, &ec)) return 1;
  if (pf != NULL) {                                      /* log_patterns.add (:353) */
    if (!PyList_CheckExact(pf)) return 1;
    Py_ssize_t n = PyList_GET_SIZE(pf);
    for (Py_ssize_t i = 0; i < n; ++i) {
      int64_t b = vocab_bits(V->patterns, PyList_GET_ITEM(pf, i));
      if (b < 0) return 1;
      r->vocab |= (uint32_t)b;
    }
  }
  if (ec == NULL) return 0;                              /* error_count += 0 (:354) */
  if (PyFloat_CheckExact(ec)) {
    double e = PyFloat_AS_DOUBLE(ec);
    if (!(isfinite(e) && floor(e) == e && fabs(e) < INT_LIMIT)) r->flags |= F_ERR_FLOAT;
    r->err = e;
  } else if (PyLong_CheckExact(ec) || PyBool_Check(ec)) {
    int overflow = 0;
    long long v = PyLong_AsLongLongAndOverflow(ec, &overflow);
    if (overflow) return 1;                              /* float(huge int): let Python decide */
    if (v >= (long long)INT_LIMIT || v <= -(long long)INT_LIMIT) r->flags |= F_ERR_FLOAT;
    r->err = (double)v;
  } else {
    return 1;
  }
  if (r->err == 0.0) r->err = 0.0;                       /* `if e:` leaves +0 for -0.0 */
  return 0;
}

static int contains(PyObject* q, PyObject* s) {
  return PyUnicode_Find(q, s, 0, PY_SSIZE_T_MAX, 1) >= 0;
}

static int enc_metric(PyObject* d, Row* r) {
  PyObject *q, *an, *cv;
  if (dget(d, k_query, &q) || dget(d, k_anomalous, &an) || dget(d, k_current, &cv)) return 1;
  if (q != NULL && !PyUnicode_CheckExact(q)) return 1;   /* `in` on a non-str: hand over */
  if (!plain(an) || !plain(cv)) return 1;
  if (q == NULL) return 0;                               /* "" contains none of the names */
  if (contains(q, s_memory) && truthy(an)) {             /* (:359-362) */
    if (cv != NULL && cv != Py_None) {
      if (!is_num(cv)) {
        if (truthy(cv)) return 1;                        /* "x" > 90 raises */
      } else if (truthy(cv) && num_cmp(cv, i_ninety, Py_GT) == 1) {
        r->flags |= F_MEMORY_HIGH;
      }
    }
  }
  if (contains(q, s_hpa) && contains(q, s_max)) {        /* (:364-365) */
    if (cv != NULL && is_num(cv) && num_cmp(cv, i_one, Py_EQ) == 1) r->flags |= F_HPA_AT_MAX;
  }
  if (contains(q, s_latency)) {                          /* (:367-368): missing -> 0 */
    if (cv != NULL) {
      if (!is_num(cv)) return 1;                         /* None / str > 1 raises */
      if (num_cmp(cv, i_one, Py_GT) == 1) r->flags |= F_LATENCY_HIGH;
    }
  }
  return 0;
}

static int enc_node(PyObject* d, Row* r) {
  PyObject *name, *conds, *ready = NULL, *st = NULL;
  if (dget(d, k_name, &name) || dget(d, k_conditions, &conds)) return 1;
  if (conds != NULL) {
    if (!PyDict_CheckExact(conds)) return 1;
    if (dget(conds, k_ready_key, &ready)) return 1;
    if (ready != NULL) {
      if (!PyDict_CheckExact(ready)) return 1;
      if (dget(ready, k_status, &st) || !plain(st)) return 1;
    }
  }
  if (!eq_str(st, s_true)) {                             /* node_issues[name] (:375-376) */
    if (name != NULL && !hashable_plain(name)) return 1;
    r->flags |= F_NODE_ISSUE;
  }
  return 0;
}

static int type_of(PyObject* t) {
  if (t == NULL || t == Py_None) return T_NONE;
  if (!PyUnicode_CheckExact(t)) return -1;
  PyObject* v = PyDict_GetItemWithError(type_map, t);   /* str keys: cannot raise */
  return v == NULL ? T_NONE : (int)PyLong_AS_LONG(v);
}

/* One row on the calling thread (GIL held): the fast path, or the Python row encoder for a row
 * it hands over.  `want_id`: also read the row's id (the first five rows of an incident).
 * Leaves row->pending_node for the caller (node_keys numbering follows row order).
 * Returns 0, or -1 with an exception set; *slow_res is a new reference to keep while *ev_id is used. */
static int encode_row_serial(PyObject* ev, const Vocab* V, PyObject* slow_row, int want_id, Row* row,
                             PyObject** ev_id, PyObject** slow_res, Py_ssize_t* n_slow) {
  Row r0 = {0, 0, NO_NODE, 0.0, NULL};
  *row = r0;
  *ev_id = NULL;
  *slow_res = NULL;
  int slow = 1;
  if (PyDict_CheckExact(ev)) {
    PyObject *t, *data;
    /* evidence_ids[:5] reads only the first five rows' ids (an exact dict's get of a str key
     * cannot raise or run user code, so skipping the rest changes nothing) */
    if (!(want_id && dget(ev, k_id, ev_id)) && !dget(ev, k_type, &t) && !dget(ev, k_data, &data)) {
      int ty = type_of(t);
      if (ty == T_NONE) {
        slow = hashable_plain(t == NULL ? Py_None : t) ? 0 : 1;
      } else if (ty > 0 && data != NULL && PyDict_CheckExact(data)) {
        switch (ty) {
          case T_POD: slow = enc_pod(data, V, row); break;
          case T_DEPLOY: slow = enc_flag(data, k_recent, F_RECENT_DEPLOY, row); break;
          case T_IMAGE: slow = enc_flag(data, k_image_changed, F_IMAGE_CHANGED, row); break;
          case T_LOG: slow = enc_log(data, V, row); break;
          case T_METRIC: slow = enc_metric(data, row); break;
          case T_NODE: slow = enc_node(data, row); break;
        }
      } else if (ty > 0 && data == NULL) {
        /* ev.get("data", {}) -> {}: every get misses */
        PyObject* empty = PyDict_New();
        if (!empty) return -1;
        switch (ty) {
          case T_POD: slow = enc_pod(empty, V, row); break;
          case T_DEPLOY: slow = 0; break;
          case T_IMAGE: slow = 0; break;
          case T_LOG: slow = enc_log(empty, V, row); break;
          case T_METRIC: slow = enc_metric(empty, row); break;
          case T_NODE: slow = enc_node(empty, row); break;
        }
        Py_DECREF(empty);
      }
    }
  }
  if (slow) {                                /* the Python encoder: same result or raise */
    ++*n_slow;
    row->pending_node = NULL;
    *slow_res = PyObject_CallOneArg(slow_row, ev);
    if (!*slow_res) return -1;
    unsigned int f, v, k;
    double e;
    PyObject* sid;
    if (!PyArg_ParseTuple(*slow_res, "OIIId", &sid, &f, &v, &k, &e)) {
      Py_CLEAR(*slow_res);
      return -1;
    }
    *ev_id = sid;
    row->flags = f; row->vocab = v; row->node = k; row->err = e;
  }
  return 0;
}

/* First-seen numbering of node names without the Python dict (the parallel pass's completion):
 * an open-addressing map over (content hash, name) -> index.  Equal only for equal characters of
 * ready exact strs -- exactly dict equality for such keys.  `materialize` writes the numbering
 * into node_keys (index order) when the dict has to take over or at the end. */
typedef struct {
  uint64_t* h;
  PyObject** key;
  uint32_t* idx;
  PyObject** by_idx;         /* names in index order */
  size_t cap, n;
} NodeMap;

static int nodemap_init(NodeMap* m, size_t want) {
  m->cap = 64;
  while (m->cap < 2 * want + 2) m->cap *= 2;
  m->n = 0;
  m->h = PyMem_Calloc(m->cap, sizeof(uint64_t));
  m->key = PyMem_Calloc(m->cap, sizeof(PyObject*));
  m->idx = PyMem_Calloc(m->cap, sizeof(uint32_t));
  m->by_idx = PyMem_Calloc(want + 1, sizeof(PyObject*));
  if (!m->h || !m->key || !m->idx || !m->by_idx) { PyErr_NoMemory(); return -1; }
  return 0;
}
static void nodemap_free(NodeMap* m) {
  PyMem_Free(m->h); PyMem_Free(m->key); PyMem_Free(m->idx); PyMem_Free(m->by_idx);
}
static inline int same_str(PyObject* a, PyObject* b) {
  return a == b || (PyUnicode_GET_LENGTH(a) == PyUnicode_GET_LENGTH(b) &&
                    PyUnicode_KIND(a) == PyUnicode_KIND(b) &&
                    memcmp(PyUnicode_DATA(a), PyUnicode_DATA(b),
                           (size_t)PyUnicode_GET_LENGTH(a) * (size_t)PyUnicode_KIND(a)) == 0);
}
/* the name's index, inserting it (capacity: at most `want` distinct names, checked by caller) */
static uint32_t nodemap_get(NodeMap* m, uint64_t h, PyObject* name) {
  size_t i = (size_t)(h ^ (h >> 29)) & (m->cap - 1);
  for (;;) {
    if (m->h[i] == 0) {
      m->h[i] = h;
      m->key[i] = name;
      m->idx[i] = (uint32_t)m->n;
      m->by_idx[m->n] = name;
      return (uint32_t)m->n++;
    }
    if (m->h[i] == h && same_str(m->key[i], name)) return m->idx[i];
    i = (i + 1) & (m->cap - 1);
  }
}
static int nodemap_materialize(NodeMap* m, PyObject* node_keys) {
  for (size_t j = 0; j < m->n; ++j) {
    PyObject* v = PyLong_FromSize_t(j);
    if (!v) return -1;
    const int rc = PyDict_SetItem(node_keys, m->by_idx[j], v);
    Py_DECREF(v);
    if (rc < 0) return -1;
  }
  m->n = 0;
  return 0;
}

/* node_keys.setdefault(name, len(node_keys)) -> the row's node key (a name seen before is a
 * plain lookup: no index object is built for it) */
static int resolve_node(const Vocab* V, Row* row) {
  if (row->pending_node == NULL) return 0;
  PyObject* seen = PyDict_GetItemWithError(V->node_keys, row->pending_node);
  if (seen != NULL) {
    row->node = (uint32_t)PyLong_AsUnsignedLong(seen);
    return 0;
  }
  if (PyErr_Occurred()) return -1;
  PyObject* idx = PyLong_FromSsize_t(PyDict_GET_SIZE(V->node_keys));
  if (!idx) return -1;
  PyObject* k = PyDict_SetDefault(V->node_keys, row->pending_node, idx);
  Py_DECREF(idx);
  if (!k) return -1;
  row->node = (uint32_t)PyLong_AsUnsignedLong(k);
  return 0;
}

/* ---- parallel row pass ---------------------------------------------------------------------
 * Large batches are encoded by worker threads while the calling thread keeps the GIL and waits,
 * so no Python code runs anywhere in the process during the pass and the evidence objects cannot
 * change.  The workers only READ objects: type checks, PyDict_Next scans (a dict "get" is a scan
 * matching the key's characters; a dict with any key that is not an exact str is handed back),
 * size / digit / character reads.  They never call into CPython's lookups, comparisons,
 * truth tests or allocators, and never touch a reference count.  A row they cannot take is
 * marked and redone, in row order, by encode_row_serial on the calling thread, which also
 * numbers the node keys and reads the ids -- so the result is the serial encoder's, bit for bit
 * (tests/test_pyhost.py runs both over the same rows). */
#include <pthread.h>

typedef struct {
  const void* data;
  Py_ssize_t len;
  int kind;
  uint32_t bits;
} WVocabEntry;

typedef struct {
  WVocabEntry* e;
  Py_ssize_t n;
} WVocab;

/* a str-keyed vocab dict as a flat table; -1 if it has a key that is not a ready exact str or a
 * value that is not an int in [0, 2^32) */
static int wvocab_build(PyObject* d, WVocab* out) {
  out->n = 0;
  out->e = PyMem_Malloc(sizeof(WVocabEntry) * (size_t)(PyDict_GET_SIZE(d) + 1));
  if (!out->e) return -1;
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(d, &pos, &k, &v)) {
    if (!PyUnicode_CheckExact(k) || !PyUnicode_IS_READY(k) || !PyLong_CheckExact(v)) return -1;
    unsigned long b = PyLong_AsUnsignedLong(v);
    if (b == (unsigned long)-1 && PyErr_Occurred()) { PyErr_Clear(); return -1; }
    WVocabEntry* e = &out->e[out->n++];
    e->data = PyUnicode_DATA(k);
    e->len = PyUnicode_GET_LENGTH(k);
    e->kind = PyUnicode_KIND(k);
    e->bits = (uint32_t)(b & 0xFFFFFFFFu);
  }
  return 0;
}

/* equal characters (two ready strs: PEP 393 keeps each in its narrowest kind, so equal strings
 * have equal kinds) */
static inline int w_str_eq(PyObject* a, const void* bd, Py_ssize_t blen, int bkind) {
  if (!PyUnicode_IS_READY(a)) return -1;
  if (PyUnicode_GET_LENGTH(a) != blen || PyUnicode_KIND(a) != bkind) return 0;
  return memcmp(PyUnicode_DATA(a), bd, (size_t)blen * (size_t)bkind) == 0;
}
static inline int w_eq_obj(PyObject* a, PyObject* b) {   /* b: one of our interned strs */
  if (a == b) return 1;
  return w_str_eq(a, PyUnicode_DATA(b), PyUnicode_GET_LENGTH(b), PyUnicode_KIND(b));
}

/* dict.get of n <= 8 keys (our interned strs, hashes cached) by one scan of an exact dict's
 * entries with their stored hashes.  A lookup compares only the entries whose hash equals the
 * key's, so only those are looked at: an exact ready str is matched by its characters; any
 * other key object there -- whose __eq__ the lookup would call -- hands the row over (1). */
static int w_get(PyObject* d, PyObject* const* keys, int n, PyObject** out) {
  Py_hash_t kh[8];
  for (int j = 0; j < n; ++j) {
    out[j] = NULL;
    kh[j] = ((PyASCIIObject*)keys[j])->hash;
  }
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  Py_hash_t h;
  while (_PyDict_Next(d, &pos, &k, &v, &h)) {
    for (int j = 0; j < n; ++j) {
      if (h != kh[j]) continue;
      if (k != keys[j]) {
        if (!PyUnicode_CheckExact(k)) return 1;
        const int eq = w_eq_obj(k, keys[j]);
        if (eq < 0) return 1;
        if (!eq) continue;
      }
      out[j] = v;
      break;
    }
  }
  return 0;
}

/* truth value of a plain value, by reading it (bool / int / float / str / list / dict / None) */
static inline int w_truthy(PyObject* o) {
  if (o == NULL || o == Py_None) return 0;
  if (PyBool_Check(o)) return o == Py_True;
  if (PyLong_CheckExact(o)) return Py_SIZE(o) != 0;
  if (PyFloat_CheckExact(o)) return PyFloat_AS_DOUBLE(o) != 0.0;
  if (PyUnicode_CheckExact(o)) return PyUnicode_GET_LENGTH(o) != 0;
  if (PyList_CheckExact(o)) return PyList_GET_SIZE(o) != 0;
  if (PyDict_CheckExact(o)) return PyDict_GET_SIZE(o) != 0;
  return -1;
}
static inline int w_eq_str(PyObject* o, PyObject* s) {
  if (o == NULL || !PyUnicode_CheckExact(o)) return 0;
  return w_eq_obj(o, s);      /* -1: not ready (hand over) */
}
/* plain number (int / bool / float) `op` a small int constant c: 1 / 0 (exact, as Python) */
static inline int w_num_cmp(PyObject* o, long c, int op) {
  if (PyFloat_CheckExact(o)) {
    const double x = PyFloat_AS_DOUBLE(o), y = (double)c;   /* small c: exact */
    return op == Py_GT ? x > y : x == y;
  }
  int ovf = 0;
  const long long x = PyLong_AsLongLongAndOverflow(o, &ovf);   /* exact int / bool: reads digits */
  if (ovf) return op == Py_GT ? ovf > 0 : 0;
  return op == Py_GT ? x > c : x == c;
}
/* vocab bits of a key: 0 absent; -1 hand over (a key that is not an exact str) */
static inline int64_t w_vocab_bits(const WVocab* V, PyObject* key) {
  if (!hashable_plain(key)) return -1;
  if (!PyUnicode_CheckExact(key) || !PyUnicode_IS_READY(key)) return -1;
  const Py_ssize_t len = PyUnicode_GET_LENGTH(key);
  const int kind = PyUnicode_KIND(key);
  const void* d = PyUnicode_DATA(key);
  for (Py_ssize_t i = 0; i < V->n; ++i)
    if (V->e[i].len == len && V->e[i].kind == kind &&
        memcmp(V->e[i].data, d, (size_t)len * (size_t)kind) == 0)
      return V->e[i].bits;
  return 0;
}
/* `s in q` for an ASCII constant s: 1 / 0 */
static int w_contains(PyObject* q, PyObject* s) {
  const Py_ssize_t n = PyUnicode_GET_LENGTH(q), m = PyUnicode_GET_LENGTH(s);
  const Py_UCS1* sd = PyUnicode_1BYTE_DATA(s);
  const int kind = PyUnicode_KIND(q);
  const void* qd = PyUnicode_DATA(q);
  for (Py_ssize_t i = 0; i + m <= n; ++i) {
    Py_ssize_t j = 0;
    while (j < m && PyUnicode_READ(kind, qd, i + j) == sd[j]) ++j;
    if (j == m) return 1;
  }
  return 0;
}

typedef struct {
  WVocab waiting, terminated, patterns;
} WVocabs;

static PyObject* K_EV[2];      /* evidence_type, data */
static PyObject* K_POD[6];     /* waiting, terminated, restart, node_name, conditions, phase */
static PyObject* K_COND[1];    /* type */
static PyObject* K_READY[2];   /* status, reason */
static PyObject* K_LOG[2];     /* patterns_found, error_count */
static PyObject* K_METRIC[3];  /* query_name, is_anomalous, current_value */
static PyObject* K_NODE[2];    /* name, conditions */

static int w_pod(PyObject* d, const WVocabs* V, Row* r) {
  PyObject* o[6];
  if (w_get(d, K_POD, 6, o)) return 1;
  PyObject *wr = o[0], *tr = o[1], *rc = o[2], *nn = o[3], *conds = o[4], *ph = o[5];
  if (!plain(wr) || !plain(tr) || !plain(nn)) return 1;
  if (rc != NULL && !is_num(rc)) return 1;
  const int wr_t = w_truthy(wr), tr_t = w_truthy(tr);
  if (wr_t < 0 || tr_t < 0) return 1;
  if (wr_t) {
    int64_t b = w_vocab_bits(&V->waiting, wr);
    if (b < 0) return 1;
    r->vocab |= (uint32_t)b;
  }
  if (tr_t) {
    int64_t b = w_vocab_bits(&V->terminated, tr);
    if (b < 0) return 1;
    r->vocab |= (uint32_t)b;
  }
  const int has_issue = wr_t || tr_t || (rc != NULL && w_num_cmp(rc, 0, Py_GT) == 1);
  const int nn_t = w_truthy(nn);
  if (nn_t < 0) return 1;
  if (nn_t && has_issue) {
    if (!hashable_plain(nn)) return 1;
    r->pending_node = nn;
  }
  PyObject* ready = NULL;
  if (conds != NULL) {
    if (!PyList_CheckExact(conds)) return 1;
    const Py_ssize_t n = PyList_GET_SIZE(conds);
    for (Py_ssize_t i = 0; i < n && ready == NULL; ++i) {
      PyObject* c = PyList_GET_ITEM(conds, i);
      if (!PyDict_CheckExact(c)) return 1;
      PyObject* t;
      if (w_get(c, K_COND, 1, &t) || !plain(t)) return 1;
      const int eq = w_eq_str(t, s_ready);
      if (eq < 0) return 1;
      if (eq) ready = c;
    }
  }
  if (ready != NULL && PyDict_GET_SIZE(ready) > 0) {
    PyObject* rr[2];
    if (w_get(ready, K_READY, 2, rr) || !plain(rr[0])) return 1;
    const int st_true = w_eq_str(rr[0], s_true);
    if (st_true < 0) return 1;
    if (!st_true) {
      if (!plain(ph)) return 1;
      const int running = w_eq_str(ph, s_running);
      if (running < 0) return 1;
      if (running) {
        r->flags |= F_NOT_READY;
        if (!plain(rr[1])) return 1;
        const int cnr = w_eq_str(rr[1], s_cnr);
        if (cnr < 0) return 1;
        if (cnr) r->flags |= F_READINESS_FAIL;
      }
    }
  }
  return 0;
}

static int w_flag(PyObject* d, PyObject* key, uint32_t bit, Row* r) {
  PyObject* v;
  if (w_get(d, &key, 1, &v) || !plain(v)) return 1;
  const int t = w_truthy(v);
  if (t < 0) return 1;
  if (t) r->flags |= bit;
  return 0;
}

static int w_log(PyObject* d, const WVocabs* V, Row* r) {
  PyObject* o[2];
  if (w_get(d, K_LOG, 2, o)) return 1;
  PyObject *pf = o[0], *ec = o[1];
  if (pf != NULL) {
    if (!PyList_CheckExact(pf)) return 1;
    const Py_ssize_t n = PyList_GET_SIZE(pf);
    for (Py_ssize_t i = 0; i < n; ++i) {
      int64_t b = w_vocab_bits(&V->patterns, PyList_GET_ITEM(pf, i));
      if (b < 0) return 1;
      r->vocab |= (uint32_t)b;
    }
  }
  if (ec == NULL) return 0;
  if (PyFloat_CheckExact(ec)) {
    const double e = PyFloat_AS_DOUBLE(ec);
    if (!(isfinite(e) && floor(e) == e && fabs(e) < INT_LIMIT)) r->flags |= F_ERR_FLOAT;
    r->err = e;
  } else if (PyLong_CheckExact(ec) || PyBool_Check(ec)) {
    int overflow = 0;
    const long long v = PyLong_AsLongLongAndOverflow(ec, &overflow);
    if (overflow) return 1;
    if (v >= (long long)INT_LIMIT || v <= -(long long)INT_LIMIT) r->flags |= F_ERR_FLOAT;
    r->err = (double)v;
  } else {
    return 1;
  }
  if (r->err == 0.0) r->err = 0.0;
  return 0;
}

static int w_metric(PyObject* d, Row* r) {
  PyObject* o[3];
  if (w_get(d, K_METRIC, 3, o)) return 1;
  PyObject *q = o[0], *an = o[1], *cv = o[2];
  if (q != NULL && (!PyUnicode_CheckExact(q) || !PyUnicode_IS_READY(q))) return 1;
  if (!plain(an) || !plain(cv)) return 1;
  if (q == NULL) return 0;
  const int an_t = w_truthy(an), cv_t = w_truthy(cv);
  if (an_t < 0 || cv_t < 0) return 1;
  if (w_contains(q, s_memory) && an_t) {
    if (cv != NULL && cv != Py_None) {
      if (!is_num(cv)) {
        if (cv_t) return 1;
      } else if (cv_t && w_num_cmp(cv, 90, Py_GT) == 1) {
        r->flags |= F_MEMORY_HIGH;
      }
    }
  }
  if (w_contains(q, s_hpa) && w_contains(q, s_max)) {
    if (cv != NULL && is_num(cv) && w_num_cmp(cv, 1, Py_EQ) == 1) r->flags |= F_HPA_AT_MAX;
  }
  if (w_contains(q, s_latency)) {
    if (cv != NULL) {
      if (!is_num(cv)) return 1;
      if (w_num_cmp(cv, 1, Py_GT) == 1) r->flags |= F_LATENCY_HIGH;
    }
  }
  return 0;
}

static int w_node(PyObject* d, Row* r) {
  PyObject* o[2];
  PyObject *ready = NULL, *st = NULL;
  if (w_get(d, K_NODE, 2, o)) return 1;
  PyObject *name = o[0], *conds = o[1];
  if (conds != NULL) {
    if (!PyDict_CheckExact(conds)) return 1;
    if (w_get(conds, &k_ready_key, 1, &ready)) return 1;
    if (ready != NULL) {
      if (!PyDict_CheckExact(ready)) return 1;
      if (w_get(ready, K_READY, 1, &st) || !plain(st)) return 1;
    }
  }
  const int st_true = w_eq_str(st, s_true);
  if (st_true < 0) return 1;
  if (!st_true) {
    if (name != NULL && !hashable_plain(name)) return 1;
    r->flags |= F_NODE_ISSUE;
  }
  return 0;
}

/* 0 = encoded, 1 = redo on the calling thread */
static int w_row(PyObject* ev, const WVocabs* V, Row* row) {
  if (!PyDict_CheckExact(ev)) return 1;
  PyObject* o[2];
  if (w_get(ev, K_EV, 2, o)) return 1;
  PyObject *t = o[0], *data = o[1];
  if (t == NULL || t == Py_None) return 0;                     /* no processor: nothing */
  if (!PyUnicode_CheckExact(t)) return 1;
  int ty = T_NONE;
  for (int i = T_POD; i <= T_NODE; ++i) {
    const int eq = w_eq_obj(t, s_type_names[i]);
    if (eq < 0) return 1;
    if (eq) { ty = i; break; }
  }
  if (ty == T_NONE) return 0;                                  /* unknown type: nothing */
  if (data == NULL || !PyDict_CheckExact(data)) return 1;      /* (missing data: serially) */
  switch (ty) {
    case T_POD: return w_pod(data, V, row);
    case T_DEPLOY: return w_flag(data, k_recent, F_RECENT_DEPLOY, row);
    case T_IMAGE: return w_flag(data, k_image_changed, F_IMAGE_CHANGED, row);
    case T_LOG: return w_log(data, V, row);
    case T_METRIC: return w_metric(data, row);
    case T_NODE: return w_node(data, row);
  }
  return 1;
}

/* FNV-1a over a ready exact str's kind, length and characters (never 0); 0 for anything else.
 * Equal strs have equal kinds (PEP 393), so equal strs hash equal. */
static inline uint64_t w_str_hash(PyObject* o) {
  if (!PyUnicode_CheckExact(o) || !PyUnicode_IS_READY(o)) return 0u;
  const Py_ssize_t len = PyUnicode_GET_LENGTH(o);
  const int kind = PyUnicode_KIND(o);
  const unsigned char* p = (const unsigned char*)PyUnicode_DATA(o);
  uint64_t h = 1469598103934665603ull ^ (uint64_t)kind ^ ((uint64_t)len << 8);
  for (Py_ssize_t i = 0; i < len * kind; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h ? h : 1u;
}

/* Software pipelining of the workers' row reads: a row costs a chain of dependent cache misses
 * (the dict, its keys table, each value object), so a worker touches rows ahead of the one it
 * works on -- row j + 6's dict, row j + 3's keys table, row j + 1's values -- and the misses of
 * the next rows overlap the current row's work.  Prefetches only: no value is used. */
static inline void row_prefetch(PyObject* evs, Py_ssize_t j, Py_ssize_t n) {
  if (j + 6 < n) __builtin_prefetch(PyList_GET_ITEM(evs, j + 6));
  if (j + 3 < n) {
    PyObject* d = PyList_GET_ITEM(evs, j + 3);
    if (PyDict_CheckExact(d)) {
      const char* k = (const char*)((PyDictObject*)d)->ma_keys;
      __builtin_prefetch(k);
      __builtin_prefetch(k + 64);
      __builtin_prefetch(k + 128);
      __builtin_prefetch(k + 192);
      __builtin_prefetch(k + 256);
    }
  }
  if (j + 1 < n) {
    PyObject* d = PyList_GET_ITEM(evs, j + 1);
    if (PyDict_CheckExact(d)) {
      Py_ssize_t pos = 0;
      PyObject *key, *v;
      Py_hash_t h;
      int c = 0;
      while (c++ < 16 && _PyDict_Next(d, &pos, &key, &v, &h)) __builtin_prefetch(v);
    }
  }
}

typedef struct {
  PyObject* const* lists;    /* the evidence lists (exact lists; their items are read in place) */
  const int64_t* base;       /* first row of each incident */
  Py_ssize_t i0, i1;         /* this worker's incidents */
  const WVocabs* V;
  uint32_t *flags, *vocab;
  double* err;
  PyObject** pend;           /* per row: the node name to number (borrowed) or NULL */
  uint64_t* phash;           /* per row with a node name: its characters' hash (0: not a str) */
  PyObject** ids5;           /* per incident: its first five rows' ids (borrowed; NULL = none) */
  uint8_t* redo;             /* per row: 1 = encode on the calling thread */
  Py_ssize_t* next;          /* the next unclaimed incident (shared by the call's jobs) */
} WJob;

/* Incidents per claim of the workers' shared cursor: rows differ in cost (a pod row reads a
 * dozen keys, an event row two), so a static split by row counts left threads idle behind the
 * slowest; claims of a few incidents balance them. */
#define W_CHUNK 8

static void* w_main(void* arg) {
  const WJob* J = (const WJob*)arg;
  for (;;) {
  const Py_ssize_t c0 = __atomic_fetch_add(J->next, (Py_ssize_t)W_CHUNK, __ATOMIC_RELAXED);
  if (c0 >= J->i1) break;
  const Py_ssize_t c1 = c0 + W_CHUNK < J->i1 ? c0 + W_CHUNK : J->i1;
  for (Py_ssize_t i = c0; i < c1; ++i) {
    PyObject* evs = J->lists[i];
    const Py_ssize_t n = PyList_GET_SIZE(evs);
    for (Py_ssize_t j = 0; j < n; ++j) {
      row_prefetch(evs, j, n);
      const Py_ssize_t r = J->base[i] + j;
      PyObject* ev = PyList_GET_ITEM(evs, j);
      Row row = {0, 0, NO_NODE, 0.0, NULL};
      int redo = w_row(ev, J->V, &row);
      if (!redo && j < 5 && w_get(ev, &k_id, 1, &J->ids5[5 * i + j])) redo = 1;
      J->redo[r] = (uint8_t)redo;
      J->flags[r] = row.flags;
      J->vocab[r] = row.vocab;
      J->err[r] = row.err;
      J->pend[r] = row.pending_node;
      J->phash[r] = (!redo && row.pending_node != NULL) ? w_str_hash(row.pending_node) : 0u;
    }
  }
  }
  return NULL;
}

/* A persistent pool of worker threads (created on first use, up to PAR_MAX_THREADS - 1; the
 * calling thread runs job 0): a call hands out its jobs and waits for them, instead of creating
 * and joining threads every time.  A job is `fn(jobs + i * job_size)`: the rules encoder's row
 * pass (w_main) and the seed attachment's (s_main) share the pool.  A forked child starts
 * without the parent's threads: the pool is rebuilt there on first use. */
#define PAR_MAX_THREADS 64
typedef void* (*JobFn)(void*);
static struct {
  pthread_mutex_t mu;
  pthread_cond_t go, done;
  int n;                          /* threads in the pool */
  unsigned long gen;              /* incremented per call */
  int pending;                    /* jobs not finished in this call */
  int njobs;
  JobFn fn;
  char* jobs;                     /* job i at jobs + i * job_size (pool threads run 1..njobs) */
  size_t job_size;
} pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0, 0, 0,
          NULL, NULL, 0};

typedef struct { int id; } PoolArg;
static PoolArg pool_args[PAR_MAX_THREADS];

static void* pool_main(void* arg) {
  const int id = ((PoolArg*)arg)->id;      /* runs job `id` of each call that has one */
  unsigned long seen = 0;
  pthread_mutex_lock(&pool.mu);
  for (;;) {
    while (pool.gen == seen) pthread_cond_wait(&pool.go, &pool.mu);
    seen = pool.gen;
    if (id < pool.njobs) {
      const JobFn fn = pool.fn;
      void* j = pool.jobs + (size_t)id * pool.job_size;
      pthread_mutex_unlock(&pool.mu);
      fn(j);
      pthread_mutex_lock(&pool.mu);
      if (--pool.pending == 0) pthread_cond_signal(&pool.done);
    }
  }
  return NULL;
}

static void pool_after_fork(void) {
  pthread_mutex_init(&pool.mu, NULL);
  pthread_cond_init(&pool.go, NULL);
  pthread_cond_init(&pool.done, NULL);
  pool.n = 0;
  pool.pending = 0;
}

/* run fn over jobs[0..n): jobs[1..) on the pool (grown as needed), jobs[0] here; returns when
 * all are done */
static void pool_run_fn(JobFn fn, void* jobs_v, size_t job_size, int n) {
  char* jobs = (char*)jobs_v;
  pthread_mutex_lock(&pool.mu);
  while (pool.n < n - 1) {
    pthread_t t;
    pool_args[pool.n + 1].id = pool.n + 1;
    if (pthread_create(&t, NULL, pool_main, &pool_args[pool.n + 1]) != 0) break;
    pthread_detach(t);
    ++pool.n;
  }
  const int m = pool.n + 1 < n ? pool.n + 1 : n;      /* jobs the pool can take */
  pool.fn = fn;
  pool.jobs = jobs;
  pool.job_size = job_size;
  pool.njobs = m;
  pool.pending = m - 1;
  ++pool.gen;
  pthread_cond_broadcast(&pool.go);
  pthread_mutex_unlock(&pool.mu);
  fn(jobs);
  for (int t = m; t < n; ++t) fn(jobs + (size_t)t * job_size);   /* jobs no thread could be created for */
  pthread_mutex_lock(&pool.mu);
  while (pool.pending > 0) pthread_cond_wait(&pool.done, &pool.mu);
  pool.njobs = 0;
  pthread_mutex_unlock(&pool.mu);
}

static void pool_run(WJob* jobs, int n) { pool_run_fn(w_main, jobs, sizeof(WJob), n); }

static int intern_worker_keys(void) {
  pthread_atfork(NULL, NULL, pool_after_fork);
  K_EV[0] = k_type; K_EV[1] = k_data;
  K_POD[0] = k_waiting; K_POD[1] = k_terminated; K_POD[2] = k_restart; K_POD[3] = k_node_name;
  K_POD[4] = k_conditions; K_POD[5] = k_phase;
  K_COND[0] = k_ctype;
  K_READY[0] = k_status; K_READY[1] = k_reason;
  K_LOG[0] = k_patterns; K_LOG[1] = k_error_count;
  K_METRIC[0] = k_query; K_METRIC[1] = k_anomalous; K_METRIC[2] = k_current;
  K_NODE[0] = k_name; K_NODE[1] = k_conditions;
  /* w_get compares entry hashes with these keys' cached hashes */
  PyObject* all[] = {k_type, k_data, k_waiting, k_terminated, k_restart, k_node_name, k_conditions,
                     k_phase, k_ctype, k_status, k_reason, k_patterns, k_error_count, k_query,
                     k_anomalous, k_current, k_name, k_ready_key, k_recent, k_image_changed};
  for (size_t i = 0; i < sizeof(all) / sizeof(all[0]); ++i)
    if (PyObject_Hash(all[i]) == -1) return -1;
  return 0;
}

/* encode_rows(evidence_lists, waiting, terminated, patterns, node_keys, slow_row,
 *             flags, vocab, node, err, seg_off[, threads]) -> (first-five-ids lists, rows handed over)
 * Output buffers are writable contiguous arrays sized by the caller (sum of len(evidence)).
 * threads > 1 and enough rows: the parallel row pass above, then the serial completion. */
#define PAR_MIN_ROWS 4096
static PyObject* encode_rows(PyObject* self, PyObject* args) {
  PyObject *lists, *slow_row;
  Vocab V;
  int threads = 1;
  Py_buffer bf = {0}, bv = {0}, bn = {0}, be = {0}, bs = {0};
  if (!PyArg_ParseTuple(args, "OO!O!O!O!Ow*w*w*w*w*|i", &lists, &PyDict_Type, &V.waiting,
                        &PyDict_Type, &V.terminated, &PyDict_Type, &V.patterns, &PyDict_Type,
                        &V.node_keys, &slow_row, &bf, &bv, &bn, &be, &bs, &threads))
    return NULL;
  PyObject* result = NULL;
  PyObject* seq = NULL;
  PyObject* ids = NULL;
  int64_t* base = NULL;
  PyObject** pend = NULL;
  uint64_t* phash = NULL;
  NodeMap nm = {NULL, NULL, NULL, NULL, 0, 0};
  int use_map = 0;                  /* node numbering in the C map (until the dict takes over) */
  PyObject** ids5 = NULL;
  uint8_t* redo = NULL;
  WVocabs WV = {{NULL, 0}, {NULL, 0}, {NULL, 0}};
  Py_ssize_t n_slow = 0;
  uint32_t* flags = (uint32_t*)bf.buf;
  uint32_t* vocab = (uint32_t*)bv.buf;
  uint32_t* node = (uint32_t*)bn.buf;
  double* err = (double*)be.buf;
  int64_t* seg = (int64_t*)bs.buf;
  Py_ssize_t cap = bf.len / 4;
  if (bv.len / 4 < cap || bn.len / 4 < cap || be.len / 8 < cap) {
    PyErr_SetString(PyExc_ValueError, "encode_rows: column buffers differ in size");
    goto done;
  }
  seq = PySequence_Fast(lists, "evidence_lists must be a sequence");
  if (!seq) goto done;
  Py_ssize_t B = PySequence_Fast_GET_SIZE(seq);
  if (bs.len / 8 < B + 1) {
    PyErr_SetString(PyExc_ValueError, "encode_rows: seg_off too small");
    goto done;
  }
  ids = PyList_New(B);
  if (!ids) goto done;
  /* the parallel pass: every evidence list an exact list, enough rows, the vocab tables flat */
  int par = threads > 1;
  Py_ssize_t total = 0;
  for (Py_ssize_t i = 0; par && i < B; ++i) {
    PyObject* evs = PySequence_Fast_GET_ITEM(seq, i);
    if (!PyList_CheckExact(evs)) par = 0;
    else total += PyList_GET_SIZE(evs);
  }
  if (par && (total < PAR_MIN_ROWS || total > cap)) par = 0;
  if (par && (wvocab_build(V.waiting, &WV.waiting) || wvocab_build(V.terminated, &WV.terminated) ||
              wvocab_build(V.patterns, &WV.patterns))) {
    if (PyErr_Occurred()) goto done;             /* (allocation failure) */
    par = 0;
  }
  if (par) {
    base = PyMem_Malloc(sizeof(int64_t) * (size_t)(B + 1));
    pend = PyMem_Malloc(sizeof(PyObject*) * (size_t)total);
    phash = PyMem_Malloc(sizeof(uint64_t) * (size_t)total);
    if (!phash) { PyErr_NoMemory(); goto done; }
    ids5 = PyMem_Calloc((size_t)B * 5, sizeof(PyObject*));
    redo = PyMem_Malloc((size_t)total);
    if (!base || !pend || !ids5 || !redo) { PyErr_NoMemory(); goto done; }
    base[0] = 0;
    for (Py_ssize_t i = 0; i < B; ++i) base[i + 1] = base[i] + PyList_GET_SIZE(PySequence_Fast_GET_ITEM(seq, i));
    if (threads > PAR_MAX_THREADS) threads = PAR_MAX_THREADS;
    WJob jobs[PAR_MAX_THREADS];
    /* every job claims W_CHUNK incidents at a time from one cursor, up to B */
    Py_ssize_t next = 0;
    for (int t = 0; t < threads; ++t)
      jobs[t] = (WJob){PySequence_Fast_ITEMS(seq), base, 0, B, &WV, flags, vocab, err, pend, phash,
                       ids5, redo, &next};
    /* (the GIL stays held: no Python code runs while the workers read) */
    pool_run(jobs, threads);
    /* node names are numbered in a C map keyed by the workers' content hashes while no Python
     * code runs and node_keys starts empty (encode_batch's fresh dict) */
    if (PyDict_GET_SIZE(V.node_keys) == 0) {
      size_t np = 0;
      int fast = 1;                  /* no row for the serial encoder, every node name a str */
      for (Py_ssize_t q = 0; q < total; ++q) {
        np += pend[q] != NULL && !redo[q];
        fast &= !redo[q] && (pend[q] == NULL || phash[q] != 0);
      }
      if (nodemap_init(&nm, np) < 0) goto done;
      use_map = 1;
      if (fast) {
        /* the completion without the serial loop: the workers wrote every row's flags / vocab /
         * err; what is left is the node numbering (first-seen order, the C map), the segment
         * offsets and each incident's first five evidence ids -- the serial pass's results for
         * rows it would only have copied */
        for (Py_ssize_t q = 0; q < total; ++q)
          node[q] = pend[q] != NULL ? nodemap_get(&nm, phash[q], pend[q]) : NO_NODE;
        seg[0] = 0;
        for (Py_ssize_t i = 0; i < B; ++i) {
          const Py_ssize_t n = base[i + 1] - base[i], m = n < 5 ? n : 5;
          PyObject* first = PyList_New(m);
          if (!first) goto done;
          for (Py_ssize_t j = 0; j < m; ++j) {
            PyObject* id = ids5[5 * i + j] != NULL ? ids5[5 * i + j] : Py_None;
            Py_INCREF(id);
            PyList_SET_ITEM(first, j, id);
          }
          PyList_SET_ITEM(ids, i, first);
          seg[i + 1] = base[i + 1];
        }
        /* (node_keys is left empty: no row went through Python, so nothing read the numbering
         * from it, and encode_batch drops it -- copying the C map out was a third of this path) */
        result = Py_BuildValue("(On)", ids, (Py_ssize_t)0);
        goto done;
      }
    }
  }
  /* serial pass (or the completion of the parallel one), in row order */
  Py_ssize_t r = 0;
  int python_ran = 0;                 /* a slow row ran Python: re-read later rows serially */
  seg[0] = 0;
  for (Py_ssize_t i = 0; i < B; ++i) {
    PyObject* evs = PySequence_Fast(PySequence_Fast_GET_ITEM(seq, i), "evidence is not iterable");
    if (!evs) goto done;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(evs);
    PyObject* first = PyList_New(0);
    if (!first) { Py_DECREF(evs); goto done; }
    PyList_SET_ITEM(ids, i, first);
    for (Py_ssize_t j = 0; j < n; ++j) {
      if (r >= cap) {
        PyErr_SetString(PyExc_ValueError, "encode_rows: more rows than the buffers hold");
        Py_DECREF(evs);
        goto done;
      }
      const int want_id = PyList_GET_SIZE(first) < 5;
      Row row;
      PyObject* ev_id = NULL;
      PyObject* slow_res = NULL;
      /* the worker's encoding, unless Python has run since the pass (it could have changed the
       * evidence: from then on every row is encoded here again) */
      if (par && !python_ran && !redo[r]) {
        row.flags = flags[r];
        row.vocab = vocab[r];
        row.node = NO_NODE;
        row.err = err[r];
        row.pending_node = pend[r];
        if (want_id) ev_id = ids5[5 * i + j];
        if (use_map && row.pending_node != NULL) {
          if (phash[r] != 0) {
            row.node = nodemap_get(&nm, phash[r], row.pending_node);
            row.pending_node = NULL;
          } else {                       /* a name that is not a str: the dict takes over */
            if (nodemap_materialize(&nm, V.node_keys) < 0) { Py_DECREF(evs); goto done; }
            use_map = 0;
          }
        }
      } else {
        if (use_map) {                   /* the serial encoder numbers through the dict */
          if (nodemap_materialize(&nm, V.node_keys) < 0) { Py_DECREF(evs); goto done; }
          use_map = 0;
        }
        const Py_ssize_t before = n_slow;
        if (encode_row_serial(PySequence_Fast_GET_ITEM(evs, j), &V, slow_row, want_id, &row,
                              &ev_id, &slow_res, &n_slow) < 0) {
          Py_DECREF(evs);
          goto done;
        }
        if (n_slow != before) python_ran = 1;
      }
      if (resolve_node(&V, &row) < 0) {
        Py_XDECREF(slow_res);
        Py_DECREF(evs);
        goto done;
      }
      flags[r] = row.flags;
      vocab[r] = row.vocab;
      node[r] = row.node;
      err[r] = row.err;
      if (want_id && PyList_Append(first, ev_id == NULL ? Py_None : ev_id) < 0) {
        Py_XDECREF(slow_res);
        Py_DECREF(evs);
        goto done;
      }
      Py_XDECREF(slow_res);
      ++r;
    }
    Py_DECREF(evs);
    seg[i + 1] = r;
  }
  if (use_map && nodemap_materialize(&nm, V.node_keys) < 0) goto done;   /* node_keys as the
                                                                            serial pass fills it */
  result = Py_BuildValue("(On)", ids, n_slow);
done:
  Py_XDECREF(ids);
  Py_XDECREF(seq);
  PyMem_Free(base);
  PyMem_Free(pend);
  PyMem_Free(phash);
  nodemap_free(&nm);
  PyMem_Free(ids5);
  PyMem_Free(redo);
  PyMem_Free(WV.waiting.e);
  PyMem_Free(WV.terminated.e);
  PyMem_Free(WV.patterns.e);
  PyBuffer_Release(&bf); PyBuffer_Release(&bv); PyBuffer_Release(&bn);
  PyBuffer_Release(&be); PyBuffer_Release(&bs);
  return result;
}

/* ---- hypothesis dicts --------------------------------------------------------------------- */

static PyObject* uuid4_str(const unsigned char* raw) {
  /* uuid.UUID(bytes=raw, version=4): version nibble 4, RFC 4122 variant */
  unsigned char b[16];
  memcpy(b, raw, 16);
  b[6] = (unsigned char)((b[6] & 0x0F) | 0x40);
  b[8] = (unsigned char)((b[8] & 0x3F) | 0x80);
  static const char hx[] = "0123456789abcdef";
  char s[36];
  int p = 0;
  for (int i = 0; i < 16; ++i) {
    if (i == 4 || i == 6 || i == 8 || i == 10) s[p++] = '-';
    s[p++] = hx[b[i] >> 4];
    s[p++] = hx[b[i] & 15];
  }
  return PyUnicode_FromStringAndSize(s, 36);
}

static int set_steal(PyObject* d, PyObject* k, PyObject* v) {
  if (!v) return -1;
  int rc = PyDict_SetItem(d, k, v);
  Py_DECREF(v);
  return rc;
}

/* assemble(templates, unknown, n_hyp, order, confidence, final_score, strength, incident_ids,
 *          evidence_ids, ranked, random_bytes) -> list of hypothesis lists
 * templates: per rule slot a tuple (category, title, description, actions list, rule_id,
 *            support_count); unknown: (category, title, description, confidence, rank,
 *            actions list, generated_by, rule_id, support_count, signal_strength).
 * order is u8 [B, S], the three f64 arrays [B, S]; random_bytes holds 16 B per hypothesis. */
static PyObject* assemble(PyObject* self, PyObject* args) {
  PyObject *templates, *unknown, *inc_ids, *ev_ids;
  Py_buffer bn = {0}, bo = {0}, bc = {0}, bfs = {0}, bst = {0}, brnd = {0};
  int ranked;
  if (!PyArg_ParseTuple(args, "O!O!y*y*y*y*y*O!O!py*", &PyTuple_Type, &templates, &PyTuple_Type,
                        &unknown, &bn, &bo, &bc, &bfs, &bst, &PyList_Type, &inc_ids,
                        &PyList_Type, &ev_ids, &ranked, &brnd))
    return NULL;
  PyObject* out = NULL;
  PyObject* gen_by = NULL;
  PyObject** tmpl = NULL;
  Py_ssize_t R = PyTuple_GET_SIZE(templates), S = R + 1;
  Py_ssize_t B = PyList_GET_SIZE(inc_ids);
  const uint8_t* n_hyp = (const uint8_t*)bn.buf;
  const uint8_t* order = (const uint8_t*)bo.buf;
  const double* conf = (const double*)bc.buf;
  const double* fscore = (const double*)bfs.buf;
  const double* strength = (const double*)bst.buf;
  const unsigned char* rnd = (const unsigned char*)brnd.buf;
  Py_ssize_t n_rnd = brnd.len / 16, used = 0;
  if (PyList_GET_SIZE(ev_ids) != B || bn.len < B || bo.len < B * S ||
      bc.len < (Py_ssize_t)(B * S * 8) || bfs.len < (Py_ssize_t)(B * S * 8) ||
      bst.len < (Py_ssize_t)(B * S * 8) || PyTuple_GET_SIZE(unknown) != 10) {
    PyErr_SetString(PyExc_ValueError, "assemble: inconsistent sizes");
    goto done;
  }
  for (Py_ssize_t s = 0; s < R; ++s) {
    PyObject* t = PyTuple_GET_ITEM(templates, s);
    if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) != 6 || !PyList_Check(PyTuple_GET_ITEM(t, 3))) {
      PyErr_SetString(PyExc_ValueError, "assemble: bad rule template");
      goto done;
    }
  }
  if (!PyList_Check(PyTuple_GET_ITEM(unknown, 5))) {
    PyErr_SetString(PyExc_ValueError, "assemble: bad unknown template");
    goto done;
  }
  gen_by = PyUnicode_InternFromString("rules_engine");
  if (!gen_by) goto done;
  /* One template dict per slot with every key in the reference's order and the values shared
   * by all of that slot's hypotheses; each hypothesis is a copy of it (a combined-table dict
   * copy: one allocation, no per-key insertion or resize) with its own values then put in
   * place -- the keys keep their positions, so the dict is the one built key by key. */
  tmpl = PyMem_Calloc((size_t)S, sizeof(PyObject*));
  if (!tmpl) { PyErr_NoMemory(); goto done; }
  for (Py_ssize_t slot = 0; slot < S; ++slot) {
    PyObject* h = tmpl[slot] = _PyDict_NewPresized(14);
    if (!h) goto done;
    int bad;
    if (slot == R) {
      PyObject* u = unknown;
      bad = PyDict_SetItem(h, h_id, Py_None) < 0 || PyDict_SetItem(h, h_incident, Py_None) < 0 ||
            PyDict_SetItem(h, h_category, PyTuple_GET_ITEM(u, 0)) < 0 ||
            PyDict_SetItem(h, h_title, PyTuple_GET_ITEM(u, 1)) < 0 ||
            PyDict_SetItem(h, h_description, PyTuple_GET_ITEM(u, 2)) < 0 ||
            PyDict_SetItem(h, h_confidence, PyTuple_GET_ITEM(u, 3)) < 0 ||
            PyDict_SetItem(h, h_rank, PyTuple_GET_ITEM(u, 4)) < 0 ||
            PyDict_SetItem(h, h_support_ids, Py_None) < 0 ||
            PyDict_SetItem(h, h_actions, Py_None) < 0 ||
            PyDict_SetItem(h, h_generated_by, PyTuple_GET_ITEM(u, 6)) < 0 ||
            PyDict_SetItem(h, h_rule_id, PyTuple_GET_ITEM(u, 7)) < 0 ||
            PyDict_SetItem(h, h_support_count, PyTuple_GET_ITEM(u, 8)) < 0 ||
            PyDict_SetItem(h, h_strength, PyTuple_GET_ITEM(u, 9)) < 0;
    } else {
      PyObject* t = PyTuple_GET_ITEM(templates, slot);
      bad = PyDict_SetItem(h, h_id, Py_None) < 0 || PyDict_SetItem(h, h_incident, Py_None) < 0 ||
            PyDict_SetItem(h, h_category, PyTuple_GET_ITEM(t, 0)) < 0 ||
            PyDict_SetItem(h, h_title, PyTuple_GET_ITEM(t, 1)) < 0 ||
            PyDict_SetItem(h, h_description, PyTuple_GET_ITEM(t, 2)) < 0 ||
            PyDict_SetItem(h, h_confidence, Py_None) < 0 ||
            PyDict_SetItem(h, h_rank, i_zero) < 0 ||
            PyDict_SetItem(h, h_support_ids, Py_None) < 0 ||
            PyDict_SetItem(h, h_actions, Py_None) < 0 ||
            PyDict_SetItem(h, h_generated_by, gen_by) < 0 ||
            PyDict_SetItem(h, h_rule_id, PyTuple_GET_ITEM(t, 4)) < 0 ||
            PyDict_SetItem(h, h_support_count, PyTuple_GET_ITEM(t, 5)) < 0 ||
            PyDict_SetItem(h, h_strength, Py_None) < 0;
    }
    if (bad || (ranked && PyDict_SetItem(h, h_final, Py_None) < 0)) goto done;
  }
  out = PyList_New(B);
  if (!out) goto done;
  for (Py_ssize_t i = 0; i < B; ++i) {
    int nh = n_hyp[i];
    PyObject* lst = PyList_New(nh);
    if (!lst) goto fail;
    PyList_SET_ITEM(out, i, lst);
    PyObject* iid = PyList_GET_ITEM(inc_ids, i);
    PyObject* eids = PyList_GET_ITEM(ev_ids, i);
    if (!PyList_Check(eids)) {
      PyErr_SetString(PyExc_TypeError, "assemble: evidence ids must be lists");
      goto fail;
    }
    for (int p = 0; p < nh; ++p) {
      int slot = order[i * S + p];
      if (slot > R || used >= n_rnd) {
        PyErr_SetString(PyExc_ValueError, "assemble: slot out of range or random bytes short");
        goto fail;
      }
      PyObject* h = PyDict_Copy(tmpl[slot]);
      if (!h) goto fail;
      PyList_SET_ITEM(lst, p, h);
      if (set_steal(h, h_id, uuid4_str(rnd + 16 * used++)) < 0) goto fail;
      if (PyDict_SetItem(h, h_incident, iid) < 0) goto fail;
      if (set_steal(h, h_support_ids, PyList_GetSlice(eids, 0, PY_SSIZE_T_MAX)) < 0) goto fail;
      if (slot == R) {                          /* _create_unknown_hypothesis (:457-478) */
        if (set_steal(h, h_actions, PyList_GetSlice(PyTuple_GET_ITEM(unknown, 5), 0, PY_SSIZE_T_MAX)) < 0)
          goto fail;
      } else {                                  /* _create_hypothesis (:235-262) */
        PyObject* t = PyTuple_GET_ITEM(templates, slot);
        if (set_steal(h, h_confidence, PyFloat_FromDouble(conf[i * S + slot])) < 0 ||
            set_steal(h, h_actions, PyList_GetSlice(PyTuple_GET_ITEM(t, 3), 0, PY_SSIZE_T_MAX)) < 0 ||
            set_steal(h, h_strength, PyFloat_FromDouble(strength[i * S + slot])) < 0)
          goto fail;
      }
      if (ranked) {                             /* HypothesisRanker.rank (:63-71) */
        if (set_steal(h, h_final, PyFloat_FromDouble(fscore[i * S + slot])) < 0 ||
            set_steal(h, h_rank, PyLong_FromLong(p + 1)) < 0)
          goto fail;
      }
    }
  }
  goto done;
fail:
  Py_CLEAR(out);
done:
  if (tmpl)
    for (Py_ssize_t slot = 0; slot < S; ++slot) Py_XDECREF(tmpl[slot]);
  PyMem_Free(tmpl);
  Py_XDECREF(gen_by);
  PyBuffer_Release(&bn); PyBuffer_Release(&bo); PyBuffer_Release(&bc);
  PyBuffer_Release(&bfs); PyBuffer_Release(&bst); PyBuffer_Release(&brnd);
  return out;
}

static PyObject* flag_bits(PyObject* self, PyObject* noargs) {
  return Py_BuildValue("(IIIIIIIIII)", F_RECENT_DEPLOY, F_IMAGE_CHANGED, F_MEMORY_HIGH,
                       F_HPA_AT_MAX, F_LATENCY_HIGH, F_NODE_ISSUE, F_NOT_READY, F_READINESS_FAIL,
                       F_ERR_FLOAT, NO_NODE);
}

/* ---- propagation seeds: attachment candidates of evidence rows (egraph/seeds.py) ----------- */

static PyObject *a_ns, *a_name, *a_strength, *a_involved, *a_kind, *a_namespace, *a_half,
    *t_pod, *t_deploy, *t_dchange, *t_ichange, *t_node, *t_hpa, *t_config, *t_event, *t_log,
    *t_metric, *s_empty, *s_node_lc, *s_colon, *p_pod, *p_deploy, *p_node, *p_hpa, *p_config,
    *p_logpattern, *p_service, *p_metric, *p_event, *kind_cache;

static PyObject* K_SEED[5];    /* evidence_type, entity_namespace, entity_name, data, signal_strength */
static PyObject* K_INV[1];     /* involved_object */
static PyObject* K_OBJ[3];     /* kind, name, namespace */

static int intern_seeds(void) {
#define S(var, text) if (!(var = PyUnicode_InternFromString(text))) return -1
  S(a_ns, "entity_namespace"); S(a_name, "entity_name"); S(a_strength, "signal_strength");
  S(a_involved, "involved_object"); S(a_kind, "kind"); S(a_namespace, "namespace");
  S(t_pod, "kubernetes_pod"); S(t_deploy, "kubernetes_deployment"); S(t_dchange, "deploy_change");
  S(t_ichange, "image_change"); S(t_node, "kubernetes_node"); S(t_hpa, "kubernetes_hpa");
  S(t_config, "config_change"); S(t_event, "kubernetes_event"); S(t_log, "log_signal");
  S(t_metric, "metric_signal"); S(s_empty, ""); S(s_node_lc, "node"); S(s_colon, ":");
  S(p_pod, "pod:"); S(p_deploy, "deployment:"); S(p_node, "node:"); S(p_hpa, "hpa:");
  S(p_config, "configmap:"); S(p_logpattern, "logpattern:"); S(p_service, "service:");
  S(p_metric, "metric:"); S(p_event, "event:");
#undef S
  if (!(kind_cache = PyDict_New())) return -1;
  if (!(a_half = PyFloat_FromDouble(0.5))) return -1;
  K_SEED[0] = k_type; K_SEED[1] = a_ns; K_SEED[2] = a_name; K_SEED[3] = k_data; K_SEED[4] = a_strength;
  K_INV[0] = a_involved;
  K_OBJ[0] = a_kind; K_OBJ[1] = k_name; K_OBJ[2] = a_namespace;
  PyObject* hk[] = {k_type, a_ns, a_name, k_data, a_strength, a_involved, a_kind, k_name, a_namespace,
                    t_pod, t_deploy, t_dchange, t_ichange, t_node, t_hpa, t_config, t_event, t_log, t_metric};
  for (size_t i = 0; i < sizeof(hk) / sizeof(hk[0]); ++i)   /* w_get reads the cached hashes */
    if (PyObject_Hash(hk[i]) == -1) return -1;
  return 0;
}

/* values an f-string / str() formats without running user code: format(x, '') == str(x) */
static inline int fmt_plain(PyObject* o) {
  return o == Py_None || PyUnicode_CheckExact(o) || PyLong_CheckExact(o) || PyBool_Check(o) ||
         PyFloat_CheckExact(o);
}

/* str(x) of a plain value (new reference) */
static inline PyObject* as_str(PyObject* o) {
  if (PyUnicode_CheckExact(o)) {
    Py_INCREF(o);
    return o;
  }
  return PyObject_Str(o);
}

/* append the id prefix + str(a) [+ ":" + str(b)] (f"{prefix}{a}:{b}"), built in one allocation;
 * -1 on error */
static int push_id(PyObject* ids, PyObject* prefix, PyObject* a, PyObject* b) {
  PyObject* part[4] = {prefix, as_str(a), b ? s_colon : NULL, b ? as_str(b) : NULL};
  const int np = b ? 4 : 2;
  int rc = -1;
  PyObject* out = NULL;
  Py_ssize_t len = 0;
  Py_UCS4 maxc = 127;
  for (int i = 0; i < np; ++i) {
    if (!part[i]) goto done;
    len += PyUnicode_GET_LENGTH(part[i]);
    const Py_UCS4 m = PyUnicode_MAX_CHAR_VALUE(part[i]);
    if (m > maxc) maxc = m;
  }
  out = PyUnicode_New(len, maxc);
  if (!out) goto done;
  {
    Py_ssize_t at = 0;
    for (int i = 0; i < np; ++i) {
      const Py_ssize_t n = PyUnicode_GET_LENGTH(part[i]);
      if (PyUnicode_CopyCharacters(out, at, part[i], 0, n) < 0) goto done;
      at += n;
    }
  }
  rc = PyList_Append(ids, out);
done:
  Py_XDECREF(out);
  Py_XDECREF(part[1]);
  Py_XDECREF(part[3]);
  return rc;
}

/* attach_ids(ev) of egraph/seeds.py for an exact dict: 1 = done (ids filled), 0 = hand over to
 * the Python statement, -1 = error */
static int cand_ids(PyObject* ev, PyObject* ids) {
  PyObject *t, *ns, *name, *data;
  if (dget(ev, k_type, &t) || dget(ev, a_ns, &ns) || dget(ev, a_name, &name) || dget(ev, k_data, &data))
    return 0;
  if (t != NULL && t != Py_None && !PyUnicode_CheckExact(t)) return 0;   /* == may run user code */
  if (!ns) ns = Py_None;
  if (!name) name = Py_None;
  if (!fmt_plain(ns) || !fmt_plain(name)) return 0;
  if (data != NULL && data != Py_None && !PyDict_CheckExact(data)) return 0;   /* `or {}` */
  if (t == NULL || t == Py_None) return 1;
  if (eq_str(t, t_pod)) return push_id(ids, p_pod, ns, name) < 0 ? -1 : 1;
  if (eq_str(t, t_deploy) || eq_str(t, t_dchange) || eq_str(t, t_ichange))
    return push_id(ids, p_deploy, ns, name) < 0 ? -1 : 1;
  if (eq_str(t, t_node)) return push_id(ids, p_node, name, NULL) < 0 ? -1 : 1;
  if (eq_str(t, t_hpa)) return push_id(ids, p_hpa, ns, name) < 0 ? -1 : 1;
  if (eq_str(t, t_config)) return push_id(ids, p_config, ns, name) < 0 ? -1 : 1;
  if (eq_str(t, t_log)) {
    if (push_id(ids, p_logpattern, ns, name) < 0 || push_id(ids, p_service, ns, name) < 0 ||
        push_id(ids, p_deploy, ns, name) < 0)
      return -1;
    return 1;
  }
  if (eq_str(t, t_metric)) return push_id(ids, p_metric, ns, name) < 0 ? -1 : 1;
  if (eq_str(t, t_event)) {
    PyObject *obj = NULL, *kind = NULL, *oname = NULL, *ons = NULL;
    if (data != NULL && data != Py_None && PyDict_GET_SIZE(data) > 0) {
      if (dget(data, a_involved, &obj)) return 0;
    }
    if (obj != NULL && obj != Py_None && !PyDict_CheckExact(obj)) return 0;
    if (obj != NULL && (obj == Py_None || PyDict_GET_SIZE(obj) == 0)) obj = NULL;
    if (obj != NULL) {
      if (dget(obj, a_kind, &kind) || dget(obj, k_name, &oname) || dget(obj, a_namespace, &ons))
        return 0;
      if ((kind && !fmt_plain(kind)) || (oname && !fmt_plain(oname)) || (ons && !fmt_plain(ons)))
        return 0;
    }
    if (push_id(ids, p_event, ns, name) < 0) return -1;
    /* kind = str(obj.get("kind", "")).lower(); the id prefix "<kind>:" is cached per str(kind)
     * (kind_cache: str(kind) -> kind.lower() + ":") */
    PyObject* ks = kind ? as_str(kind) : (Py_INCREF(s_empty), s_empty);
    if (!ks) return -1;
    PyObject* kc = PyDict_GetItemWithError(kind_cache, ks);   /* borrowed; exact str keys */
    if (!kc) {
      if (PyErr_Occurred()) { Py_DECREF(ks); return -1; }
      PyObject* kl = PyObject_CallMethod(ks, "lower", NULL);
      if (!kl) { Py_DECREF(ks); return -1; }
      kc = PyUnicode_Concat(kl, s_colon);
      Py_DECREF(kl);
      if (PyDict_GET_SIZE(kind_cache) >= 4096) PyDict_Clear(kind_cache);   /* bounded */
      if (!kc || PyDict_SetItem(kind_cache, ks, kc) < 0) { Py_XDECREF(kc); Py_DECREF(ks); return -1; }
      Py_DECREF(kc);                                   /* the cache holds it */
    }
    Py_DECREF(ks);
    if (PyUnicode_Compare(kc, p_node) == 0)            /* kind == "node" */
      return push_id(ids, p_node, oname ? oname : Py_None, NULL) < 0 ? -1 : 1;
    if (PyUnicode_GET_LENGTH(kc) > 1)                  /* kind != "": f"{kind}:{ns}:{name}" */
      return push_id(ids, kc, ons ? ons : ns, oname ? oname : Py_None) < 0 ? -1 : 1;
    return 1;
  }
  return 1;   /* any other type: no candidate */
}

/* seed_candidates(evidence_lists, slow) -> (flat ids, per-row counts (int64 bytes), columns
 * (uint32 bytes), strengths (float64 bytes)):
 * SeedCandidates.__init__ of egraph/seeds.py.  `slow(ev)` is the Python statement of one row
 * (attach_ids + the strength), used for rows whose values are not plain. */
static PyObject* seed_candidates(PyObject* self, PyObject* args) {
  PyObject *lists, *slow;
  if (!PyArg_ParseTuple(args, "OO", &lists, &slow)) return NULL;
  PyObject* seq = PySequence_Fast(lists, "evidence_lists must be a sequence");
  if (!seq) return NULL;
  PyObject* flat = PyList_New(0);
  PyObject* result = NULL;
  int64_t* cnt = NULL;      /* per seeding row: candidate count, column, strength */
  uint32_t* col = NULL;
  double* val = NULL;
  Py_ssize_t nrow = 0, cap = 0;
  if (!flat) goto done;
  const Py_ssize_t B = PySequence_Fast_GET_SIZE(seq);
  for (Py_ssize_t b = 0; b < B; ++b) {
    PyObject* evs = PySequence_Fast(PySequence_Fast_GET_ITEM(seq, b), "evidence is not iterable");
    if (!evs) goto done;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(evs);
    for (Py_ssize_t j = 0; j < n; ++j) {
      PyObject* ev = PySequence_Fast_GET_ITEM(evs, j);
      PyObject* ids = PyList_New(0);
      if (!ids) { Py_DECREF(evs); goto done; }
      double sv = 0.0;
      int fast = 0;
      if (PyDict_CheckExact(ev)) {
        PyObject* st;
        fast = cand_ids(ev, ids);
        if (fast == 1) {
          if (dget(ev, a_strength, &st)) fast = 0;
          else if (st == NULL) sv = 0.5;
          else if (PyFloat_CheckExact(st)) sv = PyFloat_AS_DOUBLE(st);
          else if (PyLong_CheckExact(st) || PyBool_Check(st)) {
            sv = PyLong_AsDouble(st);
            if (sv == -1.0 && PyErr_Occurred()) { PyErr_Clear(); fast = 0; }
          } else fast = 0;
        }
      }
      if (fast < 0) { Py_DECREF(ids); Py_DECREF(evs); goto done; }
      if (!fast) {                                   /* the Python statement decides (or raises) */
        Py_DECREF(ids);
        PyObject* r = PyObject_CallOneArg(slow, ev);
        if (!r) { Py_DECREF(evs); goto done; }
        if (!PyArg_ParseTuple(r, "Od", &ids, &sv) || !PyList_Check(ids)) {
          if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "seed_candidates: bad slow row");
          Py_DECREF(r);
          Py_DECREF(evs);
          goto done;
        }
        Py_INCREF(ids);
        Py_DECREF(r);
      }
      const Py_ssize_t k = PyList_GET_SIZE(ids);
      if (k > 0 && !(sv <= 0.0)) {                   /* `if not ids or s <= 0: continue` (NaN kept) */
        int bad = 0;
        for (Py_ssize_t i = 0; i < k && !bad; ++i) bad = PyList_Append(flat, PyList_GET_ITEM(ids, i)) < 0;
        if (!bad && nrow == cap) {
          cap = cap ? 2 * cap : 256;
          int64_t* c2 = PyMem_Realloc(cnt, cap * sizeof(int64_t));
          if (c2) cnt = c2;
          uint32_t* o2 = PyMem_Realloc(col, cap * sizeof(uint32_t));
          if (o2) col = o2;
          double* v2 = PyMem_Realloc(val, cap * sizeof(double));
          if (v2) val = v2;
          if (!c2 || !o2 || !v2) { PyErr_NoMemory(); bad = 1; }
        }
        if (bad) { Py_DECREF(ids); Py_DECREF(evs); goto done; }
        cnt[nrow] = k;
        col[nrow] = (uint32_t)b;
        val[nrow] = sv;
        ++nrow;
      }
      Py_DECREF(ids);
    }
    Py_DECREF(evs);
  }
  result = Py_BuildValue("(Oy#y#y#)", flat, (const char*)cnt, nrow * (Py_ssize_t)sizeof(int64_t),
                         (const char*)col, nrow * (Py_ssize_t)sizeof(uint32_t), (const char*)val,
                         nrow * (Py_ssize_t)sizeof(double));
done:
  Py_XDECREF(flat);
  PyMem_Free(cnt);
  PyMem_Free(col);
  PyMem_Free(val);
  Py_DECREF(seq);
  return result;
}

/* ---- seed attachment in one native pass (egraph/seeds.py seeds_for_batch) ------------------
 * seed_attach(evidence_lists, slow, find, graph[, threads]) -> (vertex u32, column u32,
 * strength f32) bytes: SeedCandidates(evidence_lists).attach(graph) without building a Python
 * str per candidate id.  Each row's candidate ids (seeds.attach_ids) are formatted as UTF-8 into
 * a scratch buffer and resolved by `find` (the address of libegraph's egr_graph_find, `graph` its
 * egr_graph*): the first id present wins; rows with no id present, no candidate or a strength
 * <= 0 seed nothing.
 * Large batches run the row pass on the worker pool while the calling thread keeps the GIL (as
 * encode_rows does): the workers take a row only when every value it reads is an exact dict /
 * ASCII str / None / bool / float / int (no user code, nothing raises) and hand every other row
 * back; the calling thread redoes those in row order through the serial path (cand_ids, or the
 * Python statement `slow` = seeds._row, which raises what the reference expression raises), and
 * once Python has run it redoes every later row too.  The graph must not change during the call
 * (GraphService holds its lock). */
/* egr_graph_find's exact type (include/egraph.h), so the call through the pointer handed over
 * from ctypes is a call of the function's own type (UBSan -fsanitize=function checks it) */
struct egr_graph;
typedef const struct egr_graph* GraphP;
typedef int32_t (*FindFn)(GraphP g, const char* id, int64_t len);


typedef struct {
  char b[448];
  size_t n;
  int ovf;
} IdBuf;

static inline void ib_put(IdBuf* B, const char* p, size_t n) {
  if (B->n + n > sizeof(B->b)) { B->ovf = 1; return; }
  memcpy(B->b + B->n, p, n);
  B->n += n;
}

/* str(o) as bytes for the values a worker formats: an ASCII exact str, None (also a missing
 * key), True / False.  -1: the serial path formats it. */
static inline int w_part(PyObject* o, const char** p, Py_ssize_t* n) {
  if (o == NULL || o == Py_None) { *p = "None"; *n = 4; return 0; }
  if (PyUnicode_CheckExact(o)) {
    if (!PyUnicode_IS_READY(o) || !PyUnicode_IS_ASCII(o)) return -1;
    *p = (const char*)PyUnicode_1BYTE_DATA(o);
    *n = PyUnicode_GET_LENGTH(o);
    return 0;
  }
  if (o == Py_True) { *p = "True"; *n = 4; return 0; }
  if (o == Py_False) { *p = "False"; *n = 5; return 0; }
  return -1;
}

enum { ST_POD, ST_DEPLOY, ST_DCHANGE, ST_ICHANGE, ST_NODE, ST_HPA, ST_CONFIG, ST_EVENT, ST_LOG,
       ST_METRIC, ST_N };
static PyObject** seed_types[ST_N] = {&t_pod, &t_deploy, &t_dchange, &t_ichange, &t_node, &t_hpa,
                                      &t_config, &t_event, &t_log, &t_metric};

/* Where a row's candidate ids go, in order: the attachment (`find` each until one is present)
 * or the key list (every id appended to a byte buffer).  put: 1 = stop (found), 0 = go on,
 * -1 = cannot (hand the row over). */
typedef struct IdSink {
  int (*put)(struct IdSink*, const char* p, size_t n);
  FindFn find;                  /* attach */
  GraphP g;
  int32_t v;
  char* buf;                    /* keys: malloc'd (worker threads hold no GIL-side allocator) */
  size_t n, cap;
  int nid;                      /* ids appended for the current row */
  int64_t* idoff;               /* keys: per id its first byte in buf, and its id_hash64 */
  int64_t* idhash;
  size_t nids, capids;
} IdSink;

static inline uint64_t id_hash64(const char* p, size_t n);

static int sink_find(IdSink* k, const char* p, size_t n) {
  k->v = k->find(k->g, p, (int64_t)n);
  return k->v >= 0;
}

/* keys: the id's bytes appended to buf, its start offset and hash to the id arrays (an id ends
 * where the next one starts, or at n) -- the final blob / offsets / hashes format, so a batch
 * whose rows all stayed on the workers is assembled by copying each job's arrays */
static int sink_keys(IdSink* k, const char* p, size_t n) {
  if (k->n + n > k->cap) {
    size_t c = k->cap ? 2 * k->cap : 1 << 16;
    while (c < k->n + n) c *= 2;
    char* b = realloc(k->buf, c);
    if (!b) return -1;
    k->buf = b;
    k->cap = c;
  }
  if (k->nids == k->capids) {
    const size_t c = k->capids ? 2 * k->capids : 4096;
    int64_t* f = realloc(k->idoff, sizeof(int64_t) * c);
    if (f) k->idoff = f;
    int64_t* h = realloc(k->idhash, sizeof(int64_t) * c);
    if (h) k->idhash = h;
    if (!f || !h) return -1;
    k->capids = c;
  }
  k->idoff[k->nids] = (int64_t)k->n;
  k->idhash[k->nids] = (int64_t)id_hash64(p, n);
  ++k->nids;
  memcpy(k->buf + k->n, p, n);
  k->n += n;
  ++k->nid;
  return 0;
}

static inline size_t sink_id_end(const IdSink* k, size_t x) {
  return x + 1 < k->nids ? (size_t)k->idoff[x + 1] : k->n;
}

static void sink_free(IdSink* k) {
  free(k->buf);
  free(k->idoff);
  free(k->idhash);
}

/* prefix + a [+ ":" + b] into the sink: its put's result, -1 = id too long (hand over) */
static inline int s_try(IdSink* k, const char* pre, size_t pn, const char* a, size_t an,
                        const char* b, Py_ssize_t bn) {
  IdBuf B;
  B.n = 0;
  B.ovf = 0;
  ib_put(&B, pre, pn);
  ib_put(&B, a, an);
  if (bn >= 0) {
    ib_put(&B, ":", 1);
    ib_put(&B, b, (size_t)bn);
  }
  if (B.ovf) return -1;
  return k->put(k, B.b, B.n);
}

/* One row on a worker: 0 = done (*seeds = the row seeds: it has candidate ids, all given to the
 * sink, and a strength > 0 or NaN in *sv), 1 = hand over.  The ids are given in attach_ids'
 * order; a sink that returns 1 stops the row there. */
static int s_row_ids(PyObject* ev, IdSink* k, int* seeds, double* svp) {
  *seeds = 0;
  if (!PyDict_CheckExact(ev)) return 1;
  PyObject* o[5];
  if (w_get(ev, K_SEED, 5, o)) return 1;
  PyObject *t = o[0], *ns = o[1], *name = o[2], *data = o[3], *st = o[4];
  /* float(ev.get("signal_strength", 0.5)): evaluated for every row (seeds._row) */
  double sv;
  if (st == NULL) sv = 0.5;
  else if (PyFloat_CheckExact(st)) sv = PyFloat_AS_DOUBLE(st);
  else if (PyBool_Check(st)) sv = st == Py_True ? 1.0 : 0.0;
  else if (PyLong_CheckExact(st)) {
    int ovf = 0;
    const long long x = PyLong_AsLongLongAndOverflow(st, &ovf);
    if (ovf) return 1;
    sv = (double)x;                 /* round to nearest, as float(int) */
  } else return 1;
  *svp = sv;
  if (t == NULL || t == Py_None) return 0;                       /* no candidate */
  if (!PyUnicode_CheckExact(t)) return 1;
  if (data != NULL && data != Py_None && !PyDict_CheckExact(data)) return 1;
  const char *a, *b;
  Py_ssize_t an, bn;
  if (w_part(ns, &a, &an) || w_part(name, &b, &bn)) return 1;
  int ty = -1;
  for (int i = 0; i < ST_N; ++i) {
    const int eq = w_eq_obj(t, *seed_types[i]);
    if (eq < 0) return 1;
    if (eq) { ty = i; break; }
  }
  if (ty < 0) return 0;                                          /* any other type: none */
  if (sv <= 0.0) return 0;                                       /* `s <= 0` (NaN seeds) */
  PyObject *kind = NULL, *oname = NULL, *ons = NULL;
  if (ty == ST_EVENT) {                   /* (the involved object is read before any id is given) */
    PyObject* obj = NULL;
    if (data != NULL && data != Py_None && PyDict_GET_SIZE(data) > 0 && w_get(data, K_INV, 1, &obj))
      return 1;
    if (obj != NULL && obj != Py_None && !PyDict_CheckExact(obj)) return 1;
    if (obj != NULL && (obj == Py_None || PyDict_GET_SIZE(obj) == 0)) obj = NULL;
    if (obj != NULL) {
      PyObject* q[3];
      if (w_get(obj, K_OBJ, 3, q)) return 1;
      kind = q[0]; oname = q[1]; ons = q[2];
    }
  }
  const char *kp = "", *op = NULL, *sp = NULL;
  Py_ssize_t kn = 0, on = 0, sn = 0;
  char kl[64];
  if (ty == ST_EVENT) {
    /* kind = str(obj.get("kind", "")).lower() (ASCII here: lower() is per-byte) */
    if (kind != NULL && w_part(kind, &kp, &kn)) return 1;
    if (kn >= (Py_ssize_t)sizeof(kl)) return 1;
    for (Py_ssize_t i = 0; i < kn; ++i) kl[i] = (char)((kp[i] >= 'A' && kp[i] <= 'Z') ? kp[i] + 32 : kp[i]);
    if (w_part(oname, &op, &on)) return 1;                      /* obj.get('name') */
    if (ons == NULL) { sp = a; sn = an; }                        /* obj.get('namespace', ns) */
    else if (w_part(ons, &sp, &sn)) return 1;
  }
  *seeds = 1;
  int r = 0;
#define TRY(pre, x, xn, y, yn) do {                                              \
    r = s_try(k, pre, sizeof(pre) - 1, x, (size_t)(xn), y, yn);                \
    if (r < 0) return 1;                                                       \
    if (r > 0) return 0;                                                       \
  } while (0)
  switch (ty) {
    case ST_POD: TRY("pod:", a, an, b, bn); break;
    case ST_DEPLOY: case ST_DCHANGE: case ST_ICHANGE: TRY("deployment:", a, an, b, bn); break;
    case ST_NODE: TRY("node:", b, bn, NULL, -1); break;
    case ST_HPA: TRY("hpa:", a, an, b, bn); break;
    case ST_CONFIG: TRY("configmap:", a, an, b, bn); break;
    case ST_LOG:
      TRY("logpattern:", a, an, b, bn);
      TRY("service:", a, an, b, bn);
      TRY("deployment:", a, an, b, bn);
      break;
    case ST_METRIC: TRY("metric:", a, an, b, bn); break;
    case ST_EVENT:
      TRY("event:", a, an, b, bn);
      if (kn == 4 && memcmp(kl, "node", 4) == 0) {
        TRY("node:", op, on, NULL, -1);
      } else if (kn > 0) {
        IdBuf B;
        B.n = 0;
        B.ovf = 0;
        ib_put(&B, kl, (size_t)kn);
        ib_put(&B, ":", 1);
        ib_put(&B, sp, (size_t)sn);
        ib_put(&B, ":", 1);
        ib_put(&B, op, (size_t)on);
        if (B.ovf) return 1;
        r = k->put(k, B.b, B.n);
        if (r < 0) return 1;
      }
      break;
  }
#undef TRY
  return 0;
}

/* One row on a worker for the attachment: 0 = done (*vout = the attached vertex or NO_NODE),
 * 1 = hand over */
static int s_row(PyObject* ev, FindFn find, GraphP g, uint32_t* vout, float* sout) {
  *vout = NO_NODE;
  IdSink k;
  memset(&k, 0, sizeof(k));
  k.put = sink_find;
  k.find = find;
  k.g = g;
  k.v = -1;
  int seeds = 0;
  double sv = 0.0;
  if (s_row_ids(ev, &k, &seeds, &sv)) return 1;
  if (seeds && k.v >= 0) {
    *vout = (uint32_t)k.v;
    *sout = (float)sv;
  }
  return 0;
}

typedef struct {
  PyObject* const* lists;
  const int64_t* base;
  Py_ssize_t i0, i1;
  FindFn find;
  GraphP g;
  uint32_t* vert;
  float* val;
  uint8_t* redo;
  Py_ssize_t* next;          /* the next unclaimed incident (shared; W_CHUNK per claim) */
} SJob;

static void* s_main(void* arg) {
  const SJob* J = (const SJob*)arg;
  for (;;) {
  const Py_ssize_t c0 = __atomic_fetch_add(J->next, (Py_ssize_t)W_CHUNK, __ATOMIC_RELAXED);
  if (c0 >= J->i1) break;
  const Py_ssize_t c1 = c0 + W_CHUNK < J->i1 ? c0 + W_CHUNK : J->i1;
  for (Py_ssize_t i = c0; i < c1; ++i) {
    PyObject* evs = J->lists[i];
    const Py_ssize_t n = PyList_GET_SIZE(evs);
    for (Py_ssize_t j = 0; j < n; ++j) {
      const Py_ssize_t r = J->base[i] + j;
      row_prefetch(evs, j, n);
      J->val[r] = 0.f;
      J->redo[r] = (uint8_t)s_row(PyList_GET_ITEM(evs, j), J->find, J->g, &J->vert[r], &J->val[r]);
    }
  }
  }
  return NULL;
}

/* One row on the calling thread (GIL held): cand_ids, or the Python statement. */
static int s_row_serial(PyObject* ev, PyObject* slow, FindFn find, GraphP g, uint32_t* vout,
                        float* sout, int* ran_python) {
  *vout = NO_NODE;
  PyObject* ids = PyList_New(0);
  if (!ids) return -1;
  double sv = 0.0;
  int fast = 0;
  if (PyDict_CheckExact(ev)) {
    PyObject* st;
    fast = cand_ids(ev, ids);
    if (fast == 1) {
      if (dget(ev, a_strength, &st)) fast = 0;
      else if (st == NULL) sv = 0.5;
      else if (PyFloat_CheckExact(st)) sv = PyFloat_AS_DOUBLE(st);
      else if (PyLong_CheckExact(st) || PyBool_Check(st)) {
        sv = PyLong_AsDouble(st);
        if (sv == -1.0 && PyErr_Occurred()) { PyErr_Clear(); fast = 0; }
      } else fast = 0;
    }
  }
  if (fast < 0) { Py_DECREF(ids); return -1; }
  if (!fast) {                                   /* the Python statement decides (or raises) */
    Py_DECREF(ids);
    *ran_python = 1;
    PyObject* r = PyObject_CallOneArg(slow, ev);
    if (!r) return -1;
    if (!PyArg_ParseTuple(r, "Od", &ids, &sv) || !PyList_Check(ids)) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "seed_attach: bad slow row");
      Py_DECREF(r);
      return -1;
    }
    Py_INCREF(ids);
    Py_DECREF(r);
  }
  const Py_ssize_t k = PyList_GET_SIZE(ids);
  int rc = 0;
  if (k > 0 && !(sv <= 0.0)) {
    for (Py_ssize_t i = 0; i < k; ++i) {
      PyObject* x = PyList_GET_ITEM(ids, i);
      Py_ssize_t n;
      const char* u = PyUnicode_Check(x) ? PyUnicode_AsUTF8AndSize(x, &n) : NULL;
      if (!u) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "seed_attach: candidate id is not a str");
        rc = -1;
        break;
      }
      const int32_t v = find(g, u, (int64_t)n);
      if (v >= 0) {
        *vout = (uint32_t)v;
        *sout = (float)sv;
        break;
      }
    }
  }
  Py_DECREF(ids);
  return rc;
}

static PyObject* seed_attach(PyObject* self, PyObject* args) {
  PyObject *lists, *slow;
  unsigned long long find_addr, g_addr;
  int threads = 1;
  if (!PyArg_ParseTuple(args, "OOKK|i", &lists, &slow, &find_addr, &g_addr, &threads)) return NULL;
  const FindFn find = (FindFn)(uintptr_t)find_addr;
  GraphP g = (GraphP)(uintptr_t)g_addr;
  if (!find || !g) {
    PyErr_SetString(PyExc_ValueError, "seed_attach: NULL find function or graph");
    return NULL;
  }
  PyObject* seq = PySequence_Fast(lists, "evidence_lists must be a sequence");
  if (!seq) return NULL;
  PyObject* result = NULL;
  int64_t* base = NULL;
  uint32_t *wv = NULL, *ov = NULL, *oc = NULL;
  float *wval = NULL, *os = NULL;
  uint8_t* redo = NULL;
  Py_ssize_t nout = 0, cap = 0;
  const Py_ssize_t B = PySequence_Fast_GET_SIZE(seq);
  int par = threads > 1;
  Py_ssize_t total = 0;
  for (Py_ssize_t i = 0; par && i < B; ++i) {
    PyObject* evs = PySequence_Fast_GET_ITEM(seq, i);
    if (!PyList_CheckExact(evs)) par = 0;
    else total += PyList_GET_SIZE(evs);
  }
  if (par && total < PAR_MIN_ROWS) par = 0;
  if (par) {
    base = PyMem_Malloc(sizeof(int64_t) * (size_t)(B + 1));
    wv = PyMem_Malloc(sizeof(uint32_t) * (size_t)total);
    wval = PyMem_Malloc(sizeof(float) * (size_t)total);
    redo = PyMem_Malloc((size_t)total);
    if (!base || !wv || !wval || !redo) { PyErr_NoMemory(); goto done; }
    base[0] = 0;
    for (Py_ssize_t i = 0; i < B; ++i) base[i + 1] = base[i] + PyList_GET_SIZE(PySequence_Fast_GET_ITEM(seq, i));
    if (threads > PAR_MAX_THREADS) threads = PAR_MAX_THREADS;
    SJob jobs[PAR_MAX_THREADS];
    Py_ssize_t next = 0;                 /* every job claims W_CHUNK incidents at a time */
    for (int t = 0; t < threads; ++t)
      jobs[t] = (SJob){PySequence_Fast_ITEMS(seq), base, 0, B, find, g, wv, wval, redo, &next};
    pool_run_fn(s_main, jobs, sizeof(SJob), threads);   /* (the GIL stays held) */
    /* no row for the Python statement: the attached rows straight from the workers' arrays, in
     * row order (the serial loop below would only copy them) */
    int fast = 1;
    for (Py_ssize_t q = 0; q < total && fast; ++q) fast = !redo[q];
    if (fast) {
      for (Py_ssize_t q = 0; q < total; ++q) nout += wv[q] != NO_NODE;
      const size_t m = nout ? (size_t)nout : 1;
      ov = PyMem_Malloc(m * sizeof(uint32_t));
      oc = PyMem_Malloc(m * sizeof(uint32_t));
      os = PyMem_Malloc(m * sizeof(float));
      if (!ov || !oc || !os) { PyErr_NoMemory(); goto done; }
      Py_ssize_t k = 0;
      for (Py_ssize_t c = 0; c < B; ++c)
        for (Py_ssize_t q = base[c]; q < base[c + 1]; ++q)
          if (wv[q] != NO_NODE) {
            ov[k] = wv[q];
            oc[k] = (uint32_t)c;
            os[k] = wval[q];
            ++k;
          }
      result = Py_BuildValue("(y#y#y#)", (const char*)ov, nout * (Py_ssize_t)sizeof(uint32_t),
                             (const char*)oc, nout * (Py_ssize_t)sizeof(uint32_t), (const char*)os,
                             nout * (Py_ssize_t)sizeof(float));
      goto done;
    }
  }
  {
    int ran_python = 0;
    Py_ssize_t r = 0;
    for (Py_ssize_t i = 0; i < B; ++i) {
      PyObject* evs = PySequence_Fast(PySequence_Fast_GET_ITEM(seq, i), "evidence is not iterable");
      if (!evs) goto done;
      const Py_ssize_t n = PySequence_Fast_GET_SIZE(evs);
      for (Py_ssize_t j = 0; j < n; ++j, ++r) {
        uint32_t v;
        float x = 0.f;
        if (par && !ran_python && !redo[r]) {
          v = wv[r];
          x = wval[r];
        } else if (!par && !ran_python &&
                   s_row(PySequence_Fast_GET_ITEM(evs, j), find, g, &v, &x) == 0) {
          /* (a small batch: the worker's row function on this thread) */
        } else if (s_row_serial(PySequence_Fast_GET_ITEM(evs, j), slow, find, g, &v, &x, &ran_python) < 0) {
          Py_DECREF(evs);
          goto done;
        }
        if (v == NO_NODE) continue;
        if (nout == cap) {
          cap = cap ? 2 * cap : 4096;
          uint32_t* v2 = PyMem_Realloc(ov, cap * sizeof(uint32_t));
          if (v2) ov = v2;
          uint32_t* c2 = PyMem_Realloc(oc, cap * sizeof(uint32_t));
          if (c2) oc = c2;
          float* s2 = PyMem_Realloc(os, cap * sizeof(float));
          if (s2) os = s2;
          if (!v2 || !c2 || !s2) { PyErr_NoMemory(); Py_DECREF(evs); goto done; }
        }
        ov[nout] = v;
        oc[nout] = (uint32_t)i;
        os[nout] = x;
        ++nout;
      }
      Py_DECREF(evs);
    }
  }
  result = Py_BuildValue("(y#y#y#)", (const char*)ov, nout * (Py_ssize_t)sizeof(uint32_t),
                         (const char*)oc, nout * (Py_ssize_t)sizeof(uint32_t), (const char*)os,
                         nout * (Py_ssize_t)sizeof(float));
done:
  PyMem_Free(base);
  PyMem_Free(wv);
  PyMem_Free(wval);
  PyMem_Free(redo);
  PyMem_Free(ov);
  PyMem_Free(oc);
  PyMem_Free(os);
  Py_DECREF(seq);
  return result;
}

/* ---- fused-rank reuse (egraph/ranker.py FusedRanks) ----------------------------------------
 * A launch's fields travel as ONE bytes block `blk` of m rows (FusedRanks.register packs it with
 * numpy); row j (stride FR_STRIDE(S), S = R + 1 slots): order_conf u8[S] @0, order_rank u8[S] @S,
 * then from a8 = (2S + 7) & ~7 confidence f64[S], signal_strength f64[S], final_score f64[S].
 * A record is (ids tuple, catalog, blk, j, cat) with cat = (R, rule categories, rule support
 * counts, (confidence, category, support, strength) of the unknown hypothesis).
 *
 * fused_records(lists, blk, cat_obj, cat) -> [(first id, record)] for the non-empty lists
 * (lists[j] = row j), so that registering a launch's lists costs no Python loop.
 *
 * fused_apply(hyps, rec) -> the ranked list, False (not the registered list: a miss), or None
 * (a value this path does not compare without Python: FusedRanks.apply decides).  The checks are
 * FusedRanks.apply's, in its order: every dict is an exact dict with the registered id at its
 * position and the four ranker inputs the kernel emitted; then final_score / rank are written as
 * egr_rank would. */
static PyObject *f_confidence, *f_category, *f_support, *f_final, *f_rank, *f_unknown, *f_half,
    *f_zero;

static inline Py_ssize_t fr_a8(Py_ssize_t S) { return (2 * S + 7) & ~(Py_ssize_t)7; }
static inline Py_ssize_t fr_stride(Py_ssize_t S) { return fr_a8(S) + 24 * S; }

/* v (borrowed, NULL = missing -> dflt) == want for plain numbers: 1 / 0, -1 = not plain */
static inline int f_num_eq(PyObject* v, PyObject* dflt, PyObject* want) {
  if (v == NULL) v = dflt;
  if (!(PyFloat_CheckExact(v) || PyLong_CheckExact(v) || PyBool_Check(v))) return -1;
  return PyObject_RichCompareBool(v, want, Py_EQ);   /* built-in numbers: no user code */
}
/* the same against a float64 the kernel wrote (Python's int == float semantics kept: a non-float
 * value is compared through a float object) */
static inline int f_num_eq_d(PyObject* v, PyObject* dflt, double want) {
  if (v == NULL) v = dflt;
  if (PyFloat_CheckExact(v)) return PyFloat_AS_DOUBLE(v) == want;
  if (!(PyLong_CheckExact(v) || PyBool_Check(v))) return -1;
  PyObject* w = PyFloat_FromDouble(want);
  if (!w) return -1;
  const int eq = PyObject_RichCompareBool(v, w, Py_EQ);
  Py_DECREF(w);
  return eq;
}

static PyObject* fused_records(PyObject* self, PyObject* args) {
  PyObject *lists, *blk, *catobj, *cat;
  if (!PyArg_ParseTuple(args, "O!O!OO!", &PyList_Type, &lists, &PyBytes_Type, &blk, &catobj,
                        &PyTuple_Type, &cat))
    return NULL;
  Py_ssize_t R;
  PyObject *cats, *sups, *unk;
  if (!PyArg_ParseTuple(cat, "nOOO", &R, &cats, &sups, &unk)) return NULL;
  const Py_ssize_t m = PyList_GET_SIZE(lists), S = R + 1;
  if (R < 0 || PyBytes_GET_SIZE(blk) < m * fr_stride(S)) {
    PyErr_SetString(PyExc_ValueError, "fused_records: the block is smaller than its rows");
    return NULL;
  }
  PyObject* out = PyList_New(0);
  if (!out) return NULL;
  for (Py_ssize_t j = 0; j < m; ++j) {
    PyObject* hyps = PyList_GET_ITEM(lists, j);
    if (!PyList_Check(hyps)) {
      PyErr_SetString(PyExc_TypeError, "fused_records: a hypothesis list is not a list");
      goto fail;
    }
    const Py_ssize_t n = PyList_GET_SIZE(hyps);
    if (n == 0) continue;
    PyObject* ids = PyTuple_New(n);
    if (!ids) goto fail;
    for (Py_ssize_t p = 0; p < n; ++p) {
      PyObject* h = PyList_GET_ITEM(hyps, p);
      PyObject* hid = PyDict_Check(h) ? PyDict_GetItemWithError(h, k_id) : NULL;
      if (!hid) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_KeyError, "id");
        Py_DECREF(ids);
        goto fail;
      }
      Py_INCREF(hid);
      PyTuple_SET_ITEM(ids, p, hid);
    }
    PyObject* rec = Py_BuildValue("(OOOnO)", ids, catobj, blk, j, cat);
    PyObject* kr = rec ? PyTuple_Pack(2, PyTuple_GET_ITEM(ids, 0), rec) : NULL;
    Py_DECREF(ids);
    Py_XDECREF(rec);
    if (!kr || PyList_Append(out, kr) < 0) { Py_XDECREF(kr); goto fail; }
    Py_DECREF(kr);
  }
  return out;
fail:
  Py_DECREF(out);
  return NULL;
}

static PyObject* fused_verify_apply(PyObject* hyps, PyObject* rec) {
  if (PyTuple_GET_SIZE(rec) != 5 || !PyTuple_Check(PyTuple_GET_ITEM(rec, 4))) Py_RETURN_NONE;
  PyObject *ids = PyTuple_GET_ITEM(rec, 0), *blk = PyTuple_GET_ITEM(rec, 2);
  const Py_ssize_t row = PyLong_AsSsize_t(PyTuple_GET_ITEM(rec, 3));
  if (row < 0) { PyErr_Clear(); Py_RETURN_NONE; }
  PyObject *cats, *sups, *unk;
  Py_ssize_t R;
  if (!PyArg_ParseTuple(PyTuple_GET_ITEM(rec, 4), "nOOO", &R, &cats, &sups, &unk)) return NULL;
  const Py_ssize_t n = PyList_GET_SIZE(hyps), S = R + 1;
  if (!PyTuple_Check(ids) || PyTuple_GET_SIZE(ids) != n || !PyBytes_Check(blk) ||
      PyBytes_GET_SIZE(blk) < (row + 1) * fr_stride(S) || !PyTuple_Check(cats) ||
      !PyTuple_Check(sups) || !PyTuple_Check(unk) || PyTuple_GET_SIZE(unk) != 4 ||
      PyTuple_GET_SIZE(cats) < R || PyTuple_GET_SIZE(sups) < R)
    Py_RETURN_NONE;
  const unsigned char* rb = (const unsigned char*)PyBytes_AS_STRING(blk) + row * fr_stride(S);
  const unsigned char *slots = rb, *orank = rb + S;
  double conf[64], strength[64], final[64];
  Py_ssize_t pos[64];
  if (n > 64 || R >= 64 || n > S) Py_RETURN_NONE;
  memcpy(conf, rb + fr_a8(S), 8 * S);
  memcpy(strength, rb + fr_a8(S) + 8 * S, 8 * S);
  memcpy(final, rb + fr_a8(S) + 16 * S, 8 * S);
  for (Py_ssize_t q = 0; q < 64; ++q) pos[q] = -1;
  for (Py_ssize_t p = 0; p < n; ++p) {
    PyObject* h = PyList_GET_ITEM(hyps, p);
    if (!PyDict_CheckExact(h)) Py_RETURN_NONE;
    PyObject *hid, *c, *cg, *sp, *st;
    if (dget(h, k_id, &hid) || dget(h, f_confidence, &c) || dget(h, f_category, &cg) ||
        dget(h, f_support, &sp) || dget(h, h_strength, &st))
      Py_RETURN_NONE;
    PyObject* want_id = PyTuple_GET_ITEM(ids, p);
    if (hid == NULL || !PyUnicode_CheckExact(hid) || !PyUnicode_CheckExact(want_id)) Py_RETURN_NONE;
    if (PyUnicode_Compare(hid, want_id) != 0) Py_RETURN_FALSE;
    const Py_ssize_t slot = slots[p];
    if (slot > R) Py_RETURN_NONE;
    int eq;
    PyObject *wcat, *wsup;
    if (slot == R) {
      wcat = PyTuple_GET_ITEM(unk, 1);
      wsup = PyTuple_GET_ITEM(unk, 2);
      eq = f_num_eq(c, f_half, PyTuple_GET_ITEM(unk, 0));
    } else {
      wcat = PyTuple_GET_ITEM(cats, slot);
      wsup = PyTuple_GET_ITEM(sups, slot);
      eq = f_num_eq_d(c, f_half, conf[slot]);
    }
    if (eq < 0) { PyErr_Clear(); Py_RETURN_NONE; }
    if (!eq) Py_RETURN_FALSE;
    if (cg == NULL) cg = f_unknown;
    if (!PyUnicode_CheckExact(cg) || !PyUnicode_CheckExact(wcat)) Py_RETURN_NONE;
    if (PyUnicode_Compare(cg, wcat) != 0) Py_RETURN_FALSE;
    if ((eq = f_num_eq(sp, f_zero, wsup)) < 0) { PyErr_Clear(); Py_RETURN_NONE; }
    if (!eq) Py_RETURN_FALSE;
    eq = slot == R ? f_num_eq(st, f_zero, PyTuple_GET_ITEM(unk, 3)) : f_num_eq_d(st, f_zero, strength[slot]);
    if (eq < 0) { PyErr_Clear(); Py_RETURN_NONE; }
    if (!eq) Py_RETURN_FALSE;
    if (pos[slot] >= 0) Py_RETURN_NONE;          /* (a slot twice: not a kernel list) */
    pos[slot] = p;
  }
  /* verified: final scores, then the kernel's order and ranks */
  PyObject* out = PyList_New(n);
  if (!out) return NULL;
  for (Py_ssize_t q = 0; q < n; ++q) {
    const Py_ssize_t slot = orank[q];
    if (slot > R || pos[slot] < 0) {
      Py_DECREF(out);
      Py_RETURN_NONE;
    }
    PyObject* h = PyList_GET_ITEM(hyps, pos[slot]);
    Py_INCREF(h);
    PyList_SET_ITEM(out, q, h);
  }
  for (Py_ssize_t p = 0; p < n; ++p) {
    PyObject* h = PyList_GET_ITEM(hyps, p);
    PyObject* f = PyFloat_FromDouble(final[slots[p]]);
    if (!f || PyDict_SetItem(h, f_final, f) < 0) { Py_XDECREF(f); Py_DECREF(out); return NULL; }
    Py_DECREF(f);
  }
  for (Py_ssize_t q = 0; q < n; ++q) {
    PyObject* r = PyLong_FromSsize_t(q + 1);
    if (!r || PyDict_SetItem(PyList_GET_ITEM(out, q), f_rank, r) < 0) {
      Py_XDECREF(r);
      Py_DECREF(out);
      return NULL;
    }
    Py_DECREF(r);
  }
  return out;
}

static PyObject* fused_apply(PyObject* self, PyObject* args) {
  PyObject *hyps, *rec;
  if (!PyArg_ParseTuple(args, "O!O!", &PyList_Type, &hyps, &PyTuple_Type, &rec)) return NULL;
  return fused_verify_apply(hyps, rec);
}

/* fused_rank(recs, hyps) -> FusedRanks.apply for an exact list, lookup included: the ranked list
 * (a hit), 0 (a miss: no record of that first id, another length, or fused_apply's False), 1
 * (not a candidate: empty, or a first item that is not a dict; counted as neither), or None (a
 * value only Python compares: FusedRanks.apply's statements decide). */
static PyObject* fused_rank(PyObject* self, PyObject* args) {
  PyObject *recs, *hyps;
  if (!PyArg_ParseTuple(args, "O!O!", &PyDict_Type, &recs, &PyList_Type, &hyps)) return NULL;
  if (PyList_GET_SIZE(hyps) == 0) return PyLong_FromLong(1);
  PyObject* h0 = PyList_GET_ITEM(hyps, 0);
  if (!PyDict_Check(h0)) return PyLong_FromLong(1);
  if (!PyDict_CheckExact(h0)) Py_RETURN_NONE;
  PyObject *hid, *rec;
  if (dget(h0, k_id, &hid)) Py_RETURN_NONE;
  if (hid == NULL) hid = Py_None;
  rec = PyDict_GetItemWithError(recs, hid);
  if (rec == NULL) {
    if (PyErr_Occurred()) { PyErr_Clear(); Py_RETURN_NONE; }   /* (an unhashable id: Python raises) */
    return PyLong_FromLong(0);
  }
  if (!PyTuple_Check(rec) || PyTuple_GET_SIZE(rec) < 1 || !PyTuple_Check(PyTuple_GET_ITEM(rec, 0)))
    Py_RETURN_NONE;
  if (PyTuple_GET_SIZE(PyTuple_GET_ITEM(rec, 0)) != PyList_GET_SIZE(hyps)) return PyLong_FromLong(0);
  Py_INCREF(rec);                                  /* (the checks below may run no Python code,
                                                      but hold the record anyway) */
  PyObject* r = fused_verify_apply(hyps, rec);
  Py_DECREF(rec);
  if (r == Py_False) { Py_DECREF(r); return PyLong_FromLong(0); }
  return r;
}

/* ---- seed attachment candidates as keys (egraph/seeds.py SeedCandidates.per_column keys=True)
 * seed_keys(evidence_lists, slow[, threads]) -> (blob, off i64 [n+1], hash i64 [n], count i64
 * [rows], col u32 [rows], val f32 [rows]): SeedCandidates(evidence_lists) with its candidate ids
 * as ONE UTF-8 blob + offsets + 64-bit hashes of the bytes (id_hash64, the alert storm's pending
 * index key; pyhost.hash_ids hashes query ids the same way) instead of a list of Python strs.
 * Row pass on the worker pool as seed_attach; rows handed over are redone serially in row order. */
static inline uint64_t id_hash64(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)n * 0xFF51AFD7ED558CCDull);
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    h = (h ^ (w * 0xC4CEB9FE1A85EC53ull)) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    p += 8;
    n -= 8;
  }
  if (n) {
    uint64_t w = 0;
    memcpy(&w, p, n);
    h = (h ^ (w * 0xC4CEB9FE1A85EC53ull)) * 0x9E3779B97F4A7C15ull;
  }
  h ^= h >> 32;
  h *= 0xD6E8FEB86659FD93ull;
  return h ^ (h >> 32);
}

typedef struct {
  PyObject* const* lists;
  const int64_t* base;
  Py_ssize_t i0, i1;
  IdSink sink;                  /* this job's ids (bytes, offsets, hashes) */
  int64_t* rowpos;              /* per row: the index of its first id in the job's sink */
  uint8_t* nid;                 /* per row: ids given (0: the row does not seed) */
  float* val;
  uint8_t* redo;
  int64_t* rcount;              /* the job's seeding rows in order: id count, column, strength */
  uint32_t* rcol;
  float* rval;
  Py_ssize_t nrows, nredo;
} KJob;

static void* k_main(void* arg) {
  KJob* J = (KJob*)arg;
  for (Py_ssize_t i = J->i0; i < J->i1; ++i) {
    PyObject* evs = J->lists[i];
    const Py_ssize_t n = PyList_GET_SIZE(evs);
    for (Py_ssize_t j = 0; j < n; ++j) {
      const Py_ssize_t r = J->base[i] + j;
      row_prefetch(evs, j, n);
      const size_t pos = J->sink.n, ipos = J->sink.nids;
      J->sink.nid = 0;
      int seeds = 0;
      double sv = 0.0;
      const int redo = s_row_ids(PyList_GET_ITEM(evs, j), &J->sink, &seeds, &sv);
      J->redo[r] = (uint8_t)redo;
      J->rowpos[r] = (int64_t)ipos;
      if (redo) {                                  /* (drop a partial row) */
        J->sink.n = pos;
        J->sink.nids = ipos;
        ++J->nredo;
      }
      J->nid[r] = (uint8_t)(redo || !seeds ? 0 : J->sink.nid);
      J->val[r] = (float)sv;
      if (J->nid[r] && !(sv <= 0.0)) {
        J->rcount[J->nrows] = J->nid[r];
        J->rcol[J->nrows] = (uint32_t)i;
        J->rval[J->nrows] = (float)sv;
        ++J->nrows;
      }
    }
  }
  return NULL;
}

typedef struct {
  char* blob;
  int64_t *off, *hash, *count;
  uint32_t* col;
  float* val;
  Py_ssize_t nb, capb, nf, capf, nr, capr;
} KOut;

static int kout_id(KOut* o, const char* p, size_t n) {
  if ((size_t)(o->capb - o->nb) < n) {
    Py_ssize_t c = o->capb ? 2 * o->capb : 1 << 16;
    while ((size_t)(c - o->nb) < n) c *= 2;
    char* b = PyMem_Realloc(o->blob, (size_t)c);
    if (!b) { PyErr_NoMemory(); return -1; }
    o->blob = b;
    o->capb = c;
  }
  if (o->nf + 2 > o->capf) {
    const Py_ssize_t c = o->capf ? 2 * o->capf : 4096;
    int64_t* f = PyMem_Realloc(o->off, sizeof(int64_t) * (size_t)c);
    if (f) o->off = f;
    int64_t* h = PyMem_Realloc(o->hash, sizeof(int64_t) * (size_t)c);
    if (h) o->hash = h;
    if (!f || !h) { PyErr_NoMemory(); return -1; }
    o->capf = c;
  }
  memcpy(o->blob + o->nb, p, n);
  o->off[o->nf] = o->nb;
  o->hash[o->nf] = (int64_t)id_hash64(p, n);
  o->nb += (Py_ssize_t)n;
  ++o->nf;
  return 0;
}

static int kout_row(KOut* o, int64_t k, uint32_t col, float v) {
  if (o->nr == o->capr) {
    const Py_ssize_t c = o->capr ? 2 * o->capr : 4096;
    int64_t* a = PyMem_Realloc(o->count, sizeof(int64_t) * (size_t)c);
    if (a) o->count = a;
    uint32_t* b = PyMem_Realloc(o->col, sizeof(uint32_t) * (size_t)c);
    if (b) o->col = b;
    float* d = PyMem_Realloc(o->val, sizeof(float) * (size_t)c);
    if (d) o->val = d;
    if (!a || !b || !d) { PyErr_NoMemory(); return -1; }
    o->capr = c;
  }
  o->count[o->nr] = k;
  o->col[o->nr] = col;
  o->val[o->nr] = v;
  ++o->nr;
  return 0;
}

/* One row on the calling thread: cand_ids or the Python statement, its ids appended */
static int k_row_serial(PyObject* ev, PyObject* slow, KOut* o, uint32_t col, int* ran_python) {
  PyObject* ids = PyList_New(0);
  if (!ids) return -1;
  double sv = 0.0;
  int fast = 0;
  if (PyDict_CheckExact(ev)) {
    PyObject* st;
    fast = cand_ids(ev, ids);
    if (fast == 1) {
      if (dget(ev, a_strength, &st)) fast = 0;
      else if (st == NULL) sv = 0.5;
      else if (PyFloat_CheckExact(st)) sv = PyFloat_AS_DOUBLE(st);
      else if (PyLong_CheckExact(st) || PyBool_Check(st)) {
        sv = PyLong_AsDouble(st);
        if (sv == -1.0 && PyErr_Occurred()) { PyErr_Clear(); fast = 0; }
      } else fast = 0;
    }
  }
  if (fast < 0) { Py_DECREF(ids); return -1; }
  if (!fast) {
    Py_DECREF(ids);
    *ran_python = 1;
    PyObject* r = PyObject_CallOneArg(slow, ev);
    if (!r) return -1;
    if (!PyArg_ParseTuple(r, "Od", &ids, &sv) || !PyList_Check(ids)) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "seed_keys: bad slow row");
      Py_DECREF(r);
      return -1;
    }
    Py_INCREF(ids);
    Py_DECREF(r);
  }
  const Py_ssize_t k = PyList_GET_SIZE(ids);
  int rc = 0;
  if (k > 0 && !(sv <= 0.0)) {
    for (Py_ssize_t i = 0; i < k && rc == 0; ++i) {
      PyObject* x = PyList_GET_ITEM(ids, i);
      Py_ssize_t n;
      const char* u = PyUnicode_Check(x) ? PyUnicode_AsUTF8AndSize(x, &n) : NULL;
      if (!u) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "seed_keys: candidate id is not a str");
        rc = -1;
      } else {
        rc = kout_id(o, u, (size_t)n);
      }
    }
    if (rc == 0) rc = kout_row(o, k, col, (float)sv);
  }
  Py_DECREF(ids);
  return rc;
}

static PyObject* seed_keys(PyObject* self, PyObject* args) {
  PyObject *lists, *slow;
  int threads = 1;
  if (!PyArg_ParseTuple(args, "OO|i", &lists, &slow, &threads)) return NULL;
  PyObject* seq = PySequence_Fast(lists, "evidence_lists must be a sequence");
  if (!seq) return NULL;
  PyObject* result = NULL;
  KOut o;
  memset(&o, 0, sizeof(o));
  IdSink one;                   /* the calling thread's row sink (small batches), reused per row */
  memset(&one, 0, sizeof(one));
  one.put = sink_keys;
  int64_t* base = NULL;
  int64_t* rowpos = NULL;
  uint8_t *nid = NULL, *redo = NULL, *jobof = NULL;
  float* wval = NULL;
  KJob jobs[PAR_MAX_THREADS];
  int njobs = 0;
  const Py_ssize_t B = PySequence_Fast_GET_SIZE(seq);
  int par = threads > 1;
  Py_ssize_t total = 0;
  for (Py_ssize_t i = 0; par && i < B; ++i) {
    PyObject* evs = PySequence_Fast_GET_ITEM(seq, i);
    if (!PyList_CheckExact(evs)) par = 0;
    else total += PyList_GET_SIZE(evs);
  }
  if (par && total < PAR_MIN_ROWS) par = 0;
  if (par) {
    base = PyMem_Malloc(sizeof(int64_t) * (size_t)(B + 1));
    rowpos = PyMem_Malloc(sizeof(int64_t) * (size_t)total);
    nid = PyMem_Malloc((size_t)total);
    redo = PyMem_Malloc((size_t)total);
    jobof = PyMem_Malloc((size_t)total);
    wval = PyMem_Malloc(sizeof(float) * (size_t)total);
    if (!base || !rowpos || !nid || !redo || !jobof || !wval) { PyErr_NoMemory(); goto done; }
    base[0] = 0;
    for (Py_ssize_t i = 0; i < B; ++i) base[i + 1] = base[i] + PyList_GET_SIZE(PySequence_Fast_GET_ITEM(seq, i));
    if (threads > PAR_MAX_THREADS) threads = PAR_MAX_THREADS;
    Py_ssize_t i = 0;
    for (int t = 0; t < threads; ++t) {
      const int64_t goal = (int64_t)((total * (t + 1)) / threads);
      const Py_ssize_t i0 = i;
      while (i < B && (base[i + 1] <= goal || t == threads - 1)) ++i;
      memset(&jobs[t], 0, sizeof(KJob));
      jobs[t].lists = PySequence_Fast_ITEMS(seq);
      jobs[t].base = base;
      jobs[t].i0 = i0;
      jobs[t].i1 = i;
      jobs[t].sink.put = sink_keys;
      jobs[t].rowpos = rowpos;
      jobs[t].nid = nid;
      jobs[t].val = wval;
      jobs[t].redo = redo;
      const size_t jr = (size_t)(base[i] - base[i0]) + 1;
      jobs[t].rcount = malloc(sizeof(int64_t) * jr);
      jobs[t].rcol = malloc(sizeof(uint32_t) * jr);
      jobs[t].rval = malloc(sizeof(float) * jr);
      njobs = t + 1;
      if (!jobs[t].rcount || !jobs[t].rcol || !jobs[t].rval) { PyErr_NoMemory(); goto done; }
      for (int64_t r = base[i0]; r < base[i]; ++r) jobof[r] = (uint8_t)t;
    }
    pool_run_fn(k_main, jobs, sizeof(KJob), threads);   /* (the GIL stays held) */
  }
  int clean = par;
  for (int t = 0; t < njobs; ++t) clean = clean && jobs[t].nredo == 0;
  if (clean) {
    /* every row stayed on the workers: the output is the jobs' arrays one after another (the jobs
     * hold consecutive lists), offsets shifted by the bytes before each job */
    Py_ssize_t nb = 0, nf = 0, nr = 0;
    for (int t = 0; t < njobs; ++t) {
      nb += (Py_ssize_t)jobs[t].sink.n;
      nf += (Py_ssize_t)jobs[t].sink.nids;
      nr += jobs[t].nrows;
    }
    o.blob = PyMem_Malloc((size_t)nb + 1);
    o.off = PyMem_Malloc(sizeof(int64_t) * (size_t)(nf + 1));
    o.hash = PyMem_Malloc(sizeof(int64_t) * (size_t)(nf + 1));
    o.count = PyMem_Malloc(sizeof(int64_t) * (size_t)(nr + 1));
    o.col = PyMem_Malloc(sizeof(uint32_t) * (size_t)(nr + 1));
    o.val = PyMem_Malloc(sizeof(float) * (size_t)(nr + 1));
    if (!o.blob || !o.off || !o.hash || !o.count || !o.col || !o.val) { PyErr_NoMemory(); goto done; }
    o.capb = nb + 1;
    o.capf = nf + 1;
    o.capr = nr + 1;
    for (int t = 0; t < njobs; ++t) {
      const IdSink* k = &jobs[t].sink;
      if (k->n) memcpy(o.blob + o.nb, k->buf, k->n);
      for (size_t x = 0; x < k->nids; ++x) o.off[o.nf + (Py_ssize_t)x] = o.nb + k->idoff[x];
      if (k->nids) memcpy(o.hash + o.nf, k->idhash, sizeof(int64_t) * k->nids);
      const Py_ssize_t m = jobs[t].nrows;
      if (m) {
        memcpy(o.count + o.nr, jobs[t].rcount, sizeof(int64_t) * (size_t)m);
        memcpy(o.col + o.nr, jobs[t].rcol, sizeof(uint32_t) * (size_t)m);
        memcpy(o.val + o.nr, jobs[t].rval, sizeof(float) * (size_t)m);
      }
      o.nb += (Py_ssize_t)k->n;
      o.nf += (Py_ssize_t)k->nids;
      o.nr += m;
    }
  } else {
    int ran_python = 0;
    Py_ssize_t r = 0;
    for (Py_ssize_t i = 0; i < B; ++i) {
      PyObject* evs = PySequence_Fast(PySequence_Fast_GET_ITEM(seq, i), "evidence is not iterable");
      if (!evs) goto done;
      const Py_ssize_t n = PySequence_Fast_GET_SIZE(evs);
      for (Py_ssize_t j = 0; j < n; ++j, ++r) {
        if (par && !ran_python && !redo[r]) {
          if (!nid[r]) continue;
          const IdSink* k = &jobs[jobof[r]].sink;
          for (size_t x = (size_t)rowpos[r]; x < (size_t)rowpos[r] + nid[r]; ++x) {
            const size_t a = (size_t)k->idoff[x];
            if (kout_id(&o, k->buf + a, sink_id_end(k, x) - a) < 0) { Py_DECREF(evs); goto done; }
          }
          if (kout_row(&o, nid[r], (uint32_t)i, wval[r]) < 0) { Py_DECREF(evs); goto done; }
        } else {
          /* (a small batch: the worker's row function on this thread first) */
          if (!par && !ran_python) {
            IdSink* const kp = &one;
            kp->n = kp->nids = 0;
            kp->nid = 0;
            int seeds = 0;
            double sv = 0.0;
            if (!s_row_ids(PySequence_Fast_GET_ITEM(evs, j), kp, &seeds, &sv)) {
              int bad = 0;
              if (seeds && kp->nid > 0) {
                for (size_t x = 0; x < kp->nids && !bad; ++x) {
                  const size_t a = (size_t)kp->idoff[x];
                  bad = kout_id(&o, kp->buf + a, sink_id_end(kp, x) - a) < 0;
                }
                if (!bad) bad = kout_row(&o, kp->nid, (uint32_t)i, (float)sv) < 0;
              }
              if (bad) { Py_DECREF(evs); goto done; }
              continue;
            }
          }
          if (k_row_serial(PySequence_Fast_GET_ITEM(evs, j), slow, &o, (uint32_t)i, &ran_python) < 0) {
            Py_DECREF(evs);
            goto done;
          }
        }
      }
      Py_DECREF(evs);
    }
  }
  if (o.nf + 1 > o.capf || !o.off) {
    int64_t* f = PyMem_Realloc(o.off, sizeof(int64_t) * (size_t)(o.nf + 1));
    if (!f) { PyErr_NoMemory(); goto done; }
    o.off = f;
  }
  o.off[o.nf] = o.nb;
  result = Py_BuildValue("(y#y#y#y#y#y#)", o.blob ? o.blob : "", o.nb,
                         (const char*)o.off, (o.nf + 1) * (Py_ssize_t)sizeof(int64_t),
                         o.hash ? (const char*)o.hash : "", o.nf * (Py_ssize_t)sizeof(int64_t),
                         o.count ? (const char*)o.count : "", o.nr * (Py_ssize_t)sizeof(int64_t),
                         o.col ? (const char*)o.col : "", o.nr * (Py_ssize_t)sizeof(uint32_t),
                         o.val ? (const char*)o.val : "", o.nr * (Py_ssize_t)sizeof(float));
done:
  sink_free(&one);
  for (int t = 0; t < njobs; ++t) {
    sink_free(&jobs[t].sink);
    free(jobs[t].rcount);
    free(jobs[t].rcol);
    free(jobs[t].rval);
  }
  PyMem_Free(base);
  PyMem_Free(rowpos);
  PyMem_Free(nid);
  PyMem_Free(redo);
  PyMem_Free(jobof);
  PyMem_Free(wval);
  PyMem_Free(o.blob);
  PyMem_Free(o.off);
  PyMem_Free(o.hash);
  PyMem_Free(o.count);
  PyMem_Free(o.col);
  PyMem_Free(o.val);
  Py_DECREF(seq);
  return result;
}

/* hash_ids(ids) -> int64 bytes: id_hash64 of each str's UTF-8 bytes (seed_keys' hashes) */
static PyObject* hash_ids(PyObject* self, PyObject* arg) {
  PyObject* seq = PySequence_Fast(arg, "ids must be a sequence");
  if (!seq) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  int64_t* h = PyMem_Malloc(sizeof(int64_t) * (size_t)(n + 1));
  PyObject* out = NULL;
  if (!h) { PyErr_NoMemory(); goto done; }
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* x = PySequence_Fast_GET_ITEM(seq, i);
    Py_ssize_t len;
    const char* u = PyUnicode_Check(x) ? PyUnicode_AsUTF8AndSize(x, &len) : NULL;
    if (!u) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "hash_ids: ids must be strs");
      goto done;
    }
    h[i] = (int64_t)id_hash64(u, (size_t)len);
  }
  out = PyBytes_FromStringAndSize((const char*)h, n * (Py_ssize_t)sizeof(int64_t));
done:
  PyMem_Free(h);
  Py_DECREF(seq);
  return out;
}

/* attach_idx(found, count) -> (vertex u32 [attached rows], ok u8 [rows], before i64 [m],
 * before_row i64 [m]): SeedCandidates.attach_found_idx's index work in one pass.  found: int64
 * bytes, the graph vertex of each flat candidate id (-1 absent); count: int64 bytes, the ids per
 * row.  A row attaches to its first present id (ok[r] = 1, its vertex appended in row order);
 * `before` lists the flat indices of the ids ranked ahead of it (every id of an unattached row)
 * with their rows. */
static PyObject* attach_idx(PyObject* self, PyObject* args) {
  Py_buffer fb, cb;
  if (!PyArg_ParseTuple(args, "y*y*", &fb, &cb)) return NULL;
  PyObject* out = NULL;
  const int64_t* found = (const int64_t*)fb.buf;
  const int64_t* count = (const int64_t*)cb.buf;
  const Py_ssize_t n = fb.len / (Py_ssize_t)sizeof(int64_t);
  const Py_ssize_t rows = cb.len / (Py_ssize_t)sizeof(int64_t);
  uint32_t* sv = PyMem_Malloc(sizeof(uint32_t) * (size_t)(rows + 1));
  uint8_t* ok = PyMem_Malloc((size_t)rows + 1);
  int64_t* bef = PyMem_Malloc(sizeof(int64_t) * (size_t)(n + 1));
  int64_t* brow = PyMem_Malloc(sizeof(int64_t) * (size_t)(n + 1));
  Py_ssize_t k = 0, m = 0, i = 0;
  if (!sv || !ok || !bef || !brow) { PyErr_NoMemory(); goto done; }
  for (Py_ssize_t r = 0; r < rows; ++r) {
    const int64_t c = count[r];
    if (c < 0 || i + c > n) {
      PyErr_SetString(PyExc_ValueError, "attach_idx: counts exceed the candidate ids");
      goto done;
    }
    ok[r] = 0;
    for (int64_t j = 0; j < c; ++j, ++i) {
      if (ok[r]) continue;
      if (found[i] >= 0) {
        ok[r] = 1;
        sv[k++] = (uint32_t)found[i];
      } else {
        bef[m] = (int64_t)i;
        brow[m++] = (int64_t)r;
      }
    }
  }
  out = Py_BuildValue("(y#y#y#y#)", (const char*)sv, k * (Py_ssize_t)sizeof(uint32_t),
                      (const char*)ok, rows, (const char*)bef, m * (Py_ssize_t)sizeof(int64_t),
                      (const char*)brow, m * (Py_ssize_t)sizeof(int64_t));
done:
  PyMem_Free(sv);
  PyMem_Free(ok);
  PyMem_Free(bef);
  PyMem_Free(brow);
  PyBuffer_Release(&fb);
  PyBuffer_Release(&cb);
  return out;
}

/* str_blob(list of str) -> (UTF-8 blob bytes, int64 offsets [n+1] as bytes), or None when the
 * argument is not an exact list of exact strs (egraph/graph.py str_blob then builds it in
 * Python).  The C-ABI's string arrays for MERGE batches and lookups: one pass for the lengths,
 * one memcpy per id, no per-id bytes object. */
static PyObject* str_blob(PyObject* self, PyObject* arg) {
  if (!PyList_CheckExact(arg)) Py_RETURN_NONE;
  const Py_ssize_t n = PyList_GET_SIZE(arg);
  int64_t* off = PyMem_Malloc(sizeof(int64_t) * (size_t)(n + 1));
  if (!off) return PyErr_NoMemory();
  PyObject* out = NULL;
  off[0] = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* x = PyList_GET_ITEM(arg, i);
    Py_ssize_t len;
    if (!PyUnicode_CheckExact(x) || !PyUnicode_AsUTF8AndSize(x, &len)) {
      PyErr_Clear();
      PyMem_Free(off);
      Py_RETURN_NONE;
    }
    off[i + 1] = off[i] + (int64_t)len;
  }
  PyObject* blob = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)off[n]);
  if (!blob) goto done;
  char* dst = PyBytes_AS_STRING(blob);
  for (Py_ssize_t i = 0; i < n; ++i) {
    Py_ssize_t len;
    const char* u = PyUnicode_AsUTF8AndSize(PyList_GET_ITEM(arg, i), &len);  /* cached: no alloc */
    memcpy(dst + off[i], u, (size_t)len);
  }
  PyObject* ob = PyBytes_FromStringAndSize((const char*)off, (n + 1) * (Py_ssize_t)sizeof(int64_t));
  if (!ob) { Py_DECREF(blob); goto done; }
  out = PyTuple_Pack(2, blob, ob);
  Py_DECREF(blob);
  Py_DECREF(ob);
done:
  PyMem_Free(off);
  return out;
}

/* ---- ranked root-cause entities (src/database/graph.py GraphService._rank_locked) ----------
 * entity_rows(ids u32 [B*k], scores f32 [B*k], labels u8 [B*k], k, vertex_ids list, label_names
 * list) -> B lists of {"id": vertex_ids[v], "labels": [label_names[label]], "score": float,
 * "rank": r}: each list stops at the first EGR_NO_NODE.  Dicts are copies of one 4-key template
 * (keys in the Python statement's order); scores are the f32 values as Python floats, as
 * ndarray.tolist() gives them. */
static PyObject *e_id, *e_labels, *e_score, *e_rank;

static PyObject* entity_rows(PyObject* self, PyObject* args) {
  Py_buffer bi = {0}, bs = {0}, bl = {0};
  PyObject *vids, *names;
  Py_ssize_t k;
  if (!PyArg_ParseTuple(args, "y*y*y*nO!O!", &bi, &bs, &bl, &k, &PyList_Type, &vids, &PyList_Type, &names))
    return NULL;
  PyObject* out = NULL;
  PyObject* tmpl = NULL;
  const Py_ssize_t n = bi.len / 4;
  if (k <= 0 || n % k || bs.len / 4 != n || bl.len != n) {
    PyErr_SetString(PyExc_ValueError, "entity_rows: ids / scores / labels differ in size or k");
    goto done;
  }
  const uint32_t* ids = (const uint32_t*)bi.buf;
  const float* sc = (const float*)bs.buf;
  const uint8_t* lab = (const uint8_t*)bl.buf;
  const Py_ssize_t B = n / k, NV = PyList_GET_SIZE(vids), NL = PyList_GET_SIZE(names);
  if (!(tmpl = PyDict_New())) goto done;
  if (PyDict_SetItem(tmpl, e_id, Py_None) < 0 || PyDict_SetItem(tmpl, e_labels, Py_None) < 0 ||
      PyDict_SetItem(tmpl, e_score, Py_None) < 0 || PyDict_SetItem(tmpl, e_rank, Py_None) < 0)
    goto done;
  if (!(out = PyList_New(B))) goto done;
  /* (the cyclic GC deferred while ~3 objects per entity are created, as the hypothesis
   * assembly does: collections triggered by them traverse the caller's whole heap) */
  const int gc_was = PyGC_Disable();
  /* the id strings are scattered over the heap (one per graph vertex) and each entity takes a
   * reference to one: their headers are prefetched PF entities ahead, so the cache misses of
   * the reference counts overlap instead of queueing one by one */
  enum { PF = 16 };
  for (Py_ssize_t j = 0; j < PF && j < n; ++j)
    if (ids[j] < (uint32_t)NV) __builtin_prefetch(PyList_GET_ITEM(vids, ids[j]), 1, 0);
  for (Py_ssize_t b = 0; b < B; ++b) {
    Py_ssize_t m = 0;
    while (m < k && ids[b * k + m] != NO_NODE) ++m;
    PyObject* row = PyList_New(m);
    if (!row) goto fail;
    PyList_SET_ITEM(out, b, row);
    for (Py_ssize_t r = 0; r < m; ++r) {
      const Py_ssize_t jp = b * k + r + PF;
      if (jp < n && ids[jp] < (uint32_t)NV) __builtin_prefetch(PyList_GET_ITEM(vids, ids[jp]), 1, 0);
      const uint32_t v = ids[b * k + r];
      const uint8_t l = lab[b * k + r];
      if ((Py_ssize_t)v >= NV || (Py_ssize_t)l >= NL) {
        PyErr_SetString(PyExc_IndexError, "entity_rows: vertex or label index out of range");
        goto fail;
      }
      PyObject* d = PyDict_Copy(tmpl);
      if (!d) goto fail;
      PyList_SET_ITEM(row, r, d);
      PyObject* ls = PyList_New(1);
      PyObject* f = PyFloat_FromDouble((double)sc[b * k + r]);
      PyObject* rk = PyLong_FromSsize_t(r + 1);
      if (!ls || !f || !rk) { Py_XDECREF(ls); Py_XDECREF(f); Py_XDECREF(rk); goto fail; }
      PyObject* nm = PyList_GET_ITEM(names, l);
      Py_INCREF(nm);
      PyList_SET_ITEM(ls, 0, nm);
      const int bad = PyDict_SetItem(d, e_id, PyList_GET_ITEM(vids, v)) < 0 ||
                      PyDict_SetItem(d, e_labels, ls) < 0 || PyDict_SetItem(d, e_score, f) < 0 ||
                      PyDict_SetItem(d, e_rank, rk) < 0;
      Py_DECREF(ls);
      Py_DECREF(f);
      Py_DECREF(rk);
      if (bad) goto fail;
    }
  }
  if (gc_was) PyGC_Enable();
  goto done;
fail:
  if (gc_was) PyGC_Enable();
  Py_CLEAR(out);
done:
  Py_XDECREF(tmpl);
  PyBuffer_Release(&bi);
  PyBuffer_Release(&bs);
  PyBuffer_Release(&bl);
  return out;
}

static PyMethodDef methods[] = {
    {"seed_candidates", seed_candidates, METH_VARARGS, "evidence rows -> seed attachment candidates"},
    {"entity_rows", entity_rows, METH_VARARGS, "frontier top-k -> ranked root-cause entity dicts"},
    {"seed_keys", seed_keys, METH_VARARGS, "evidence rows -> seed candidates as a keyed blob"},
    {"hash_ids", hash_ids, METH_O, "64-bit hashes of ids' UTF-8 bytes"},
    {"attach_idx", attach_idx, METH_VARARGS, "first present candidate per row + the ids before it"},
    {"str_blob", str_blob, METH_O, "list of str -> (UTF-8 blob, int64 offsets)"},
    {"fused_apply", fused_apply, METH_VARARGS, "verify + apply a registered fused ranking"},
    {"fused_rank", fused_rank, METH_VARARGS, "FusedRanks.apply for an exact list, lookup included"},
    {"fused_records", fused_records, METH_VARARGS, "a launch's hypothesis lists -> fused-rank records"},
    {"seed_attach", seed_attach, METH_VARARGS, "evidence rows -> attached (vertex, column, strength) seeds"},
    {"encode_rows", encode_rows, METH_VARARGS, "evidence dicts -> row columns"},
    {"assemble", assemble, METH_VARARGS, "kernel outputs -> hypothesis dicts"},
    {"flag_bits", flag_bits, METH_NOARGS, "the EGR_F_* bits and EGR_NO_NODE compiled in"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_egr_pyhost", NULL, -1, methods};

PyMODINIT_FUNC PyInit__egr_pyhost(void) {
  if (intern_all() < 0 || intern_seeds() < 0 || intern_worker_keys() < 0) return NULL;
#define S(var, text) if (!(var = PyUnicode_InternFromString(text))) return NULL
  S(f_confidence, "confidence"); S(f_category, "category"); S(f_support, "support_count");
  S(f_final, "final_score"); S(f_rank, "rank"); S(f_unknown, "unknown");
  S(e_id, "id"); S(e_labels, "labels"); S(e_score, "score"); S(e_rank, "rank");
#undef S
  if (!(f_half = PyFloat_FromDouble(0.5)) || !(f_zero = PyLong_FromLong(0))) return NULL;
  return PyModule_Create(&module);
}
