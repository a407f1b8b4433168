/*
 * keto_oracle.c -- C restatement of Keto's check / expand engines over the ordered tuple
 * table.  TEST INFRASTRUCTURE ONLY: used by tests/ (parity checker), __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg.  Never linked into, or called by, the keto_amd product.
 *
 * Parity status: pinned.  tests/test_oracle_c.py checks this restatement against the
 * SQL-level oracle (oracle/oracle_sql.py, itself pinned to the reference's golden vectors in
 * tests/golden/reference_cases.json) on every golden case and on thousands of random graphs.
 *
 * The table is the content of keto_relation_tuples in the reference ORDER BY
 *   nid, namespace_id, object, relation, subject_id, subject_set_namespace_id,
 *   subject_set_object, subject_set_relation, commit_time
 * (internal/persistence/sql/relationtuples.go:250), with strings interned to ids whose
 * numeric order equals byte order (BINARY collation).  Pages are emulated exactly:
 * LIMIT page_size OFFSET (page-1)*page_size, TotalPages = ceil(count/page_size)
 * (relationtuples.go:249-265, persister.go:106-134).
 *
 * Followed reference lines (relative to /root/reference):
 *   check   internal/check/engine.go:36-80 (subjectIsAllowed), :82-114 (checkOneIndirectionFurther),
 *           :116-123 (SubjectIsAllowed, depth clamp)
 *   expand  internal/expand/engine.go:33-102 (BuildTree)
 *   visited internal/x/graph/graph_utils.go:13-35 (CheckAndAddVisited; fresh map when ctx has none)
 *   where   internal/persistence/sql/relationtuples.go:178-198 (empty field = no filter)
 *   rows    internal/persistence/sql/relationtuples.go:43-80 (toInternal: unknown ns id -> NotFound)
 *   ns      internal/driver/config/namespace_memory.go:30-48 (linear scan, first match)
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORA_ANY_NS INT64_MIN

typedef struct {
    uint64_t n;               /* tuples in ORDER BY order */
    const int32_t* ns;        /* namespace_id */
    const uint32_t* obj;      /* interned object */
    const uint32_t* rel;      /* interned relation */
    const uint8_t* kind;      /* 0 = subject_id, 1 = subject set */
    const uint32_t* sid;      /* interned subject_id (kind 0) */
    const int32_t* sns;       /* subject_set_namespace_id (kind 1) */
    const uint32_t* sobj;     /* interned subject_set_object (kind 1) */
    const uint32_t* srel;     /* interned subject_set_relation (kind 1) */
    const uint32_t* key;      /* interned Subject.String() of the tuple's subject */
    uint32_t n_ns;            /* configured namespaces, config order */
    const int32_t* ns_ids;
    const uint32_t* ns_name;  /* interned namespace name */
    uint32_t empty_str;       /* id of "" in the object/relation/name string space */
    uint32_t page_size;
} ora_table;

typedef struct {              /* a RelationQuery after whereQuery: ANY = no filter */
    int64_t ns;               /* resolved namespace id or ORA_ANY_NS */
    uint32_t obj, rel;        /* string ids; empty_str = no filter */
} ora_query;

typedef struct {              /* a typed Subject */
    uint8_t kind;             /* 0 id, 1 set */
    uint32_t sid;             /* kind 0 */
    uint32_t name, obj, rel;  /* kind 1: namespace NAME id (typed equality compares names) */
    uint32_t key;             /* interned String() */
} ora_subject;

typedef struct {
    ora_query q;              /* the request tuple's (namespace, object, relation) */
    int32_t q_ns_unknown;     /* request namespace name not configured -> NotFound -> false */
    ora_subject t;            /* requested subject */
    int32_t max_depth;        /* request max-depth */
} ora_check_req;

/* ------------------------------------------------------------------ namespaces */
static int ns_by_id(const ora_table* t, int32_t id) {        /* GetNamespaceByConfigID */
    for (uint32_t i = 0; i < t->n_ns; ++i)
        if (t->ns_ids[i] == id) return (int)i;
    return -1;
}
static int ns_by_name(const ora_table* t, uint32_t name) {   /* GetNamespaceByName */
    for (uint32_t i = 0; i < t->n_ns; ++i)
        if (t->ns_name[i] == name) return (int)i;
    return -1;
}

/* ------------------------------------------------------------------ visited map */
typedef struct vmap {
    uint32_t* slot;   /* key+1, 0 = empty */
    uint32_t cap, n;
} vmap;

static void vm_init(vmap* m) { m->cap = 64; m->n = 0; m->slot = (uint32_t*)calloc(m->cap, 4); }
static void vm_free(vmap* m) { free(m->slot); m->slot = NULL; }
static uint32_t vm_h(uint32_t k) { k ^= k >> 16; k *= 0x7feb352dU; k ^= k >> 15; k *= 0x846ca68bU; k ^= k >> 16; return k; }
static int vm_insert_raw(uint32_t* s, uint32_t cap, uint32_t k) {
    uint32_t i = vm_h(k) & (cap - 1);
    for (;;) {
        if (s[i] == 0) { s[i] = k + 1; return 1; }
        if (s[i] == k + 1) return 0;
        i = (i + 1) & (cap - 1);
    }
}
/* returns 1 if k was already present; otherwise inserts it and returns 0 */
static int vm_test_and_add(vmap* m, uint32_t k) {
    if ((m->n + 1) * 2 > m->cap) {
        uint32_t nc = m->cap * 2; uint32_t* ns = (uint32_t*)calloc(nc, 4);
        for (uint32_t i = 0; i < m->cap; ++i) if (m->slot[i]) vm_insert_raw(ns, nc, m->slot[i] - 1);
        free(m->slot); m->slot = ns; m->cap = nc;
    }
    if (vm_insert_raw(m->slot, m->cap, k)) { m->n++; return 0; }
    return 1;
}

/* ------------------------------------------------------------------ pages */
static int match(const ora_table* t, const ora_query* q, uint64_t i) {
    if (q->ns != ORA_ANY_NS && (int64_t)t->ns[i] != q->ns) return 0;
    if (q->obj != t->empty_str && t->obj[i] != q->obj) return 0;
    if (q->rel != t->empty_str && t->rel[i] != q->rel) return 0;
    return 1;
}
static int cmp_row(const ora_table* t, uint64_t i, int64_t ns, uint32_t obj, uint32_t rel) {
    if ((int64_t)t->ns[i] != ns) return (int64_t)t->ns[i] < ns ? -1 : 1;
    if (t->obj[i] != obj) return t->obj[i] < obj ? -1 : 1;
    if (t->rel[i] != rel) return t->rel[i] < rel ? -1 : 1;
    return 0;
}

typedef struct {          /* result set of one RelationQuery: either a contiguous range or a list */
    uint64_t lo, hi;      /* contiguous [lo,hi) when list == NULL */
    uint64_t* list; uint64_t n;
} rset;

static void query_rows(const ora_table* t, const ora_query* q, rset* r) {
    r->list = NULL;
    if (q->ns != ORA_ANY_NS && q->obj != t->empty_str && q->rel != t->empty_str) {
        uint64_t a = 0, b = t->n;   /* lower bound */
        while (a < b) { uint64_t m = (a + b) / 2; if (cmp_row(t, m, q->ns, q->obj, q->rel) < 0) a = m + 1; else b = m; }
        uint64_t lo = a; b = t->n;
        while (a < b) { uint64_t m = (a + b) / 2; if (cmp_row(t, m, q->ns, q->obj, q->rel) <= 0) a = m + 1; else b = m; }
        r->lo = lo; r->hi = a; r->n = a - lo;
        return;
    }
    /* wildcard: full scan in ORDER BY order (the SQL planner's result order is the ORDER BY) */
    uint64_t cnt = 0;
    for (uint64_t i = 0; i < t->n; ++i) cnt += match(t, q, i);
    r->list = (uint64_t*)malloc((cnt ? cnt : 1) * sizeof(uint64_t)); r->n = cnt;
    cnt = 0;
    for (uint64_t i = 0; i < t->n; ++i) if (match(t, q, i)) r->list[cnt++] = i;
}
static uint64_t rs_at(const rset* r, uint64_t k) { return r->list ? r->list[k] : r->lo + k; }
static void rs_free(rset* r) { free(r->list); r->list = NULL; }

/* toInternal for one row: 0 ok, -1 NotFound (relationtuples.go:48,64-71) */
static int row_ok(const ora_table* t, uint64_t i) {
    if (ns_by_id(t, t->ns[i]) < 0) return -1;
    if (t->kind[i] == 1 && ns_by_id(t, t->sns[i]) < 0) return -1;
    return 0;
}
/* fetch page (1-based): returns -1 on NotFound; sets [*b,*e) offsets into rs and *last */
static int get_page(const ora_table* t, const rset* r, uint64_t page, uint64_t* b, uint64_t* e, int* last) {
    uint64_t ps = t->page_size;
    uint64_t total_pages = (r->n + ps - 1) / ps;
    *b = (page - 1) * ps; if (*b > r->n) *b = r->n;
    *e = *b + ps; if (*e > r->n) *e = r->n;
    for (uint64_t k = *b; k < *e; ++k) if (row_ok(t, rs_at(r, k)) < 0) return -1;
    *last = page >= total_pages;
    return 0;
}

/* the subject of tuple i as a typed subject */
static void subject_of(const ora_table* t, uint64_t i, ora_subject* s) {
    s->kind = t->kind[i]; s->key = t->key[i];
    if (s->kind == 0) { s->sid = t->sid[i]; s->name = s->obj = s->rel = 0; return; }
    int k = ns_by_id(t, t->sns[i]);
    s->sid = 0; s->name = t->ns_name[k]; s->obj = t->sobj[i]; s->rel = t->srel[i];
}
static int subj_equals(const ora_subject* a, const ora_subject* b) {   /* definitions.go:252-266 */
    if (a->kind != b->kind) return 0;
    if (a->kind == 0) return a->sid == b->sid;
    return a->name == b->name && a->obj == b->obj && a->rel == b->rel;
}
/* RelationQuery{Namespace: s.Namespace, Object: s.Object, Relation: s.Relation} through whereQuery;
 * returns -1 when the namespace name is unknown (NotFound) */
static int set_query(const ora_table* t, const ora_subject* s, ora_query* q) {
    q->obj = s->obj; q->rel = s->rel;
    if (s->name == t->empty_str) { q->ns = ORA_ANY_NS; return 0; }
    int k = ns_by_name(t, s->name);
    if (k < 0) return -1;
    q->ns = t->ns_ids[k];
    return 0;
}

/* ------------------------------------------------------------------ check */
static int further(const ora_table* t, const ora_subject* T, const ora_query* q, int rest, vmap* V);

static int subject_is_allowed(const ora_table* t, const ora_subject* T, const rset* r, uint64_t b, uint64_t e,
                              int rest, vmap* V) {                   /* engine.go:36-80 */
    for (uint64_t k = b; k < e; ++k) {
        uint64_t i = rs_at(r, k);
        ora_subject s; subject_of(t, i, &s);
        vmap fresh; vmap* Vi = V;
        if (V == NULL) { vm_init(&fresh); vm_test_and_add(&fresh, s.key); Vi = &fresh; }   /* new map */
        else if (vm_test_and_add(V, s.key)) continue;                                       /* seen */
        int res = 0;
        if (subj_equals(T, &s)) res = 1;
        else if (s.kind == 1) {
            ora_query q2;
            if (set_query(t, &s, &q2) == 0) res = further(t, T, &q2, rest - 1, Vi);
            /* an unknown namespace name surfaces as NotFound in the nested call -> false */
        }
        if (V == NULL) vm_free(&fresh);
        if (res) return 1;
    }
    return 0;
}

static int further(const ora_table* t, const ora_subject* T, const ora_query* q, int rest, vmap* V) {
    if (rest <= 0) return 0;                                           /* engine.go:88-91 */
    rset r; query_rows(t, q, &r);
    int res = 0;
    for (uint64_t page = 1;; ++page) {                                 /* engine.go:96-113 */
        uint64_t b, e; int last;
        if (get_page(t, &r, page, &b, &e, &last) < 0) { res = 0; break; }   /* ErrNotFound -> false */
        res = subject_is_allowed(t, T, &r, b, e, rest, V);
        if (res || last) break;
    }
    rs_free(&r);
    return res;
}

int ora_check(const ora_table* t, const ora_check_req* rq, int32_t global_max_depth) {
    int d = rq->max_depth;                                              /* engine.go:118-120 */
    if (d <= 0 || global_max_depth < d) d = global_max_depth;
    if (rq->q_ns_unknown) return 0;                                     /* whereQuery NotFound -> false */
    return further(t, &rq->t, &rq->q, d, NULL);
}

typedef struct {
    const ora_table* t; const ora_check_req* rq; uint64_t n; int32_t g; uint8_t* out;
    uint64_t* next; pthread_mutex_t* mu;
} job;

static void* worker(void* p) {
    job* j = (job*)p;
    for (;;) {
        pthread_mutex_lock(j->mu);
        uint64_t s = *j->next; *j->next += 64;
        pthread_mutex_unlock(j->mu);
        if (s >= j->n) break;
        uint64_t e = s + 64 < j->n ? s + 64 : j->n;
        for (uint64_t i = s; i < e; ++i) j->out[i] = (uint8_t)ora_check(j->t, &j->rq[i], j->g);
    }
    return NULL;
}

/* batch of independent checks on n_threads host threads (the cpu_baseline leg) */
int ora_check_batch(const ora_table* t, const ora_check_req* rq, uint64_t n, int32_t g, uint8_t* out, int n_threads) {
    if (n_threads < 1) n_threads = 1;
    pthread_t th[256]; job jb; uint64_t next = 0; pthread_mutex_t mu; pthread_mutex_init(&mu, NULL);
    jb.t = t; jb.rq = rq; jb.n = n; jb.g = g; jb.out = out; jb.next = &next; jb.mu = &mu;
    if (n_threads > 256) n_threads = 256;
    for (int i = 0; i < n_threads; ++i) pthread_create(&th[i], NULL, worker, &jb);
    for (int i = 0; i < n_threads; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&mu);
    return 0;
}

/* ------------------------------------------------------------------ BFS-count mode (measurement)
 * Algorithmic bytes of one check as SURVEY.md section 8(d) defines them:
 *   B_check(q) = 12 + 2 + sum over rows r in Rows(q) of (8 + 4 deg(r))
 * Rows(q) = the distinct subject-set rows at BFS levels 0 .. L(q)-1 from the request row (one
 * visited set per request), L(q) = the BFS level of the first tuple equal to the requested subject
 * (1 .. D), or D if there is none.  deg(r) = tuples in the row.  This is the traffic of a CSR scan
 * that reads each row it expands in full; bench.py prices its roofline with it. */
uint64_t ora_bfs_bytes(const ora_table* t, const ora_check_req* rq, int32_t global_max_depth) {
    int d = rq->max_depth;
    if (d <= 0 || global_max_depth < d) d = global_max_depth;
    uint64_t bytes = 14;
    if (rq->q_ns_unknown) return bytes;
    vmap V; vm_init(&V);
    ora_query* cur = (ora_query*)malloc(sizeof(ora_query)); uint64_t nc = 1, capc = 1;
    cur[0] = rq->q;
    ora_query* nxt = NULL; uint64_t nn = 0, capn = 0;
    for (int level = 0; level < d && nc > 0; ++level) {
        int hit = 0;
        nn = 0;
        for (uint64_t x = 0; x < nc; ++x) {
            rset r; query_rows(t, &cur[x], &r);
            bytes += 8 + 4 * r.n;
            for (uint64_t k = 0; k < r.n; ++k) {
                ora_subject s; subject_of(t, rs_at(&r, k), &s);
                if (subj_equals(&rq->t, &s)) hit = 1;
                if (s.kind == 1 && !vm_test_and_add(&V, s.key)) {
                    ora_query q2;
                    if (set_query(t, &s, &q2) == 0) {
                        if (nn == capn) { capn = capn ? 2 * capn : 16; nxt = (ora_query*)realloc(nxt, capn * sizeof(ora_query)); }
                        nxt[nn++] = q2;
                    }
                }
            }
            rs_free(&r);
        }
        if (hit) break;                                   /* L(q) = level + 1: rows 0 .. level counted */
        ora_query* tq = cur; cur = nxt; nxt = tq;
        uint64_t tc = capc; capc = capn; capn = tc;
        nc = nn;
    }
    free(cur); free(nxt); vm_free(&V);
    return bytes;
}

typedef struct {
    const ora_table* t; const ora_check_req* rq; uint64_t n; int32_t g; uint64_t* out;
    uint64_t* next; pthread_mutex_t* mu;
} bjob;

static void* bworker(void* p) {
    bjob* j = (bjob*)p;
    for (;;) {
        pthread_mutex_lock(j->mu);
        uint64_t s = *j->next; *j->next += 64;
        pthread_mutex_unlock(j->mu);
        if (s >= j->n) break;
        uint64_t e = s + 64 < j->n ? s + 64 : j->n;
        for (uint64_t i = s; i < e; ++i) j->out[i] = ora_bfs_bytes(j->t, &j->rq[i], j->g);
    }
    return NULL;
}

int ora_bfs_bytes_batch(const ora_table* t, const ora_check_req* rq, uint64_t n, int32_t g, uint64_t* out, int n_threads) {
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256]; bjob jb; uint64_t next = 0; pthread_mutex_t mu; pthread_mutex_init(&mu, NULL);
    jb.t = t; jb.rq = rq; jb.n = n; jb.g = g; jb.out = out; jb.next = &next; jb.mu = &mu;
    for (int i = 0; i < n_threads; ++i) pthread_create(&th[i], NULL, bworker, &jb);
    for (int i = 0; i < n_threads; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&mu);
    return 0;
}

/* ------------------------------------------------------------------ expand */
typedef struct {                 /* pre-order tree node */
    uint8_t type;                /* 0 union, 1 leaf */
    uint8_t kind;                /* subject kind */
    uint32_t sid, name, obj, rel;
    uint32_t n_children;
} ora_node;

typedef struct { ora_node* v; uint64_t n, cap; } nbuf;
static uint64_t nb_push(nbuf* b, const ora_node* x) {
    if (b->n == b->cap) { b->cap = b->cap ? b->cap * 2 : 64; b->v = (ora_node*)realloc(b->v, b->cap * sizeof(ora_node)); }
    b->v[b->n] = *x; return b->n++;
}
static void leaf_of(const ora_subject* s, ora_node* n) {
    n->type = 1; n->kind = s->kind; n->sid = s->sid; n->name = s->name; n->obj = s->obj; n->rel = s->rel; n->n_children = 0;
}

/* returns 1 = node written, 0 = nil, -1 = error (NotFound propagates: engine.go:63-66) */
static int build(const ora_table* t, const ora_subject* s, int rest, vmap** V, nbuf* out) {
    if (s->kind == 0) { ora_node n; leaf_of(s, &n); nb_push(out, &n); return 1; }   /* :97-101 */
    if (*V == NULL) { *V = (vmap*)malloc(sizeof(vmap)); vm_init(*V); vm_test_and_add(*V, s->key); }
    else if (vm_test_and_add(*V, s->key)) return 0;                                  /* :40-43 */
    ora_query q;
    if (set_query(t, s, &q) < 0) return -1;
    rset r; query_rows(t, &q, &r);
    ora_node self; leaf_of(s, &self); self.type = 0;
    uint64_t at = (uint64_t)-1;
    int res = 1;
    for (uint64_t page = 1;; ++page) {                                               /* :55-92 */
        uint64_t b, e; int last;
        if (get_page(t, &r, page, &b, &e, &last) < 0) { res = -1; break; }
        if (e == b) { res = 0; break; }                                              /* :68-70 */
        if (rest <= 1) {                                                             /* :72-75 */
            if (at == (uint64_t)-1) { self.type = 1; nb_push(out, &self); }
            else out->v[at].type = 1;
            res = 1; break;
        }
        if (at == (uint64_t)-1) at = nb_push(out, &self);
        for (uint64_t k = b; k < e; ++k) {
            ora_subject c; subject_of(t, rs_at(&r, k), &c);
            int cr = build(t, &c, rest - 1, V, out);
            if (cr < 0) { res = -1; break; }
            if (cr == 0) { ora_node n; leaf_of(&c, &n); nb_push(out, &n); }
            out->v[at].n_children++;
        }
        if (res < 0 || last) break;
    }
    rs_free(&r);
    return res;
}

/* BuildTree(root, max_depth): returns 1 tree, 0 nil, -1 error; *nodes is malloc'd (free with ora_free) */
int ora_expand(const ora_table* t, const ora_subject* root, int32_t max_depth, int32_t global_max_depth,
               ora_node** nodes, uint64_t* n_nodes) {
    int d = max_depth;                                                               /* :35-37 */
    if (d <= 0 || global_max_depth < d) d = global_max_depth;
    nbuf b = {0, 0, 0};
    vmap* V = NULL;
    int r = build(t, root, d, &V, &b);
    if (V) { vm_free(V); free(V); }
    if (r != 1) { free(b.v); b.v = NULL; b.n = 0; }
    *nodes = b.v; *n_nodes = b.n;
    return r;
}

void ora_free(void* p) { free(p); }
