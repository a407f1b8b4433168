/* Study (dev tool, not product): on a synthetic CSR graph, how many check requests can be decided
 * "false" by a hop-bounded reachability test, and how much DFS work the rest still needs.
 *
 * A request (R, T, D) can only be allowed if some row holding the subject id T is entered by the
 * reference DFS (internal/check/engine.go:36-114), and every entered row lies within D - 1 set hops
 * of R.  So "no row holding T within D - 1 hops of R" proves the decision false.  This tool runs,
 * per request: the reference DFS (rows entered, decision) and a bidirectional BFS (forward from R
 * over set edges, backward from the rows holding T over reversed set edges) for that bound.
 *
 * Edges: bit 31 set = subject set (row index in the low bits), else a subject id.
 * Build: gcc -O2 -fopenmp -shared -fPIC -o tools/dev/libbidir_study.so tools/dev/bidir_study.c
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint32_t row, target, flags;
    int32_t max_depth;
} req_t;

typedef struct {
    uint64_t dfs_steps;    /* set edges walked + rows entered */
    uint32_t dfs_rows;     /* rows entered */
    uint8_t allowed;
    uint8_t within;        /* a row holding T lies within D - 1 hops */
    uint32_t bidir_work;   /* rows + edges touched by the bidirectional search */
    uint64_t par_steps;    /* top-level items in parallel, each pre-tested: steps until decided */
    uint64_t par_nocancel; /* the same without cancelling an allowed request's other items */
    uint64_t worst_item;   /* longest kept item */
    uint8_t worst_hit;
    uint64_t par_work;     /* steps of the items that pass their pre-test */
    uint32_t n_items, n_items_within;
} res_t;

typedef struct {
    uint64_t n_rows;
    const uint64_t* ptr;
    const uint32_t* e;
    uint64_t* rptr;        /* reverse set edges */
    uint32_t* rsrc;
    uint64_t* pptr;        /* postings: id -> rows holding it */
    uint32_t* prow;
    uint32_t n_ids;
} graph_t;

static graph_t G;
static uint32_t work_cap = 1u << 26;
void bs_cap(uint32_t c) { work_cap = c; }

static uint32_t n_sets(uint64_t r) {
    uint64_t b = G.ptr[r], e = G.ptr[r + 1], k = b;
    while (k < e && (G.e[k] & 0x80000000u)) ++k;
    return (uint32_t)(k - b);
}

int bs_init(uint64_t n_rows, const uint64_t* ptr, const uint32_t* e, uint32_t n_ids) {
    G.n_rows = n_rows;
    G.ptr = ptr;
    G.e = e;
    G.n_ids = n_ids;
    G.rptr = calloc(n_rows + 2, 8);
    G.pptr = calloc((uint64_t)n_ids + 2, 8);
    if (!G.rptr || !G.pptr) return -1;
    for (uint64_t r = 0; r < n_rows; ++r)
        for (uint64_t k = ptr[r]; k < ptr[r + 1]; ++k) {
            if (e[k] & 0x80000000u) G.rptr[(e[k] & 0x7FFFFFFFu) + 1]++;
            else G.pptr[e[k] + 1]++;
        }
    for (uint64_t r = 0; r < n_rows; ++r) G.rptr[r + 1] += G.rptr[r];
    for (uint64_t i = 0; i < n_ids; ++i) G.pptr[i + 1] += G.pptr[i];
    G.rsrc = malloc((G.rptr[n_rows] + 1) * 4);
    G.prow = malloc((G.pptr[n_ids] + 1) * 4);
    uint64_t* rc = malloc((n_rows + 1) * 8);
    uint64_t* pc = malloc(((uint64_t)n_ids + 1) * 8);
    if (!G.rsrc || !G.prow || !rc || !pc) return -1;
    memcpy(rc, G.rptr, n_rows * 8);
    memcpy(pc, G.pptr, (uint64_t)n_ids * 8);
    for (uint64_t r = 0; r < n_rows; ++r)
        for (uint64_t k = ptr[r]; k < ptr[r + 1]; ++k) {
            if (e[k] & 0x80000000u) G.rsrc[rc[e[k] & 0x7FFFFFFFu]++] = (uint32_t)r;
            else {
                uint64_t* c = &pc[e[k]];
                if (*c == G.pptr[e[k]] || G.prow[*c - 1] != (uint32_t)r) G.prow[(*c)++] = (uint32_t)r;
            }
        }
    /* duplicate ids in one row were skipped; close the gaps by keeping counts in pc */
    for (uint64_t i = 0; i < n_ids; ++i) G.pptr[i] = G.pptr[i] | ((pc[i] - G.pptr[i]) << 40);
    free(rc);
    free(pc);
    return 0;
}

static void post(uint32_t id, uint64_t* b, uint64_t* n) {
    *b = G.pptr[id] & ((1ull << 40) - 1);
    *n = G.pptr[id] >> 40;
}

typedef struct {
    uint32_t* mark;        /* per row: epoch << 1 | side (bidir), epoch for dfs visited */
    uint32_t* dmark;
    uint32_t epoch;
    uint32_t* qa;          /* frontiers */
    uint32_t* qb;
    uint32_t* qn;
    uint64_t* stk;
} scratch_t;

/* the reference DFS for an id request (no collisions, no overlays) */
static int within(scratch_t* s, uint32_t R, uint32_t T, int L, uint32_t* work);
/* one top-level item: a fresh map, the DFS from child c at remaining depth k */
static uint64_t item_dfs(scratch_t* s, uint32_t c, uint32_t T, int k0, int* hit) {
    uint64_t steps = 1, sp = 0;
    uint32_t ep = ++s->epoch;
    uint32_t* ks = (uint32_t*)(s->stk + (1u << 16));
    *hit = 0;
    s->dmark[c] = ep;
    if (k0 < 1) return steps;
    s->stk[sp++] = ((uint64_t)c << 32);
    ks[0] = (uint32_t)k0;
    ++steps;
    {
        uint32_t nc = n_sets(c);
        for (uint64_t k = G.ptr[c] + nc; k < G.ptr[c + 1]; ++k)
            if (G.e[k] == T) { *hit = 1; return steps; }
    }
    while (sp) {
        uint64_t top = s->stk[sp - 1];
        uint32_t r = (uint32_t)(top >> 32), j = (uint32_t)top;
        uint32_t nr = n_sets(r);
        if (j >= nr) { --sp; ++steps; continue; }
        s->stk[sp - 1] = ((uint64_t)r << 32) | (j + 1);
        uint32_t ch = G.e[G.ptr[r] + j] & 0x7FFFFFFFu;
        ++steps;
        if (s->dmark[ch] == ep) continue;
        s->dmark[ch] = ep;
        uint32_t k = ks[sp - 1];
        if (k < 2) continue;
        ks[sp] = k - 1;
        s->stk[sp++] = ((uint64_t)ch << 32);
        uint32_t nc = n_sets(ch);
        for (uint64_t q = G.ptr[ch] + nc; q < G.ptr[ch + 1]; ++q)
            if (G.e[q] == T) { *hit = 1; return steps; }
    }
    return steps;
}

static void par_items(scratch_t* s, uint32_t R, uint32_t T, int D, res_t* o) {
    uint32_t ns = n_sets(R);
    o->n_items = ns;
    o->n_items_within = 0;
    o->par_steps = 1;
    o->par_work = 1;
    for (uint64_t k = G.ptr[R] + ns; k < G.ptr[R + 1]; ++k)
        if (G.e[k] == T) return;
    uint64_t best_hit = ~0ull, worst = 0;
    for (uint32_t i = 0; i < ns; ++i) {
        uint32_t c = G.e[G.ptr[R] + i] & 0x7FFFFFFFu;
        uint32_t wk;
        if (D < 2 || !within(s, c, T, D - 2, &wk)) continue;
        o->n_items_within++;
        int hit;
        uint64_t st = item_dfs(s, c, T, D - 1, &hit);
        o->par_work += st;
        if (hit && st < best_hit) best_hit = st;
        if (st > worst) { worst = st; o->worst_hit = (uint8_t)hit; }
    }
    o->par_steps += best_hit != ~0ull ? best_hit : worst;
    o->par_nocancel = 1 + worst;
    o->worst_item = worst;
}

static uint64_t dfs(scratch_t* s, uint32_t R, uint32_t T, int D, uint32_t* rows, uint8_t* allowed) {
    uint64_t steps = 0;
    *rows = 0;
    *allowed = 0;
    /* entering R (k = D) */
    uint32_t ep = ++s->epoch;
    /* stack of (row, position, k) */
    uint64_t sp = 0;
    uint32_t ns = n_sets(R);
    ++*rows;
    ++steps;
    for (uint64_t k = G.ptr[R] + ns; k < G.ptr[R + 1]; ++k)
        if (G.e[k] == T) { *allowed = 1; return steps; }
    /* top level: a fresh map per top-level tuple */
    for (uint32_t i = 0; i < ns; ++i) {
        uint32_t c = G.e[G.ptr[R] + i] & 0x7FFFFFFFu;
        ep = ++s->epoch;
        ++steps;
        s->dmark[c] = ep;
        if (D < 2) continue;
        /* enter c with k = D - 1 */
        sp = 0;
        s->stk[sp++] = ((uint64_t)c << 32) | 0;   /* row, next set index */
        uint32_t* ks = (uint32_t*)(s->stk + (1u << 16));
        ks[0] = (uint32_t)(D - 1);
        ++*rows;
        ++steps;
        {
            uint32_t nc = n_sets(c);
            for (uint64_t k = G.ptr[c] + nc; k < G.ptr[c + 1]; ++k)
                if (G.e[k] == T) { *allowed = 1; return steps; }
        }
        while (sp) {
            uint64_t top = s->stk[sp - 1];
            uint32_t r = (uint32_t)(top >> 32), j = (uint32_t)top;
            uint32_t nr = n_sets(r);
            if (j >= nr) { --sp; ++steps; continue; }
            s->stk[sp - 1] = ((uint64_t)r << 32) | (j + 1);
            uint32_t ch = G.e[G.ptr[r] + j] & 0x7FFFFFFFu;
            ++steps;
            if (s->dmark[ch] == ep) continue;
            s->dmark[ch] = ep;
            uint32_t k = ks[sp - 1];
            if (k < 2) continue;
            ks[sp] = k - 1;
            s->stk[sp++] = ((uint64_t)ch << 32) | 0;
            ++*rows;
            uint32_t nc = n_sets(ch);
            for (uint64_t q = G.ptr[ch] + nc; q < G.ptr[ch + 1]; ++q)
                if (G.e[q] == T) { *allowed = 1; return steps; }
        }
    }
    return steps;
}

/* is some row holding T within L hops of R?  bidirectional BFS, expanding the smaller side */
static int within(scratch_t* s, uint32_t R, uint32_t T, int L, uint32_t* work) {
    uint64_t pb, pn;
    post(T, &pb, &pn);
    *work = 0;
    if (pn == 0 || L < 0) return 0;
    uint32_t ep = ++s->epoch;
    uint32_t fa = ep * 2u, fb = ep * 2u + 1u;   /* side tags in mark */
    uint32_t *A = s->qa, *B = s->qb, *Q = s->qn, na = 0, nb = 0;
    s->mark[R] = fa;
    A[na++] = R;
    for (uint64_t i = 0; i < pn; ++i) {
        uint32_t r = G.prow[pb + i];
        if (r == R) return 1;
        if (s->mark[r] != fb) { s->mark[r] = fb; B[nb++] = r; }
    }
    *work += (uint32_t)pn + 1;
    int da = 0, db = 0;
    while (da + db < L && na && nb) {
        uint32_t nn = 0;
        if (na <= nb) {
            for (uint32_t i = 0; i < na; ++i) {
                uint32_t r = A[i];
                uint32_t ns = n_sets(r);
                *work += 1 + ns;
                for (uint32_t j = 0; j < ns; ++j) {
                    uint32_t c = G.e[G.ptr[r] + j] & 0x7FFFFFFFu;
                    if (s->mark[c] == fb) return 1;
                    if (s->mark[c] != fa) { s->mark[c] = fa; Q[nn++] = c; }
                }
            }
            uint32_t* t = A; A = Q; Q = t; na = nn; ++da;
        } else {
            for (uint32_t i = 0; i < nb; ++i) {
                uint32_t r = B[i];
                *work += 1 + (uint32_t)(G.rptr[r + 1] - G.rptr[r]);
                for (uint64_t k = G.rptr[r]; k < G.rptr[r + 1]; ++k) {
                    uint32_t c = G.rsrc[k];
                    if (s->mark[c] == fa) return 1;
                    if (s->mark[c] != fb) { s->mark[c] = fb; Q[nn++] = c; }
                }
            }
            uint32_t* t = B; B = Q; Q = t; nb = nn; ++db;
        }
        if (*work > work_cap) return 1;   /* give up: treat as reachable */
    }
    return 0;
}

int bs_run(const req_t* q, uint64_t n, int gmd, res_t* out, int threads) {
#pragma omp parallel num_threads(threads)
    {
        scratch_t s;
        s.mark = calloc(G.n_rows, 4);
        s.dmark = calloc(G.n_rows, 4);
        s.epoch = 0;
        s.qa = malloc(G.n_rows * 4);
        s.qb = malloc(G.n_rows * 4);
        s.qn = malloc(G.n_rows * 4);
        s.stk = malloc((1u << 17) * 8);
#pragma omp for schedule(dynamic, 64)
        for (uint64_t i = 0; i < n; ++i) {
            int d = q[i].max_depth;
            if (d <= 0 || gmd < d) d = gmd;
            res_t* o = &out[i];
            o->dfs_steps = dfs(&s, q[i].row, q[i].target, d, &o->dfs_rows, &o->allowed);
            if (s.epoch > 0x7FFFFF00u) { memset(s.mark, 0, G.n_rows * 4); memset(s.dmark, 0, G.n_rows * 4); s.epoch = 0; }
            o->within = (uint8_t)within(&s, q[i].row, q[i].target, d - 1, &o->bidir_work);
            par_items(&s, q[i].row, q[i].target, d, o);
        }
        free(s.mark); free(s.dmark); free(s.qa); free(s.qb); free(s.qn); free(s.stk);
    }
    return 0;
}
