/*
 * keto_consumer.c -- a plain C consumer of include/keto_mi355x.h, written against the header only.
 *
 * It makes the calls, in the order, the Go integration makes (integration/go/internal/gpu/gpu.go,
 * batcher.go; internal/driver/registry_gpu.go): build a snapshot from the keto_relation_tuples rows
 * (strings, commit order), check batches and expand batches as the micro-batchers flush them, trees
 * rebuilt from the node arena and keto_subject_fields (what gpu.ExpandBatch hands internal/expand),
 * write transactions applied after they commit (keto_snapshot_apply) and, when the library answers
 * KETO_E_REBUILD, a rebuild from the table the consumer keeps, as the registry's persister wrapper
 * does.  tests/test_consumer_c.py compiles it with gcc against the header and runs it: host-only
 * (device -1: compute must fail with KETO_E_HIP) on the CPU, and on the GPU the reference's golden
 * cases (tests/golden/reference_cases.json) and seeded write / check / expand sequences compared with
 * the SQL oracle.  Every check batch also goes through keto_check_batch_packed (the Go shim's call),
 * once alone and then from four threads at once, three times each (the batcher keeps batches in
 * flight per engine, KETO_GPU_INFLIGHT): decisions and statuses must equal keto_check_batch's.
 *
 * Several GPUs in the one server process (registry_gpu.go EnableGPU over a device list): with an
 * "R" line the consumer keeps one replica per listed device -- the first built from the table, the
 * others made by keto_snapshot_clone -- deals its check and expand batches over them round-robin,
 * applies every write transaction to each replica, and rebuilds them all when one answers
 * KETO_E_REBUILD.
 *
 * A graph partitioned over the server's GPUs ("Q" line, registry_gpu.go when the replicated arena does
 * not fit a device): the table is built once host-only, cloned host-only per part, and each clone is
 * uploaded as one shared-rows part (keto_snapshot_upload_part_mode, KETO_PART_SHARED) on its device;
 * one keto_comm_init_local rank per part, each driven by its own thread.  A check batch is split over
 * the ranks and every rank calls keto_check_batch_routed with its slice (an empty slice too), then
 * keto_check_batch_routed_packed with the slice packed (the Go Partition's call; both must agree); an
 * expand batch the same way through keto_expand_batch_routed; every write transaction is applied to
 * every part.  A restart in this mode builds a host-only snapshot from the table, saves it, loads the
 * file host-only and partitions it again (the Go server's persisted-file path).
 *
 * A restart ("S" line): the server saves the first replica (keto_snapshot_save, tagged with its
 * version), releases every replica, loads the file back onto the first device (keto_snapshot_load)
 * and clones it to the others, as registry_gpu.go's loadFile does when the table has not changed.
 *
 * Input (tab-separated lines; empty fields allowed), executed in order:
 *   P <page_size>        V <device>        R <device> <device> ...   (replicas; default: V's device)
 *   Q <device> <device> ...   (instead of replicas: one shared-rows part per listed device)
 *   N <ns id> <name>
 *   T <ns id> <object> <relation> I <subject id>                          (a row of the initial table)
 *   T <ns id> <object> <relation> S <set ns id> <set object> <set relation>
 *   C <ns> <object> <relation> I <subject id> <max depth> <global max depth>
 *   C <ns> <object> <relation> S <set ns> <set object> <set relation> <max depth> <global max depth>
 *   E I <subject id> <max depth> <global max depth>
 *   E S <ns> <object> <relation> <max depth> <global max depth>
 *   A+ <tuple as after T>   A- <tuple as after T>   A!   (one write transaction: inserts, deletes, commit)
 *   S <path>             (restart from a persisted snapshot)
 * Consecutive C lines with one global max depth form one keto_check_batch; consecutive E lines one
 * keto_expand_batch.  Output (tab-separated): "check <i> <allowed> <status>",
 * "expand <i> <status> <json|null|error> <proto hex|->", "apply <rc> <version> <rebuilt>", "stats ...",
 * "restart <version> <tag>", "nodevice <rc>", "done".
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "keto_mi355x.h"

#define MAXF 12

typedef struct {
    char* f[MAXF];
    int n;
} line_t;

static char* dupn(const char* s, size_t n) {
    char* p = (char*)malloc(n + 1);
    if (!p) exit(3);
    memcpy(p, s, n);
    p[n] = 0;
    return p;
}

static int split(char* s, line_t* l) {
    l->n = 0;
    size_t len = strlen(s);
    while (len && (s[len - 1] == '\n' || s[len - 1] == '\r')) s[--len] = 0;
    char* p = s;
    for (;;) {
        char* t = strchr(p, '\t');
        if (l->n == MAXF) return -1;
        l->f[l->n++] = t ? dupn(p, (size_t)(t - p)) : dupn(p, strlen(p));
        if (!t) break;
        p = t + 1;
    }
    return l->n;
}

static keto_str ks(const char* s) {
    keto_str r;
    r.p = s;
    r.n = (uint32_t)strlen(s);
    return r;
}

static void fail(const char* what, int rc) {
    fprintf(stderr, "%s failed: %d (%s)\n", what, rc, keto_last_error());
    exit(2);
}

static void* xrealloc(void* p, size_t n) {
    p = realloc(p, n ? n : 1);
    if (!p) exit(3);
    return p;
}

/* ---- the table the consumer keeps (the SQL table of the Go server): tuples in commit order */
typedef struct {
    keto_tuple* t;
    size_t n, cap;
} table_t;

static keto_tuple tuple_of(line_t* l, int k) { /* fields k..: <ns id> <obj> <rel> I <sid> | S <sns> <sobj> <srel> */
    keto_tuple t;
    memset(&t, 0, sizeof t);
    t.namespace_id = atoi(l->f[k]);
    t.object = ks(l->f[k + 1]);
    t.relation = ks(l->f[k + 2]);
    if (!strcmp(l->f[k + 3], "I")) {
        t.subject_kind = 0;
        t.subject_id = ks(l->f[k + 4]);
    } else {
        t.subject_kind = 1;
        t.set_namespace_id = atoi(l->f[k + 4]);
        t.set_object = ks(l->f[k + 5]);
        t.set_relation = ks(l->f[k + 6]);
    }
    return t;
}

static int str_eq(keto_str a, keto_str b) { return a.n == b.n && (a.n == 0 || memcmp(a.p, b.p, a.n) == 0); }

/* DeleteRelationTuples' WHERE: namespace, object, relation and subject all equal (relationtuples.go:200-223) */
static int tuple_eq(const keto_tuple* a, const keto_tuple* b) {
    if (a->namespace_id != b->namespace_id || !str_eq(a->object, b->object) || !str_eq(a->relation, b->relation) ||
        a->subject_kind != b->subject_kind)
        return 0;
    if (a->subject_kind == 0) return str_eq(a->subject_id, b->subject_id);
    return a->set_namespace_id == b->set_namespace_id && str_eq(a->set_object, b->set_object) &&
           str_eq(a->set_relation, b->set_relation);
}

static void table_insert(table_t* tb, keto_tuple t) {
    if (tb->n == tb->cap) {
        tb->cap = tb->cap ? 2 * tb->cap : 64;
        tb->t = (keto_tuple*)xrealloc(tb->t, tb->cap * sizeof(keto_tuple));
    }
    tb->t[tb->n++] = t;
}

static void table_delete(table_t* tb, const keto_tuple* d) {
    size_t w = 0;
    for (size_t i = 0; i < tb->n; ++i)
        if (!tuple_eq(&tb->t[i], d)) tb->t[w++] = tb->t[i];
    tb->n = w;
}

/* ---- protobuf of a tree rebuilt from its nodes and subject fields (Tree.ToProto + proto.Marshal,
 * internal/expand/tree.go:165-188): node_type = 1 (UNION 1, LEAF 4), subject = 2 (Subject: id = 1 |
 * set = 2 {namespace 1, object 2, relation 3, empty strings omitted}), children = 3 */
typedef struct {
    uint8_t* p;
    size_t n, cap;
} buf_t;

static void put(buf_t* b, const void* s, size_t n) {
    if (b->n + n > b->cap) {
        b->cap = (b->n + n) * 2 + 64;
        b->p = (uint8_t*)xrealloc(b->p, b->cap);
    }
    if (n) memcpy(b->p + b->n, s, n);
    b->n += n;
}
static void put_varint(buf_t* b, uint64_t v) {
    uint8_t x[10];
    int k = 0;
    while (v >= 0x80) {
        x[k++] = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    x[k++] = (uint8_t)v;
    put(b, x, (size_t)k);
}
static void put_field(buf_t* b, uint8_t tag, const char* s, size_t n) {
    put(b, &tag, 1);
    put_varint(b, n);
    put(b, s, n);
}

typedef struct {
    int set;
    const char *a, *b, *c; /* id | namespace, object, relation */
    uint32_t na, nb, nc;
} fields_t;

/* encodes the subtree at nodes[*at] into out; returns 0, or -1 on a malformed arena */
static int encode(const keto_tree_node* nodes, uint64_t n, uint64_t* at, const fields_t* f, buf_t* out, int depth) {
    if (*at >= n || depth > 4096) return -1;
    const uint64_t me = (*at)++;
    const int leaf = (nodes[me].info & 0x80000000u) != 0;
    const uint32_t nc = leaf ? 0 : nodes[me].info & 0x7FFFFFFFu;
    uint8_t tt[2] = {0x08, (uint8_t)(leaf ? 4 : 1)};
    put(out, tt, 2);
    buf_t sub = {0, 0, 0};
    const fields_t* s = &f[me];
    if (!s->set) {
        put_field(&sub, 0x0A, s->a, s->na);
    } else {
        buf_t in = {0, 0, 0};
        if (s->na) put_field(&in, 0x0A, s->a, s->na);
        if (s->nb) put_field(&in, 0x12, s->b, s->nb);
        if (s->nc) put_field(&in, 0x1A, s->c, s->nc);
        put_field(&sub, 0x12, (const char*)in.p, in.n);
        free(in.p);
    }
    put_field(out, 0x12, (const char*)sub.p, sub.n);
    free(sub.p);
    for (uint32_t c = 0; c < nc; ++c) {
        buf_t child = {0, 0, 0};
        if (encode(nodes, n, at, f, &child, depth + 1)) return -1;
        put_field(out, 0x1A, (const char*)child.p, child.n);
        free(child.p);
    }
    return 0;
}

/* tree i of arena ar through keto_tree_nodes + keto_subject_fields (size, then fill), as protobuf */
static int tree_via_fields(keto_snapshot* snap, keto_tree_arena* ar, uint32_t i, buf_t* out) {
    uint64_t n = 0;
    const keto_tree_node* nodes = keto_tree_nodes(ar, i, &n);
    if (!nodes || !n) return 0;
    uint32_t* refs = (uint32_t*)xrealloc(NULL, n * sizeof(uint32_t));
    uint32_t* lens = (uint32_t*)xrealloc(NULL, 3 * n * sizeof(uint32_t));
    for (uint64_t k = 0; k < n; ++k) refs[k] = nodes[k].subject;
    const int64_t total = keto_subject_fields(snap, ar, refs, n, NULL, 0, lens);
    if (total < 0) fail("keto_subject_fields", (int)total);
    char* text = (char*)xrealloc(NULL, (size_t)total + 1);
    if (keto_subject_fields(snap, ar, refs, n, text, (uint64_t)total, lens) != total) return -1;
    fields_t* f = (fields_t*)xrealloc(NULL, n * sizeof(fields_t));
    size_t at = 0;
    for (uint64_t k = 0; k < n; ++k) {
        f[k].set = (refs[k] & 0x80000000u) != 0;
        f[k].na = lens[3 * k];
        f[k].nb = lens[3 * k + 1];
        f[k].nc = lens[3 * k + 2];
        f[k].a = text + at;
        at += f[k].na;
        f[k].b = text + at;
        at += f[k].nb;
        f[k].c = text + at;
        at += f[k].nc;
    }
    uint64_t pos = 0;
    const int rc = encode(nodes, n, &pos, f, out, 0) || pos != n ? -1 : 0;
    free(refs);
    free(lens);
    free(text);
    free(f);
    return rc;
}

static keto_snapshot* build(const keto_namespace* ns, size_t n_ns, const table_t* tb, uint32_t page_size, int device) {
    keto_snapshot_opts opts;
    opts.page_size = page_size;
    opts.device = device;
    opts.flags = 0;
    keto_snapshot* snap = NULL;
    const int rc = keto_snapshot_build(ns, (uint32_t)n_ns, tb->t, tb->n, &opts, &snap);
    if (rc != KETO_OK) fail("keto_snapshot_build", rc);
    return snap;
}

#define MAX_REPLICAS 8

/* one replica per device: the table sorted and uploaded once, cloned to the other devices */
static void build_replicas(const keto_namespace* ns, size_t n_ns, const table_t* tb, uint32_t page_size,
                           const int* devices, int n, keto_snapshot** reps) {
    reps[0] = build(ns, n_ns, tb, page_size, devices[0]);
    for (int k = 1; k < n; ++k) {
        const int rc = keto_snapshot_clone(reps[0], devices[k], &reps[k]);
        if (rc != KETO_OK) fail("keto_snapshot_clone", rc);
    }
}

/* ---- a graph partitioned over the devices: one shared-rows part and one local rank per device */
typedef struct {
    int n;
    int devices[MAX_REPLICAS];
    keto_snapshot* parts[MAX_REPLICAS];
    keto_comm* comms[MAX_REPLICAS];
    uint8_t id[KETO_COMM_ID_BYTES];
} partition_t;

/* a check batch packed as the Go shim packs it (keto_check_batch_packed's layout): every request's
   strings back to back in *blob, one record per request */
static void pack_batch(const keto_check_req* q, size_t m, char** blob, size_t* total, keto_check_packed** pk) {
    size_t t = 0;
    for (size_t k = 0; k < m; ++k) {
        const keto_check_req* r = &q[k];
        t += r->namespace_.n + r->object.n + r->relation.n;
        t += r->subject.kind == 0 ? r->subject.id.n
                                  : r->subject.set_namespace.n + r->subject.set_object.n + r->subject.set_relation.n;
    }
    *blob = (char*)xrealloc(NULL, t ? t : 1);
    *pk = (keto_check_packed*)calloc(m ? m : 1, sizeof(keto_check_packed));
    if (!*pk) exit(3);
    size_t at = 0;
    for (size_t k = 0; k < m; ++k) {
        const keto_check_req* r = &q[k];
        keto_str f[6] = {r->namespace_, r->object, r->relation, r->subject.id, {NULL, 0}, {NULL, 0}};
        int nf = 4;
        if (r->subject.kind == 1) {
            f[3] = r->subject.set_namespace;
            f[4] = r->subject.set_object;
            f[5] = r->subject.set_relation;
            nf = 6;
        }
        (*pk)[k].off = (uint32_t)at;
        (*pk)[k].kind = r->subject.kind;
        (*pk)[k].max_depth = r->max_depth;
        for (int j = 0; j < nf; ++j) {
            (*pk)[k].len[j] = (uint16_t)f[j].n;
            if (f[j].n) memcpy(*blob + at, f[j].p, f[j].n);
            at += f[j].n;
        }
    }
    *total = t;
}

/* one rank's share of a collective call, run on its own thread */
typedef struct {
    partition_t* pt;
    int rank;
    int op;                                   /* 0 init, 1 check, 2 expand, 3 packed check */
    const keto_check_req* q;
    const char* blob;                         /* op 3: the rank's slice packed */
    size_t blob_len;
    const keto_check_packed* pk;
    const keto_expand_req* e;
    uint32_t n;
    int32_t gmd;
    uint8_t* allowed;
    uint8_t* status;
    keto_tree_arena* ar;
    int rc;
} rank_call_t;

/* one thread's packed batches (keto_check_batch_packed from several threads on one snapshot) */
#define PACKED_THREADS 4
typedef struct {
    keto_snapshot* snap;
    const char* blob;
    size_t total;
    const keto_check_packed* pk;
    uint32_t m;
    int32_t gmd;
    const uint8_t* want_allowed;
    const uint8_t* want_status;
    int bad;
} packed_call_t;

static void* packed_main(void* arg) {
    packed_call_t* c = (packed_call_t*)arg;
    uint8_t* a = (uint8_t*)malloc(c->m ? c->m : 1);
    uint8_t* st = (uint8_t*)malloc(c->m ? c->m : 1);
    if (!a || !st) exit(3);
    for (int rep = 0; rep < 3 && !c->bad; ++rep) {
        if (keto_check_batch_packed(c->snap, c->blob, c->total, c->pk, c->m, c->gmd, a, st) != KETO_OK) {
            c->bad = 1;
            break;
        }
        for (uint32_t k = 0; k < c->m; ++k)
            if (a[k] != c->want_allowed[k] || st[k] != c->want_status[k]) c->bad = 1;
    }
    free(a);
    free(st);
    return NULL;
}

static void* rank_main(void* arg) {
    rank_call_t* c = (rank_call_t*)arg;
    partition_t* pt = c->pt;
    if (c->op == 0)
        c->rc = keto_comm_init_local(pt->id, pt->n, c->rank, pt->devices[c->rank], &pt->comms[c->rank]);
    else if (c->op == 1)
        c->rc = keto_check_batch_routed(pt->comms[c->rank], pt->parts[c->rank], c->q, c->n, c->gmd, c->allowed, c->status);
    else if (c->op == 3)
        c->rc = keto_check_batch_routed_packed(pt->comms[c->rank], pt->parts[c->rank], c->blob, c->blob_len, c->pk, c->n,
                                               c->gmd, c->allowed, c->status);
    else
        c->rc = keto_expand_batch_routed(pt->comms[c->rank], pt->parts[c->rank], c->e, c->n, c->gmd, &c->ar);
    return NULL;
}

/* every rank's call at once (collective); calls[k] are filled by the caller; returns the first rc */
static int ranks_run(partition_t* pt, rank_call_t* calls) {
    pthread_t th[MAX_REPLICAS];
    for (int k = 0; k < pt->n; ++k) {
        calls[k].pt = pt;
        calls[k].rank = k;
        if (pthread_create(&th[k], NULL, rank_main, &calls[k]) != 0) exit(3);
    }
    int rc = KETO_OK;
    for (int k = 0; k < pt->n; ++k) {
        pthread_join(th[k], NULL);
        if (rc == KETO_OK) rc = calls[k].rc;
    }
    for (int k = 1; k < pt->n; ++k)
        if (calls[k].rc != calls[0].rc) return 14;       /* an error must be agreed by every rank */
    return rc;
}

/* parts from a host-only snapshot `base` (consumed: it becomes part 0), one per device, and the ranks */
static void partition_from(keto_snapshot* base, partition_t* pt) {
    static int generation = 0;
    pt->parts[0] = base;
    for (int k = 1; k < pt->n; ++k) {
        const int rc = keto_snapshot_clone(base, -1, &pt->parts[k]);
        if (rc != KETO_OK) fail("keto_snapshot_clone", rc);
    }
    for (int k = 0; k < pt->n; ++k) {
        const int rc = keto_snapshot_upload_part_mode(pt->parts[k], (uint32_t)k, (uint32_t)pt->n, pt->devices[k],
                                                      KETO_PART_SHARED);
        if (rc != KETO_OK) fail("keto_snapshot_upload_part_mode", rc);
    }
    memset(pt->id, 0, sizeof pt->id);
    snprintf((char*)pt->id, sizeof pt->id, "keto_consumer partition %d", generation++);
    rank_call_t calls[MAX_REPLICAS];
    memset(calls, 0, sizeof calls);
    for (int k = 0; k < pt->n; ++k) calls[k].op = 0;
    const int rc = ranks_run(pt, calls);
    if (rc != KETO_OK) fail("keto_comm_init_local", rc);
}

static void partition_release(partition_t* pt) {
    for (int k = 0; k < pt->n; ++k) {
        keto_comm_free(pt->comms[k]);
        keto_snapshot_release(pt->parts[k]);
    }
}

/* prints the m trees of arena ar ("expand" lines): per-tree and batch JSON, protobuf, and the tree
   rebuilt from nodes + subject fields re-encoded; returns 0, or the exit code of a mismatch */
static int print_trees(keto_snapshot* snap, keto_tree_arena* ar, uint32_t m, int* expands) {
    if (keto_tree_count(ar) != m) return 5;
    /* the batch JSON (size query, then fill) */
    uint64_t* offs = (uint64_t*)xrealloc(NULL, (m + 1) * sizeof(uint64_t));
    const int64_t an = keto_tree_json_all(snap, ar, NULL, 0, offs);
    if (an < 0) fail("keto_tree_json_all", (int)an);
    char* all = (char*)xrealloc(NULL, (size_t)an + 1);
    if (keto_tree_json_all(snap, ar, all, (uint64_t)an, offs) != an) return 6;
    for (uint32_t k = 0; k < m; ++k) {
        const int s = keto_tree_status(ar, k);
        const int64_t jn = keto_tree_json(snap, ar, k, NULL, 0);
        char* js = NULL;
        if (jn >= 0) {
            js = (char*)malloc((size_t)jn + 1);
            if (!js || keto_tree_json(snap, ar, k, js, (uint64_t)jn + 1) != jn) return 6;
        }
        const uint64_t tl = offs[k + 1] - offs[k];
        if (js ? (tl != (uint64_t)jn || memcmp(all + offs[k], js, tl) != 0) : tl != 0) return 6;
        const int64_t pn = keto_tree_proto(snap, ar, k, NULL, 0);
        printf("expand\t%d\t%d\t%s\t", (*expands)++, s, js ? js : "error");
        buf_t via = {0, 0, 0};
        if (tree_via_fields(snap, ar, k, &via)) return 9;
        if (pn > 0) {
            uint8_t* pb = (uint8_t*)malloc((size_t)pn);
            if (!pb || keto_tree_proto(snap, ar, k, pb, (uint64_t)pn) != pn) return 7;
            /* the tree the Go shim builds from nodes + fields encodes to the same bytes */
            if (via.n != (size_t)pn || memcmp(via.p, pb, (size_t)pn) != 0) return 10;
            for (int64_t x = 0; x < pn; ++x) printf("%02x", pb[x]);
            free(pb);
        } else {
            if (via.n != 0) return 10;
            printf("-");
        }
        free(via.p);
        printf("\n");
        free(js);
    }
    free(all);
    free(offs);
    return 0;
}

static void subject_of(line_t* l, int* k, keto_subject* s) {
    memset(s, 0, sizeof *s);
    if (!strcmp(l->f[(*k)++], "I")) {
        s->kind = 0;
        s->id = ks(l->f[(*k)++]);
    } else {
        s->kind = 1;
        s->set_namespace = ks(l->f[(*k)++]);
        s->set_object = ks(l->f[(*k)++]);
        s->set_relation = ks(l->f[(*k)++]);
    }
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <input>\n", argv[0]);
        return 1;
    }
    FILE* in = fopen(argv[1], "r");
    if (!in) return 1;
    if (keto_abi_version() != KETO_ABI_VERSION) {
        fprintf(stderr, "ABI %d != header %d\n", keto_abi_version(), KETO_ABI_VERSION);
        return 2;
    }
    line_t** lines = NULL;
    size_t n_lines = 0;
    char buf[1 << 16];
    uint32_t page_size = 100;
    int device = -1;
    int devices[MAX_REPLICAS], n_reps = 0;
    partition_t part;
    memset(&part, 0, sizeof part);
    while (fgets(buf, sizeof buf, in)) {
        line_t* l = (line_t*)calloc(1, sizeof(line_t));
        if (!l || split(buf, l) < 1) return 1;
        if (!strcmp(l->f[0], "P")) page_size = (uint32_t)atoi(l->f[1]);
        else if (!strcmp(l->f[0], "V")) device = atoi(l->f[1]);
        else if (!strcmp(l->f[0], "R"))
            for (int k = 1; k < l->n && n_reps < MAX_REPLICAS; ++k) devices[n_reps++] = atoi(l->f[k]);
        else if (!strcmp(l->f[0], "Q"))
            for (int k = 1; k < l->n && part.n < MAX_REPLICAS; ++k) part.devices[part.n++] = atoi(l->f[k]);
        lines = (line_t**)xrealloc(lines, (n_lines + 1) * sizeof(line_t*));
        lines[n_lines++] = l;
    }
    fclose(in);

    /* namespaces (config order) and the initial table (commit order) */
    size_t n_ns = 0;
    keto_namespace* ns = NULL;
    table_t table = {0, 0, 0};
    for (size_t i = 0; i < n_lines; ++i) {
        line_t* l = lines[i];
        if (!strcmp(l->f[0], "N")) {
            ns = (keto_namespace*)xrealloc(ns, (n_ns + 1) * sizeof(keto_namespace));
            ns[n_ns].id = atoi(l->f[1]);
            ns[n_ns++].name = ks(l->f[2]);
        } else if (!strcmp(l->f[0], "T")) {
            table_insert(&table, tuple_of(l, 1));
        }
    }
    if (n_reps == 0) devices[n_reps++] = device;
    keto_snapshot* reps[MAX_REPLICAS];
    const int parted = part.n > 0;
    if (parted) {
        device = part.devices[0];
        partition_from(build(ns, n_ns, &table, page_size, -1), &part);
        n_reps = 1;
        reps[0] = part.parts[0];
    } else {
        build_replicas(ns, n_ns, &table, page_size, devices, n_reps, reps);
    }
    keto_snapshot* snap = reps[0];
    int batches = 0;                          /* batches dealt round-robin over the replicas */
    keto_snapshot_stats st;
    int rc = keto_snapshot_get_stats(snap, &st);
    if (rc != KETO_OK) fail("keto_snapshot_get_stats", rc);
    printf("stats tuples=%llu rows=%u real=%u wildcard=%u seq=%u poisoned=%u strings=%u collisions=%u\n",
           (unsigned long long)st.n_tuples, st.n_rows, st.n_real_rows, st.n_wildcard_rows, st.n_seq_rows,
           st.n_poisoned_rows, st.n_strings, st.n_collision_keys);

    int checks = 0, expands = 0;
    keto_tuple* ins = NULL;
    keto_tuple* del = NULL;
    size_t n_ins = 0, n_del = 0;
    for (size_t i = 0; i < n_lines;) {
        line_t* l = lines[i];
        if (!strcmp(l->f[0], "C")) {
            /* one micro-batch: the consecutive checks with this global max depth */
            const int32_t gmd = atoi(l->f[l->n - 1]);
            size_t j = i;
            while (j < n_lines && !strcmp(lines[j]->f[0], "C") && atoi(lines[j]->f[lines[j]->n - 1]) == gmd) ++j;
            const size_t m = j - i;
            keto_check_req* q = (keto_check_req*)calloc(m, sizeof(keto_check_req));
            uint8_t* allowed = (uint8_t*)malloc(m);
            uint8_t* status = (uint8_t*)malloc(m);
            if (!q || !allowed || !status) return 3;
            for (size_t k = 0; k < m; ++k) {
                line_t* c = lines[i + k];
                q[k].namespace_ = ks(c->f[1]);
                q[k].object = ks(c->f[2]);
                q[k].relation = ks(c->f[3]);
                int f = 4;
                subject_of(c, &f, &q[k].subject);
                q[k].max_depth = atoi(c->f[f]);
            }
            snap = reps[batches++ % n_reps];
            if (parted) {
                /* every rank its slice of the batch (the last ranks' slices may be empty) */
                rank_call_t calls[MAX_REPLICAS];
                memset(calls, 0, sizeof calls);
                for (int k = 0; k < part.n; ++k) {
                    const size_t lo = m * (size_t)k / (size_t)part.n, hi = m * (size_t)(k + 1) / (size_t)part.n;
                    calls[k].op = 1;
                    calls[k].q = q + lo;
                    calls[k].n = (uint32_t)(hi - lo);
                    calls[k].gmd = gmd;
                    calls[k].allowed = allowed + lo;
                    calls[k].status = status + lo;
                }
                rc = ranks_run(&part, calls);
                if (rc != KETO_OK) fail("keto_check_batch_routed", rc);
                {
                    /* the Go Partition's call: every rank's slice packed and resolved on its device
                       (keto_check_batch_routed_packed); decisions and statuses must equal the named form's */
                    uint8_t* pa = (uint8_t*)malloc(m ? m : 1);
                    uint8_t* ps = (uint8_t*)malloc(m ? m : 1);
                    char* blobs[MAX_REPLICAS];
                    keto_check_packed* pks[MAX_REPLICAS];
                    if (!pa || !ps) return 3;
                    for (int k = 0; k < part.n; ++k) {
                        pack_batch(calls[k].q, calls[k].n, &blobs[k], &calls[k].blob_len, &pks[k]);
                        calls[k].op = 3;
                        calls[k].blob = blobs[k];
                        calls[k].pk = pks[k];
                        calls[k].allowed = pa + (calls[k].q - q);
                        calls[k].status = ps + (calls[k].q - q);
                    }
                    rc = ranks_run(&part, calls);
                    if (rc != KETO_OK) fail("keto_check_batch_routed_packed", rc);
                    for (size_t k = 0; k < m; ++k)
                        if (pa[k] != allowed[k] || ps[k] != status[k]) return 15;
                    for (int k = 0; k < part.n; ++k) {
                        free(blobs[k]);
                        free(pks[k]);
                    }
                    free(pa);
                    free(ps);
                }
                for (size_t k = 0; k < m; ++k) printf("check\t%d\t%u\t%u\n", checks++, allowed[k], status[k]);
                free(q);
                free(allowed);
                free(status);
                i = j;
                continue;
            }
            rc = keto_check_batch(snap, q, (uint32_t)m, gmd, allowed, status);
            if (device < 0) {
                printf("nodevice %d\n", rc);
                if (rc != KETO_E_HIP || !keto_last_error()[0]) return 4;
                break;
            }
            if (rc != KETO_OK) fail("keto_check_batch", rc);
            {
                /* the Go shim's path: the same batch packed in one string blob, resolved on the GPU
                   (keto_check_batch_packed); decisions and statuses must equal keto_check_batch's */
                size_t total = 0;
                char* blob = NULL;
                keto_check_packed* pk = NULL;
                pack_batch(q, m, &blob, &total, &pk);
                uint8_t* pa = (uint8_t*)malloc(m);
                uint8_t* ps = (uint8_t*)malloc(m);
                if (!pa || !ps) return 3;
                rc = keto_check_batch_packed(snap, blob, total, pk, (uint32_t)m, gmd, pa, ps);
                if (rc != KETO_OK) fail("keto_check_batch_packed", rc);
                for (size_t k = 0; k < m; ++k)
                    if (pa[k] != allowed[k] || ps[k] != status[k]) return 13;
                /* several threads at once, as the Go batcher keeps batches in flight per engine: the
                   library runs one's upload and resolution under another's check; every thread's
                   decisions and statuses must equal keto_check_batch's */
                {
                    packed_call_t pc[PACKED_THREADS];
                    pthread_t th[PACKED_THREADS];
                    for (int t = 0; t < PACKED_THREADS; ++t) {
                        pc[t] = (packed_call_t){snap, blob, total, pk, (uint32_t)m, gmd, allowed, status, 0};
                        if (pthread_create(&th[t], NULL, packed_main, &pc[t]) != 0) exit(3);
                    }
                    for (int t = 0; t < PACKED_THREADS; ++t) pthread_join(th[t], NULL);
                    for (int t = 0; t < PACKED_THREADS; ++t)
                        if (pc[t].bad) return 14;
                }
                free(blob);
                free(pk);
                free(pa);
                free(ps);
            }
            for (size_t k = 0; k < m; ++k) printf("check\t%d\t%u\t%u\n", checks++, allowed[k], status[k]);
            free(q);
            free(allowed);
            free(status);
            i = j;
            continue;
        }
        if (!strcmp(l->f[0], "E") && device >= 0) {
            const int32_t gmd = atoi(l->f[l->n - 1]);
            size_t j = i;
            while (j < n_lines && !strcmp(lines[j]->f[0], "E") && atoi(lines[j]->f[lines[j]->n - 1]) == gmd) ++j;
            const size_t m = j - i;
            keto_expand_req* r = (keto_expand_req*)calloc(m, sizeof(keto_expand_req));
            if (!r) return 3;
            for (size_t k = 0; k < m; ++k) {
                int f = 1;
                subject_of(lines[i + k], &f, &r[k].subject);
                r[k].max_depth = atoi(lines[i + k]->f[f]);
            }
            if (parted) {
                rank_call_t calls[MAX_REPLICAS];
                memset(calls, 0, sizeof calls);
                for (int k = 0; k < part.n; ++k) {
                    const size_t lo = m * (size_t)k / (size_t)part.n, hi = m * (size_t)(k + 1) / (size_t)part.n;
                    calls[k].op = 2;
                    calls[k].e = r + lo;
                    calls[k].n = (uint32_t)(hi - lo);
                    calls[k].gmd = gmd;
                }
                rc = ranks_run(&part, calls);
                if (rc != KETO_OK) fail("keto_expand_batch_routed", rc);
                for (int k = 0; k < part.n; ++k) {
                    /* each rank's trees, in request order, read through its own part's host tables */
                    const int e = print_trees(part.parts[k], calls[k].ar, calls[k].n, &expands);
                    keto_tree_arena_free(calls[k].ar);
                    if (e) return e;
                }
            } else {
                keto_tree_arena* ar = NULL;
                snap = reps[batches++ % n_reps];
                rc = keto_expand_batch(snap, r, (uint32_t)m, gmd, &ar);
                if (rc != KETO_OK) fail("keto_expand_batch", rc);
                const int e = print_trees(snap, ar, (uint32_t)m, &expands);
                keto_tree_arena_free(ar);
                if (e) return e;
            }
            free(r);
            i = j;
            continue;
        }
        if (!strcmp(l->f[0], "A+") || !strcmp(l->f[0], "A-")) {
            const keto_tuple t = tuple_of(l, 1);
            if (l->f[0][1] == '+') {
                ins = (keto_tuple*)xrealloc(ins, (n_ins + 1) * sizeof(keto_tuple));
                ins[n_ins++] = t;
            } else {
                del = (keto_tuple*)xrealloc(del, (n_del + 1) * sizeof(keto_tuple));
                del[n_del++] = t;
            }
        } else if (!strcmp(l->f[0], "A!")) {
            /* the transaction committed in SQL: the table changes, then the snapshot follows */
            for (size_t k = 0; k < n_ins; ++k) table_insert(&table, ins[k]);
            for (size_t k = 0; k < n_del; ++k) table_delete(&table, &del[k]);
            /* every replica follows the transaction; one refusal rebuilds them all */
            /* (a partitioned graph: every part applies every transaction) */
            keto_snapshot** tgt = parted ? part.parts : reps;
            const int n_tgt = parted ? part.n : n_reps;
            uint64_t v0 = keto_snapshot_version(tgt[0]), v = 0;
            int rebuilt = 0;
            rc = KETO_OK;
            for (int k = 0; k < n_tgt && rc == KETO_OK; ++k) {
                uint64_t vk = 0;
                rc = keto_snapshot_apply(tgt[k], ins, n_ins, del, n_del, &vk);
                if (rc == KETO_OK && (vk != v0 + 1 || keto_snapshot_version(tgt[k]) != vk)) return 12;
                if (rc == KETO_E_REBUILD && keto_snapshot_version(tgt[k]) != v0) return 11; /* left unchanged */
                v = vk;
            }
            if (rc == KETO_E_REBUILD && parted) {
                partition_release(&part);
                partition_from(build(ns, n_ns, &table, page_size, -1), &part);
                reps[0] = part.parts[0];
                rebuilt = 1;
                v = keto_snapshot_version(reps[0]);
            } else if (rc == KETO_E_REBUILD) {
                for (int k = 0; k < n_reps; ++k) keto_snapshot_release(reps[k]);
                build_replicas(ns, n_ns, &table, page_size, devices, n_reps, reps);
                rebuilt = 1;
                v = keto_snapshot_version(reps[0]);
            } else if (rc != KETO_OK) {
                fail("keto_snapshot_apply", rc);
            }
            snap = reps[0];
            printf("apply\t%d\t%llu\t%d\n", rc, (unsigned long long)v, rebuilt);
            n_ins = n_del = 0;
        } else if (!strcmp(l->f[0], "S") && parted) {
            /* the partitioned server's restart: a host-only snapshot of the table saved, the parts
               released, the file loaded host-only and partitioned again */
            keto_snapshot* base = build(ns, n_ns, &table, page_size, -1);
            const uint64_t v0 = keto_snapshot_version(base);
            rc = keto_snapshot_save(base, l->f[1], v0);
            if (rc != KETO_OK) fail("keto_snapshot_save", rc);
            keto_snapshot_release(base);
            partition_release(&part);
            uint64_t tag = 0;
            rc = keto_snapshot_load(l->f[1], -1, &base, &tag);
            if (rc != KETO_OK) fail("keto_snapshot_load", rc);
            if (tag != v0 || keto_snapshot_version(base) != v0) return 13;
            partition_from(base, &part);
            snap = reps[0] = part.parts[0];
            printf("restart\t%llu\t%llu\n", (unsigned long long)v0, (unsigned long long)tag);
        } else if (!strcmp(l->f[0], "S")) {
            const uint64_t v0 = keto_snapshot_version(reps[0]);
            rc = keto_snapshot_save(reps[0], l->f[1], v0);
            if (rc != KETO_OK) fail("keto_snapshot_save", rc);
            for (int k = 0; k < n_reps; ++k) keto_snapshot_release(reps[k]);
            uint64_t tag = 0;
            rc = keto_snapshot_load(l->f[1], devices[0], &reps[0], &tag);
            if (rc != KETO_OK) fail("keto_snapshot_load", rc);
            if (tag != v0 || keto_snapshot_version(reps[0]) != v0) return 13;
            for (int k = 1; k < n_reps; ++k) {
                rc = keto_snapshot_clone(reps[0], devices[k], &reps[k]);
                if (rc != KETO_OK) fail("keto_snapshot_clone", rc);
            }
            snap = reps[0];
            printf("restart\t%llu\t%llu\n", (unsigned long long)v0, (unsigned long long)tag);
        }
        ++i;
    }
    /* an error path: a NULL argument must fail with a message, not crash */
    rc = keto_check_batch(reps[0], NULL, 1, 5, NULL, NULL);
    if (rc != KETO_E_INVALID || !keto_last_error()[0]) return 8;
    if (parted)
        partition_release(&part);
    else
        for (int k = 0; k < n_reps; ++k) keto_snapshot_release(reps[k]);
    for (size_t i = 0; i < n_lines; ++i) {
        for (int k = 0; k < lines[i]->n; ++k) free(lines[i]->f[k]);
        free(lines[i]);
    }
    free(lines);
    free(ns);
    free(table.t);
    free(ins);
    free(del);
    printf("done\n");
    return 0;
}
