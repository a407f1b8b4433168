/*
 * keto_consumer.c -- a plain C consumer of include/keto_mi355x.h, written against the header only.
 *
 * It makes the calls, in the order, the Go shim (integration/go/internal/gpu/gpu.go) makes: build a
 * snapshot from the keto_relation_tuples rows (strings, commit order), check and expand batches,
 * read the per-request statuses, the expand trees as JSON (size query, then fill) and as protobuf,
 * the last error, and free everything.  tests/test_consumer_c.py compiles it with gcc against the
 * header and runs it: host-only (device -1: compute must fail with KETO_E_HIP) on the CPU, and the
 * reference's golden cases (tests/golden/reference_cases.json) on the GPU.
 *
 * Input (tab-separated lines; empty fields allowed):
 *   P <page_size>        V <device>
 *   N <ns id> <name>
 *   T <ns id> <object> <relation> I <subject id>
 *   T <ns id> <object> <relation> S <set ns id> <set object> <set relation>
 *   C <ns> <object> <relation> I <subject id> <max depth> <global max depth>
 *   C <ns> <object> <relation> S <set ns> <set object> <set relation> <max depth> <global max depth>
 *   E I <subject id> <max depth> <global max depth>
 *   E S <ns> <object> <relation> <max depth> <global max depth>
 * Output (tab-separated): "check <i> <allowed> <status>", "expand <i> <status> <json|null|error> <proto hex>",
 * "stats ...", "nodevice <rc>".
 */
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

typedef struct {
    void** v;
    size_t n, cap;
} vec;

static void push(vec* v, void* x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 16;
        v->v = (void**)realloc(v->v, v->cap * sizeof(void*));
        if (!v->v) exit(3);
    }
    v->v[v->n++] = x;
}

static void fail(const char* what, int rc) {
    fprintf(stderr, "%s failed: %d (%s)\n", what, rc, keto_last_error());
    exit(2);
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
    vec lines = {0, 0, 0};
    char buf[1 << 16];
    uint32_t page_size = 100;
    int device = -1;
    while (fgets(buf, sizeof buf, in)) {
        line_t* l = (line_t*)calloc(1, sizeof(line_t));
        if (!l || split(buf, l) < 1) return 1;
        if (!strcmp(l->f[0], "P")) page_size = (uint32_t)atoi(l->f[1]);
        else if (!strcmp(l->f[0], "V")) device = atoi(l->f[1]);
        else push(&lines, l);
    }
    fclose(in);

    /* namespaces and tuples (commit order) */
    size_t n_ns = 0, n_t = 0;
    for (size_t i = 0; i < lines.n; ++i) {
        line_t* l = (line_t*)lines.v[i];
        n_ns += !strcmp(l->f[0], "N");
        n_t += !strcmp(l->f[0], "T");
    }
    keto_namespace* ns = (keto_namespace*)calloc(n_ns ? n_ns : 1, sizeof(keto_namespace));
    keto_tuple* tu = (keto_tuple*)calloc(n_t ? n_t : 1, sizeof(keto_tuple));
    size_t a = 0, b = 0;
    for (size_t i = 0; i < lines.n; ++i) {
        line_t* l = (line_t*)lines.v[i];
        if (!strcmp(l->f[0], "N")) {
            ns[a].id = atoi(l->f[1]);
            ns[a++].name = ks(l->f[2]);
        } else if (!strcmp(l->f[0], "T")) {
            keto_tuple* t = &tu[b++];
            t->namespace_id = atoi(l->f[1]);
            t->object = ks(l->f[2]);
            t->relation = ks(l->f[3]);
            if (!strcmp(l->f[4], "I")) {
                t->subject_kind = 0;
                t->subject_id = ks(l->f[5]);
            } else {
                t->subject_kind = 1;
                t->set_namespace_id = atoi(l->f[5]);
                t->set_object = ks(l->f[6]);
                t->set_relation = ks(l->f[7]);
            }
        }
    }
    keto_snapshot_opts opts;
    opts.page_size = page_size;
    opts.device = device;
    opts.flags = 0;
    keto_snapshot* snap = NULL;
    int rc = keto_snapshot_build(ns, (uint32_t)n_ns, tu, n_t, &opts, &snap);
    if (rc != KETO_OK) fail("keto_snapshot_build", rc);
    keto_snapshot_stats st;
    rc = keto_snapshot_get_stats(snap, &st);
    if (rc != KETO_OK) fail("keto_snapshot_get_stats", rc);
    printf("stats tuples=%llu rows=%u real=%u wildcard=%u seq=%u poisoned=%u strings=%u collisions=%u\n",
           (unsigned long long)st.n_tuples, st.n_rows, st.n_real_rows, st.n_wildcard_rows, st.n_seq_rows,
           st.n_poisoned_rows, st.n_strings, st.n_collision_keys);

    /* checks: one batch per request, as the micro-batcher's smallest flush */
    int checks = 0, expands = 0;
    for (size_t i = 0; i < lines.n; ++i) {
        line_t* l = (line_t*)lines.v[i];
        if (!strcmp(l->f[0], "C")) {
            keto_check_req q;
            memset(&q, 0, sizeof q);
            q.namespace_ = ks(l->f[1]);
            q.object = ks(l->f[2]);
            q.relation = ks(l->f[3]);
            int k = 5;
            if (!strcmp(l->f[4], "I")) {
                q.subject.kind = 0;
                q.subject.id = ks(l->f[k++]);
            } else {
                q.subject.kind = 1;
                q.subject.set_namespace = ks(l->f[k++]);
                q.subject.set_object = ks(l->f[k++]);
                q.subject.set_relation = ks(l->f[k++]);
            }
            q.max_depth = atoi(l->f[k++]);
            const int32_t gmd = atoi(l->f[k]);
            uint8_t allowed = 9, status = 9;
            rc = keto_check_batch(snap, &q, 1, gmd, &allowed, &status);
            if (device < 0) {
                printf("nodevice %d\n", rc);
                if (rc != KETO_E_HIP || !keto_last_error()[0]) return 4;
                break;
            }
            if (rc != KETO_OK) fail("keto_check_batch", rc);
            printf("check\t%d\t%u\t%u\n", checks++, allowed, status);
        } else if (!strcmp(l->f[0], "E") && device >= 0) {
            keto_expand_req r;
            memset(&r, 0, sizeof r);
            int k = 2;
            if (!strcmp(l->f[1], "I")) {
                r.subject.kind = 0;
                r.subject.id = ks(l->f[k++]);
            } else {
                r.subject.kind = 1;
                r.subject.set_namespace = ks(l->f[k++]);
                r.subject.set_object = ks(l->f[k++]);
                r.subject.set_relation = ks(l->f[k++]);
            }
            r.max_depth = atoi(l->f[k++]);
            const int32_t gmd = atoi(l->f[k]);
            keto_tree_arena* ar = NULL;
            rc = keto_expand_batch(snap, &r, 1, gmd, &ar);
            if (rc != KETO_OK) fail("keto_expand_batch", rc);
            if (keto_tree_count(ar) != 1) return 5;
            const int s = keto_tree_status(ar, 0);
            const int64_t jn = keto_tree_json(snap, ar, 0, NULL, 0);
            char* js = NULL;
            if (jn >= 0) {
                js = (char*)malloc((size_t)jn + 1);
                if (keto_tree_json(snap, ar, 0, js, (uint64_t)jn + 1) != jn) return 6;
            }
            {   /* the batch form (what the Go shim calls): the same text, "" for an error root */
                uint64_t offs[2];
                const int64_t an = keto_tree_json_all(snap, ar, NULL, 0, offs);
                if (an < 0) fail("keto_tree_json_all", (int)an);
                char* all = (char*)malloc((size_t)an + 1);
                if (keto_tree_json_all(snap, ar, all, (uint64_t)an, offs) != an) return 6;
                if (offs[0] != 0 || offs[1] != (uint64_t)an) return 6;
                if (js ? (an != jn || memcmp(all, js, (size_t)an) != 0) : an != 0) return 6;
                free(all);
            }
            const int64_t pn = keto_tree_proto(snap, ar, 0, NULL, 0);
            printf("expand\t%d\t%d\t%s\t", expands++, s, js ? js : "error");
            if (pn > 0) {
                uint8_t* pb = (uint8_t*)malloc((size_t)pn);
                if (keto_tree_proto(snap, ar, 0, pb, (uint64_t)pn) != pn) return 7;
                for (int64_t x = 0; x < pn; ++x) printf("%02x", pb[x]);
                free(pb);
            } else {
                printf("-");
            }
            printf("\n");
            free(js);
            keto_tree_arena_free(ar);
        }
    }
    /* an error path: a NULL argument must fail with a message, not crash */
    rc = keto_check_batch(snap, NULL, 1, 5, NULL, NULL);
    if (rc != KETO_E_INVALID || !keto_last_error()[0]) return 8;
    keto_snapshot_release(snap);
    for (size_t i = 0; i < lines.n; ++i) {
        line_t* l = (line_t*)lines.v[i];
        for (int k = 0; k < l->n; ++k) free(l->f[k]);
        free(l);
    }
    free(lines.v);
    free(ns);
    free(tu);
    printf("done\n");
    return 0;
}
