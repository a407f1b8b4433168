/*
 * keto_mi355x.h -- C-ABI of the MI355X batched check / expand engine.
 *
 * This is the drop-in boundary for Keto's read hot path.  Each entry point replaces one
 * reference interface (paths relative to the reference tree, icyphox/keto = ory/keto v0.8.1):
 *
 *   keto_snapshot_build      replaces the per-node SQL reads the engines issue through
 *                            relationtuple.Manager.GetRelationTuples
 *                            (internal/relationtuple/definitions.go:29;
 *                             internal/persistence/sql/relationtuples.go:238-277) with one
 *                            immutable CSR snapshot built from a full scan of keto_relation_tuples
 *                            in the same ORDER BY (relationtuples.go:250).
 *   keto_check_batch         replaces check.(*Engine).SubjectIsAllowed
 *                            (internal/check/engine.go:116-123), batched.
 *   keto_expand_batch        replaces expand.(*Engine).BuildTree
 *                            (internal/expand/engine.go:33-102), batched.
 *   keto_tree_*              replace the expand.Tree value and its JSON codec
 *                            (internal/expand/tree.go:26-30,156-163).
 *
 * All strings are borrowed (keto_str = pointer + length, not NUL-terminated) and only read
 * during the call.  The library keeps no caller pointers after a call returns.  A snapshot may be
 * shared by concurrent *_batch calls from any threads; calls on one snapshot run one at a time on its
 * device (a batch's persistent grid fills the whole GPU, so overlapping two would not finish either
 * sooner), each call's host-side work (resolution, staging) runs in the calling thread.  The
 * exception is keto_check_batch_packed with a small batch (below), whose calls from several threads
 * keep up to KETO_PACKED_SLOTS (default 2) batches in flight: one's upload and resolution run while
 * another's check does.
 * Every call returns KETO_OK (0) or a negative KETO_E_* code; keto_last_error() then holds a
 * thread-local message.  There is no CPU fallback inside the library: when the HIP runtime or a
 * device is missing, compute calls fail with KETO_E_HIP.
 */
#ifndef KETO_MI355X_H
#define KETO_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KETO_ABI_VERSION 6
/* The largest arena one snapshot (a replica) or one partition part takes on a device: handles are
 * 32-bit; below 2^31 a count of 16-byte units (subject-set targets, and the root rows of the first
 * 32 GiB), above it a count of 32-, 64- or 128-byte units of the root rows past 32 GiB (arenas past
 * 64 GiB, whatever unit gives every root row a handle).  A graph past it is served as several
 * shared-rows parts, more than one per device if need be (each part holds the subject-set targets and
 * its share of the root rows).  Targets alone are capped at 32 GiB. */
#define KETO_ARENA_MAX_BYTES (288ull << 30)

/* return codes */
#define KETO_OK 0
#define KETO_E_INVALID (-1)     /* bad argument */
#define KETO_E_HIP (-2)         /* HIP runtime / device error, or no device */
#define KETO_E_NOMEM (-3)       /* host or device allocation failed */
#define KETO_E_CONFIG (-4)      /* namespace config not supported (duplicate ids or names) */
#define KETO_E_RANGE (-5)       /* a size limit of the snapshot format was exceeded */
#define KETO_E_REBUILD (-6)     /* keto_snapshot_apply: this write needs a rebuild (snapshot unchanged) */

/* per-query status of keto_check_batch (allowed_out is always valid) */
#define KETO_CHECK_OK 0                 /* decision equals the reference engine's */
#define KETO_CHECK_UNKNOWN_NAMESPACE 1  /* request namespace unknown: reference returns false (engine.go:98-100) */
#define KETO_CHECK_UNDECIDED 2          /* no tier could decide it within the engine's limits (allowed_out = 0):
                                           ask the reference engine; the other requests of
                                           the batch are decided as usual */

/* decision byte of the ids / device entry points: 0 = denied, 1 = allowed, KETO_UNDECIDED = the
 * request exceeded the engine's limits on its final tier (per request, never the whole batch) */
#define KETO_UNDECIDED 2

/* per-root status of keto_expand_batch */
#define KETO_EXPAND_TREE 0              /* a tree (BuildTree returned a non-nil *Tree) */
#define KETO_EXPAND_NIL 1               /* BuildTree returned nil, nil (JSON null) */
#define KETO_EXPAND_NOT_FOUND 2         /* BuildTree returned herodot.ErrNotFound (unknown namespace, A.Q8/Q9) */
#define KETO_EXPAND_UNDECIDED 3         /* the tree exceeded the engine's limits: ask the reference engine */

/* node types of an expand tree (internal/expand/tree.go:16-23; only union and leaf are produced) */
#define KETO_NODE_UNION 0
#define KETO_NODE_LEAF 1

typedef struct {
    const char* p;
    uint32_t n;
} keto_str;

/* namespace.Namespace{ID, Name} (internal/namespace/definitions.go:9-13), in config order */
typedef struct {
    int32_t id;
    keto_str name;
} keto_namespace;

/* one row of keto_relation_tuples (internal/persistence/sql/relationtuples.go:19-31).
 * Array order = commit order (commit_time ties are broken by position). */
typedef struct {
    int32_t namespace_id;
    keto_str object;
    keto_str relation;
    uint8_t subject_kind;       /* 0 = subject_id, 1 = subject set */
    keto_str subject_id;        /* kind 0 */
    int32_t set_namespace_id;   /* kind 1 */
    keto_str set_object;        /* kind 1 */
    keto_str set_relation;      /* kind 1 */
} keto_tuple;

/* a Subject by name (internal/relationtuple/definitions.go:77-117) */
typedef struct {
    uint8_t kind;               /* 0 = SubjectID, 1 = SubjectSet */
    keto_str id;                /* kind 0 */
    keto_str set_namespace;     /* kind 1 */
    keto_str set_object;
    keto_str set_relation;
} keto_subject;

/* check request = InternalRelationTuple + request max-depth (CheckRequest, check_service.proto) */
typedef struct {
    keto_str namespace_;
    keto_str object;
    keto_str relation;
    keto_subject subject;
    int32_t max_depth;          /* <= 0 or > global -> global (engine.go:118-120) */
} keto_check_req;

/* pre-resolved check request (keto_resolve_checks), 16 bytes; the form the device consumes.
 * Rows are named by *row handles* (their place in the device arena; keto_row_handles maps row ids,
 * i.e. positions in (namespace_id, object, relation) order, to handles). */
typedef struct {
    uint32_t row;               /* top-level row handle, or KETO_NO_ROW */
    uint32_t target;            /* subject: ID string id, or row handle of a subject set, or KETO_NO_TARGET */
    uint32_t flags;             /* bit0: target is a subject set */
    int32_t max_depth;          /* request max-depth (clamped on the device) */
} keto_check_ids;
#define KETO_NO_ROW 0xFFFFFFFFu
#define KETO_NO_TARGET 0xFFFFFFFFu

/* expand request (ExpandRequest, expand_service.proto) */
typedef struct {
    keto_subject subject;
    int32_t max_depth;
} keto_expand_req;

/* one node of an expand tree in pre-order.  subject: bit31 set -> subject set (bits 0..30 = row
 * id), else subject id (bits 0..30 = string id).  info: bit31 set -> leaf, bits 0..30 = number of
 * children (all children follow in pre-order). */
typedef struct {
    uint32_t subject;
    uint32_t info;
} keto_tree_node;

typedef struct {
    uint32_t page_size;         /* 0 -> 100 (internal/persistence/sql/persister.go:46) */
    int32_t device;             /* HIP device ordinal; -1 = host-only snapshot (no compute) */
    uint32_t flags;             /* reserved, 0 */
} keto_snapshot_opts;

typedef struct keto_snapshot keto_snapshot;
typedef struct keto_tree_arena keto_tree_arena;

typedef struct {
    uint64_t n_tuples;
    uint64_t n_edges;           /* including materialized wildcard rows */
    uint32_t n_rows;            /* real + empty + wildcard rows */
    uint32_t n_real_rows;
    uint32_t n_wildcard_rows;
    uint32_t n_seq_rows;        /* rows on the ordered (collision / wildcard) path */
    uint32_t n_poisoned_rows;
    uint32_t n_strings;
    uint32_t n_collision_keys;
    uint64_t device_bytes;
} keto_snapshot_stats;

int keto_abi_version(void);
const char* keto_last_error(void);

/* Build a snapshot from the tuple table; sorts with the reference ORDER BY itself. */
int keto_snapshot_build(const keto_namespace* namespaces, uint32_t n_namespaces, const keto_tuple* tuples,
                        uint64_t n_tuples, const keto_snapshot_opts* opts, keto_snapshot** out);

/* Bulk loader for pre-interned, pre-ordered data (synthetic / exported snapshots).
 * row_ns/row_obj/row_rel: per row, namespace id and string ids; rows must be in
 * (namespace_id, object bytes, relation bytes) order.  row_ptr: n_rows+1 offsets into edges.
 * edges: per row, subject sets first (bit31 set, bits 0..30 = target row) in reference order, then
 * subject ids (bits 0..30 = string id) in byte order.  strings: n_strings strings in byte order
 * (string id = index).  The caller guarantees that no Subject.String() of two different subjects
 * coincide and that every subject set resolves to a row (pass empty rows for dangling sets). */
int keto_snapshot_from_csr(const keto_namespace* namespaces, uint32_t n_namespaces, uint32_t n_rows,
                           const int32_t* row_ns, const uint32_t* row_obj, const uint32_t* row_rel,
                           const uint64_t* row_ptr, const uint32_t* edges, const keto_str* strings,
                           uint32_t n_strings, const keto_snapshot_opts* opts, keto_snapshot** out);

void keto_snapshot_release(keto_snapshot* s);

/* A replica of an unpartitioned snapshot for another device (device = -1: host only), at the source's
 * current version, without scanning or sorting the table again: the host tables are copied and laid
 * out afresh, then uploaded.  One server process serving the node's GPUs keeps one replica per
 * device, deals batches among them and applies every write transaction to each (the reference serves
 * every request from one process, internal/driver/daemon.go:62-69, on engines built once per registry,
 * internal/driver/registry_default.go:159-171).  Replicas are independent snapshots afterwards. */
int keto_snapshot_clone(const keto_snapshot* src, int32_t device, keto_snapshot** out);

/* Persisted snapshot (the optional on-disk CSR): keto_snapshot_save writes the
 * host tables of an unpartitioned snapshot at its current version (the interned strings, the rows in
 * ORDER BY order with their page cuts and edges, the collision classes, the rows writes changed) to
 * `path` (through <path>.tmp and a rename, so an interrupted save leaves an older file intact), with
 * the caller's 64-bit `tag` -- e.g. the table's last commit covered, so that a restarting server
 * replays only later transactions (the reference re-reads the table on every query,
 * internal/persistence/sql/relationtuples.go:249-251; a GPU server otherwise rebuilds the snapshot
 * from a full scan and sort).  keto_snapshot_load reads it back, lays it out and uploads it to
 * `device` (-1: host only); *tag_out (may be NULL) gets the tag.  The loaded snapshot answers every
 * call exactly as the saved one did and has its version.  A file that is not a snapshot, has another
 * format, is truncated or fails a section checksum: KETO_E_INVALID. */
int keto_snapshot_save(const keto_snapshot* s, const char* path, uint64_t tag);
int keto_snapshot_load(const char* path, int32_t device, keto_snapshot** out, uint64_t* tag_out);

/* Snapshot lifecycle: apply one write transaction the way TransactRelationTuples does
 * (internal/persistence/sql/relationtuples.go:289-297): the inserts first (each after every equal
 * tuple, as commit_time orders them, :128-149), then the deletes (every tuple equal in namespace,
 * object, relation and subject, :200-223).  The changed rows are rewritten in the device arena in
 * place (forwards when a row outgrows its place; the tail grows on demand) and closure filters are
 * re-closed, between batches; later batches see the new version.  New Subject.String() collisions
 * (collision classes, ROW_SEQ rows) and stored subject sets with an empty field (their materialized
 * rows, re-materialized when a row they match changes) are patched in place too.  A part of an
 * edge-partitioned snapshot (KETO_PART_SHARED) takes every transaction and writes the rows it holds;
 * a migrating part takes none (KETO_E_INVALID).  An unknown namespace id fails the whole transaction
 * (KETO_E_INVALID), like GetNamespaceByName.  KETO_E_REBUILD: the write touches a poisoned row (a
 * tuple of an unconfigured namespace) or a wildcard row that matches one; the snapshot is unchanged
 * and the caller rebuilds it from the table.  Row handles (keto_row_handles,
 * keto_resolve_checks) are per version: resolve again after a write.  *version_out (may be NULL)
 * gets the new version: the snaptoken the reference leaves "not yet implemented"
 * (internal/check/handler.go:182). */
int keto_snapshot_apply(keto_snapshot* s, const keto_tuple* inserts, uint64_t n_inserts, const keto_tuple* deletes,
                        uint64_t n_deletes, uint64_t* version_out);
/* Version of the snapshot: 0 after the build, +1 per keto_snapshot_apply. */
uint64_t keto_snapshot_version(const keto_snapshot* s);

/* Edge-partitioned upload, for graphs larger than one GPU (one process per GPU, n_parts parts).
 * Takes a host-only snapshot (built with device = -1) and uploads to `device` only
 *   - every row that is the target of some subject set (these are kept on all parts), and
 *   - the root rows (rows no subject set points at) whose hash(namespace_id, object) % n_parts
 *     == part.
 * A check or expand whose top-level row is a root row must run on the part keto_row_owner names
 * (requests are routed with one all-to-all; see keto_amd/multi.py); the traversal below the top
 * level only visits rows every part holds, so each part answers exactly.  Calls naming another
 * part's root row fail with KETO_E_INVALID.  Replaces nothing in the reference. */
int keto_snapshot_upload_part(keto_snapshot* s, uint32_t part, uint32_t n_parts, int32_t device);

/* Partition modes of keto_snapshot_upload_part_mode. */
#define KETO_PART_SHARED 0      /* keto_snapshot_upload_part: set targets on every part, root rows by hash */
#define KETO_PART_MIGRATE 1     /* every row on exactly one part by hash(namespace_id, object) */
#define KETO_MIG_MAX_PARTS 30
/* Edge-partitioned upload in either mode.  KETO_PART_MIGRATE is for graphs whose set-target rows
 * (folders, groups) do not fit on one GPU either: each part holds only its own rows, plus a stub for
 * every other part's row one of its subject sets points at, and a check's DFS migrates between parts
 * at those crossings (keto_mig_begin / keto_mig_round).  After the upload the parts exchange closure
 * filters (keto_part_stubs / keto_part_filters / keto_part_close) until no filter changes anywhere,
 * then call keto_part_closure_done.  A migrating part answers checks only through keto_mig_*;
 * expand and the other check entry points fail with KETO_E_INVALID.  n_parts <= 30. */
int keto_snapshot_upload_part_mode(keto_snapshot* s, uint32_t part, uint32_t n_parts, int32_t device, uint32_t mode);
/* KETO_PART_MIGRATE with the rows most subject sets point at (the hottest in-degree bands whose rows
 * fit hot_bytes of arena) replicated on every part, at the same place: searches cross parts only on
 * the colder rows.  hot_bytes = 0 is keto_snapshot_upload_part_mode(..., KETO_PART_MIGRATE); every
 * part of one partition must be uploaded with the same hot_bytes. */
int keto_snapshot_upload_part_migrate(keto_snapshot* s, uint32_t part, uint32_t n_parts, int32_t device,
                                      uint64_t hot_bytes);
/* Arena a part of an edge-partitioned upload would hold (host-only snapshots; sizing aid):
 * arena_bytes of the part's device arena, shared_bytes of it in rows every part keeps. */
typedef struct {
    uint64_t arena_bytes;
    uint64_t shared_bytes;
    uint32_t rows;              /* rows on the part (stubs not counted) */
    uint32_t shared_rows;       /* of them: rows on every part (KETO_PART_SHARED: set targets; KETO_PART_MIGRATE:
                                   the replicated hot rows, shared_bytes their arena) */
    uint32_t root_rows;         /* of them: this part's root rows */
    uint64_t stub_rows;         /* KETO_PART_MIGRATE: stubs of other parts' rows */
} keto_part_stats;
int keto_snapshot_part_stats(keto_snapshot* s, uint32_t part, uint32_t n_parts, keto_part_stats* out);
int keto_snapshot_part_stats_mode(keto_snapshot* s, uint32_t part, uint32_t n_parts, uint32_t mode,
                                  keto_part_stats* out);

/* Closure-filter exchange of a migrating partition.  A closure filter (KETO_FILTER_WORDS words) is
 * the bloom filter of every subject id reachable from a row; a stub must carry its row's filter from
 * the owner part.  Round: every part lists its stubs (keto_part_stubs: row ids, ascending; returns
 * the count, writes at most cap), asks each stub's owner (keto_row_owner) for its current filter
 * (keto_part_filters on the owner: the filters of rows it holds, stubs included), and ORs the answers into its stubs
 * (keto_part_close, which then re-closes the part's own filters; *changed_out = filters that
 * changed).  When a round changes nothing on any part, every filter is exact: keto_part_closure_done
 * (converged = 1).  converged = 0 gives all-ones filters (no pruning; still exact answers). */
#define KETO_FILTER_WORDS 22
int64_t keto_part_stubs(const keto_snapshot* s, uint32_t* rows_out, uint64_t cap);
int keto_part_filters(keto_snapshot* s, const uint32_t* rows, uint64_t n, uint32_t* filters_out);
int keto_part_close(keto_snapshot* s, const uint32_t* stub_rows, uint64_t n, const uint32_t* filters,
                    uint64_t* changed_out);
int keto_part_closure_done(keto_snapshot* s, int converged);

/* Check batches on a migrating partition (replaces check.(*Engine).SubjectIsAllowed,
 * internal/check/engine.go:116-123, for graphs spread over several GPUs).  keto_mig_begin takes the
 * requests routed to this part (row-id form, every top-level row owned here: keto_row_owner /
 * keto_route_rows_device) and runs their searches until each is decided or crosses to another
 * part.  The crossings come back as continuation records grouped by destination part (out->units[p]
 * 16-B units at d_records + the prefix of units before p, out->records[p] records whose unit
 * offsets inside p's segment are at d_offsets + the prefix of records before p; valid until the next
 * call on this snapshot).  The caller exchanges them (one all-to-all: each part receives the
 * segments addressed to it from every source part, concatenated in source order) and passes what it
 * received to keto_mig_round (in_records[s], in_units[s] per source part s), which continues the
 * searches and emits the next records.  Decisions land in d_allowed_out (the routed batch's order)
 * of the part that began the request.  The batch is done when a round emits no record on any part.
 * Decision bytes as keto_check_batch_device (KETO_UNDECIDED: a search beyond the engine's limits). */
typedef struct {
    uint64_t units[KETO_MIG_MAX_PARTS];
    uint32_t records[KETO_MIG_MAX_PARTS];
    const void* d_records;
    const uint32_t* d_offsets;
    uint32_t decided;           /* decisions written on this part in the call */
    uint32_t undecided;         /* of the searches ended in the call: KETO_UNDECIDED */
    uint32_t processed;         /* records (requests, continuations, decisions) handled in the call */
    uint32_t reruns;            /* of them: re-run with bigger visited tables or a bigger record pool */
} keto_mig_out;
int keto_mig_begin(keto_snapshot* s, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                   uint8_t* d_allowed_out, void* stream, keto_mig_out* out);
int keto_mig_round(keto_snapshot* s, const void* d_records, const uint32_t* d_offsets, const uint32_t* in_records,
                   const uint64_t* in_units, void* stream, keto_mig_out* out);
/* Free and total device memory of HIP device `device` (hipMemGetInfo): the Go server sizes its
 * placement with it -- replicas while the replicated arena (keto_snapshot_part_stats_mode with
 * n_parts = 1) and the engine's workspaces fit every device, else shared-rows parts over the devices
 * (the reference serves any table size from one process, internal/driver/daemon.go:62-69). */
int keto_device_memory(int32_t device, uint64_t* free_out, uint64_t* total_out);
/* Device-to-device copy on `stream`, returning when it is done: for callers whose exchange layer
 * needs the records in buffers of its own (e.g. torch.distributed tensors). */
int keto_device_copy(void* dst, const void* src, uint64_t bytes, void* stream);
/* keto_check_batch_device on requests that name rows by row id (row and subject-set target), the
 * form requests travel in between parts: each is translated to this device's handles first.  A
 * request for another part's root row fails the call with KETO_E_INVALID. */
int keto_check_batch_rows_device(keto_snapshot* s, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                                 uint8_t* d_allowed_out, void* stream);
/* Owner part of each row id for n_parts parts: -1 = a row every part holds (route anywhere; a
 * KETO_PART_SHARED part's set targets).  A KETO_PART_MIGRATE part owns every row it holds. */
int keto_row_owner(const keto_snapshot* s, const uint32_t* rows, uint64_t n, uint32_t n_parts, int32_t* out);
/* Device-side routing of a row-id batch over n_parts (<= 64) parts, all buffers on one device:
 * a stable counting sort by destination part = d_owner[row] (keto_row_owner's output as int16,
 * n_rows entries), or self_part for rows every part holds, KETO_NO_ROW and out-of-range rows (the
 * destination's keto_check_batch_rows_device then rejects the latter).  Writes d_send (the n
 * requests grouped by part, batch order kept inside each part), d_order (batch index of each
 * d_send entry) and counts_out[n_parts] (host: requests per part, the all-to-all split sizes).
 * d_work: keto_route_work_bytes(n, n_parts) bytes of device scratch.  Synchronizes `stream`.
 * Replaces the host-side grouping of a partitioned batch (repo:keto_amd/multi.py). */
uint64_t keto_route_work_bytes(uint32_t n, uint32_t n_parts);
int keto_route_rows_device(const keto_check_ids* d_reqs, uint32_t n, const int16_t* d_owner, uint32_t n_rows,
                           uint32_t self_part, uint32_t n_parts, void* d_work, uint64_t work_bytes,
                           keto_check_ids* d_send, uint32_t* d_order, uint32_t* counts_out, void* stream);
/* Inverse of the routing for the decisions: d_out[d_order[j]] = d_back[j] for j < n (enqueued on
 * `stream`). */
int keto_unroute_device(const uint8_t* d_back, const uint32_t* d_order, uint32_t n, uint8_t* d_out, void* stream);
int keto_snapshot_get_stats(const keto_snapshot* s, keto_snapshot_stats* out);

/* Row ids (snapshot row order; KETO_NO_ROW passes through) -> row handles for keto_check_ids. */
int keto_row_handles(const keto_snapshot* s, const uint32_t* rows, uint64_t n, uint32_t* out);

/* Resolve named requests to device form; status_out gets KETO_CHECK_* (may be NULL). */
int keto_resolve_checks(const keto_snapshot* s, const keto_check_req* reqs, uint32_t n, keto_check_ids* out,
                        uint8_t* status_out);

/* Batched SubjectIsAllowed.  allowed_out[i] = 0/1, status_out[i] = KETO_CHECK_* (may be NULL). */
int keto_check_batch(keto_snapshot* s, const keto_check_req* reqs, uint32_t n, int32_t global_max_depth,
                     uint8_t* allowed_out, uint8_t* status_out);

/* Check requests with their strings packed back to back in one buffer, resolved on the GPU.  Request
 * i's fields start at blob + reqs[i].off: namespace, object, relation, then the subject id (kind 0)
 * or the subject set's namespace, object and relation (kind 1), with their byte lengths in
 * reqs[i].len -- the form a caller that already copies a batch's strings into one arena (the Go
 * batcher's C memory) hands over without building keto_check_req structs.  The library copies blob
 * and records to the device and resolves every request there against the snapshot's string and row
 * indexes (whereQuery, internal/persistence/sql/relationtuples.go:178-198; the indexes are uploaded
 * once per snapshot version), then checks them (check.(*Engine).SubjectIsAllowed,
 * internal/check/engine.go:116-123): decisions and statuses equal keto_check_batch's on the same
 * requests.  Requests with an empty namespace, object or relation (wildcard queries, in the subject
 * set too) are resolved on the host as keto_check_batch does.  blob_len < 2^32; fields of up to
 * 65535 bytes (longer ones: keto_check_batch).  A request whose fields lie outside the blob fails the
 * call (KETO_E_INVALID, naming the first such request) before anything is written to the outputs.
 * Large batches are pipelined (pieces of KETO_PACKED_CHUNK requests, default 2^21, uploaded while
 * earlier pieces are resolved and checked): fastest when the strings are packed in request order, as
 * the Go batcher packs them; any other layout gives the same answers after a second pass.  Pinned
 * blob and records (keto_host_alloc) let the upload run asynchronously. */
typedef struct {
    uint32_t off;               /* byte offset of the request's first field in blob */
    uint16_t len[6];            /* namespace, object, relation, subject id | set namespace, set object, set relation */
    uint8_t kind;               /* 0 = subject id (len[0..3]), 1 = subject set (len[0..5]) */
    uint8_t reserved;
    int32_t max_depth;          /* <= 0 or > global -> global (engine.go:118-120) */
} keto_check_packed;
int keto_check_batch_packed(keto_snapshot* s, const char* blob, uint64_t blob_len, const keto_check_packed* reqs,
                            uint32_t n, int32_t global_max_depth, uint8_t* allowed_out, uint8_t* status_out);

/* Same with pre-resolved requests in host memory (decision bytes as above, KETO_UNDECIDED
 * included).  Host-buffer calls run as a pipeline of chunks: the H2D copy of the next chunk and the
 * D2H copy of the previous one overlap the check of the current one.  Buffers from keto_host_alloc
 * (pinned) are copied directly; pageable ones go through the library's pinned staging. */
int keto_check_batch_ids(keto_snapshot* s, const keto_check_ids* reqs, uint32_t n, int32_t global_max_depth,
                         uint8_t* allowed_out);

/* Same with requests that name rows by row id (row, and subject-set targets): the form a caller
 * that interned names once keeps (snapshot row order, keto_row_handles' input).  Translated to
 * device handles on the device, inside the pipeline. */
int keto_check_batch_rows(keto_snapshot* s, const keto_check_ids* reqs, uint32_t n, int32_t global_max_depth,
                          uint8_t* allowed_out);

/* Compact 8-byte request of keto_check_batch_pairs: the top-level row by row id, and the subject:
 * bit31 set -> a subject set (bits 0..30 = its row id), else a subject-id string id;
 * KETO_NO_TARGET = a subject the snapshot does not know. */
typedef struct {
    uint32_t row;
    uint32_t subject;
} keto_check_pair;

/* keto_check_batch_rows for batches whose requests share one request max-depth (the usual case:
 * CheckRequest.max_depth unset -> 0 -> the global maximum): half the PCIe bytes per request. */
int keto_check_batch_pairs(keto_snapshot* s, const keto_check_pair* reqs, uint32_t n, int32_t max_depth,
                           int32_t global_max_depth, uint8_t* allowed_out);

/* Pinned (page-locked) host memory for request / decision buffers of the host-buffer calls. */
int keto_host_alloc(uint64_t bytes, void** out);
void keto_host_free(void* p);

/* Same with requests and results resident in device memory of the snapshot's device; enqueued on
 * `stream` (a hipStream_t, NULL = default stream).  Returns after enqueueing; results are ready
 * when the stream is synchronized. */
int keto_check_batch_device(keto_snapshot* s, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                            uint8_t* d_allowed_out, void* stream);

/* ---- Multi-GPU: communicators (repo:keto_amd/csrc/comm.cpp) ----
 * The exchanges of SURVEY.md 8(e) inside the library, for callers without Python (the Go server
 * process, internal/driver/daemon.go:62-69, calling check.(*Engine).SubjectIsAllowed per request,
 * internal/check/engine.go:116-123).  Every call below taking a keto_comm is collective: all ranks of
 * the communicator call it.  Errors are agreed: a rank whose own part fails (a bad argument, a
 * request it cannot route, an allocation or kernel error) still takes part in the status exchange
 * that precedes every data exchange, and every rank then returns the same code (that of the lowest
 * failing rank; keto_last_error says which rank failed), so a local error never leaves the peers
 * waiting.  Only a failing transport (RCCL, or a local rank that does not arrive within
 * KETO_COMM_TIMEOUT_MS, default 600000) returns KETO_E_HIP without agreement.
 *
 * Two transports:
 *   keto_comm_init        one process per GPU over RCCL (xGMI).  keto_comm_id makes a communicator id
 *                         on one rank; the caller hands its KETO_COMM_ID_BYTES to every rank (its own
 *                         channel), and every rank calls keto_comm_init with it.
 *   keto_comm_init_local  the ranks are threads of ONE process (one server process driving several
 *                         GPUs, or several parts on one GPU), each rank's calls made from its own
 *                         thread; the exchanges are device copies (peer copies between GPUs).  The id
 *                         is any KETO_COMM_ID_BYTES the caller chooses (the same for every rank of the
 *                         communicator, unique among the process's live local communicators). */
#define KETO_COMM_ID_BYTES 128
typedef struct keto_comm keto_comm;
int keto_comm_id(uint8_t* id_out);
int keto_comm_init(const uint8_t* id, int32_t n_ranks, int32_t rank, int32_t device, keto_comm** out);
int keto_comm_init_local(const uint8_t* id, int32_t n_ranks, int32_t rank, int32_t device, keto_comm** out);
void keto_comm_free(keto_comm* c);
/* Replicated snapshot (every rank uploaded the whole graph): every rank passes the same n named
 * requests (keto_check_batch's form); rank r decides the r-th contiguous shard, and one all-gather
 * returns all n decisions and statuses to every rank. */
int keto_check_batch_sharded(keto_comm* c, keto_snapshot* s, const keto_check_req* reqs, uint32_t n,
                             int32_t global_max_depth, uint8_t* allowed_out, uint8_t* status_out);
/* Edge-partitioned snapshot (this rank's part: keto_snapshot_upload_part_mode with part = rank and
 * n_parts = ranks): every rank passes its own batch; requests go to the parts owning their rows
 * (one all-to-all), are decided there -- on a migrating part by continuation-record rounds with an
 * all-reduce and all-to-alls per round -- and the decisions come back (a second all-to-all).  A
 * wildcard query that no stored subject set uses has no row to route by: a shared-rows part answers
 * it itself (its batch-local row from the whole graph's host tables); a migrating part sends one
 * request per matching row (each top-level tuple is searched with a fresh visited map, so the query
 * is allowed iff one of those rows is); when a page of the query's ORDER BY sequence fails, the rows
 * before that page go whole and the row it cuts one top-level tuple at a time (relationtuples.go:
 * 64-71; engine.go:98-100).  Every rank returns the same code when any rank fails. */
int keto_check_batch_routed(keto_comm* c, keto_snapshot* s, const keto_check_req* reqs, uint32_t n,
                            int32_t global_max_depth, uint8_t* allowed_out, uint8_t* status_out);
/* The same for a packed batch (the keto_check_batch_packed layout: strings back to back in
 * blob, one keto_check_packed record per request), resolved on this rank's device instead of on
 * host threads (ABI 6): the partitioned form of the Go shim's CheckBatch
 * (integration/go/internal/gpu/partition.go).  Decisions, statuses and errors as
 * keto_check_batch_routed; a request whose fields lie outside the blob fails the call on every rank. */
int keto_check_batch_routed_packed(keto_comm* c, keto_snapshot* s, const char* blob, uint64_t blob_len,
                                   const keto_check_packed* reqs, uint32_t n, int32_t global_max_depth,
                                   uint8_t* allowed_out, uint8_t* status_out);
/* BuildTree (internal/expand/engine.go:33-102) over an edge-partitioned snapshot of shared-rows
 * parts (KETO_PART_SHARED; this rank's part as above): every rank passes its own roots; a root row
 * another part owns is expanded on that part (one all-to-all of roots, one of trees), every other
 * root here, as keto_expand_batch does.  *out: one arena in request order, read with keto_tree_*
 * against this rank's snapshot.  A migrating part (KETO_PART_MIGRATE) expands every root itself: the
 * other parts' rows its trees reach are copied into the call's overlay from the host tables (which
 * every part holds whole) in rounds of the count pass; nothing is routed.  Errors are agreed as above. */
int keto_expand_batch_routed(keto_comm* c, keto_snapshot* s, const keto_expand_req* reqs, uint32_t n,
                             int32_t global_max_depth, keto_tree_arena** out);
/* A migrating partition's closure-filter exchange, once after every rank uploaded its part (before
 * the first keto_check_batch_routed; replaces the keto_part_filters / keto_part_close /
 * keto_part_closure_done loop a caller would otherwise run). */
int keto_comm_close_filters(keto_comm* c, keto_snapshot* s, uint32_t* rounds_out);

/* Device time of the last keto_check_* call on this snapshot, per tier (tier 0 = every request,
 * tiers 1/2 = requests whose visited map outgrew the previous tier's table), from HIP events on
 * the call's stream; summed over the chunks of a host-buffer call. */
typedef struct {
    float tier_ms[3];
    uint32_t requests[3];
    uint32_t undecided;         /* requests left KETO_UNDECIDED */
    uint32_t chunks;            /* host-buffer calls: pipeline chunks (0 for device calls) */
    float wall_ms;              /* host-buffer calls: entry to return, H2D + checks + D2H */
    float resolve_ms;           /* keto_check_batch: name resolution on host threads before the device part */
    float items_ms;             /* deep batches (max-depth > 9): top-level items split and pretested */
    uint32_t items;             /* deep batches: work requests (items + requests checked whole) */
    uint32_t items_kept;        /* deep batches: of them, checked after the reachability pretest */
    float index_ms;             /* deep batches: reverse / postings index (re)built for this snapshot version
                                   before the batch (host threads + upload; 0 when it was current) */
    uint32_t streamed;          /* pair batches from pinned memory: 1 = decided by the one streamed launch */
    uint32_t stream_stalls;     /* of the streamed launch: lanes whose wait for a chunk hit KETO_STREAM_WAIT_MS */
    uint32_t stream_fallbacks;  /* 1 = the streamed launch gave up (a stall) and the chunked pipeline decided */
} keto_batch_timing;
int keto_last_batch_timing(const keto_snapshot* s, keto_batch_timing* out);

/* Work counters of the traversal for a device-resident batch (instrumented kernels; same results):
 * out[0] row records read, out[1] subject-set edges scanned, out[2] subject-id words read by the
 * membership searches, out[3] visited-table probes, out[4] visited-table inserts, out[5] top-level
 * subject sets expanded (fresh visited maps).  Used for the roofline's algorithmic bytes.
 * out[6..12] are 128-B line touches per access stream (requests, row headers, edges, id tables,
 * id searches, frame pushes, frame pops): an upper bound of the kernel's L2 line traffic. */
#define KETO_WORK_SLOTS 16
/* Name of the tier-0 check kernel a batch at this global max-depth launches (as rocprofv3 prints
 * it, without the argument list), for matching profiles to bench lines.  Static storage. */
const char* keto_check_kernel_name(int32_t global_max_depth);
int keto_check_work_device(keto_snapshot* s, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                           uint8_t* d_allowed_out, uint64_t out[KETO_WORK_SLOTS]);

/* Per-request loop iterations of the check_kernel tiers (deep batches, global max-depth > 9): the
 * length of each request's serial chain of dependent steps, for its latency histogram.  d_steps:
 * n uint32 on the device (instrumented kernels, same decisions). */
int keto_check_steps_device(keto_snapshot* s, const keto_check_ids* d_reqs, uint32_t n, int32_t global_max_depth,
                            uint8_t* d_allowed_out, uint32_t* d_steps);

/* Batched BuildTree.  The arena owns all trees; free it with keto_tree_arena_free.  Its node array
 * lives in page-locked host memory from a process-wide pool (blocks are recycled by later arenas;
 * up to 1 GiB of idle blocks is kept), so keto_tree_proto_all_device uploads it in one DMA. */
int keto_expand_batch(keto_snapshot* s, const keto_expand_req* reqs, uint32_t n, int32_t global_max_depth,
                      keto_tree_arena** out);
/* Same with pre-resolved roots: roots[i] bit31 set -> subject set (bits 0..30 = row id), else a
 * subject id (bits 0..30 = string id). */
int keto_expand_batch_ids(keto_snapshot* s, const uint32_t* roots, const int32_t* max_depth, uint32_t n,
                          int32_t global_max_depth, keto_tree_arena** out);
void keto_tree_arena_free(keto_tree_arena* a);
uint32_t keto_tree_count(const keto_tree_arena* a);
int keto_tree_status(const keto_tree_arena* a, uint32_t i);
/* pre-order nodes of tree i (NULL, *n = 0 for nil / error) */
const keto_tree_node* keto_tree_nodes(const keto_tree_arena* a, uint32_t i, uint64_t* n_nodes);
/* JSON of tree i exactly as Tree.MarshalJSON (internal/expand/tree.go:156-163); "null" for nil.
 * Writes at most cap bytes (NUL-terminated) and returns the full length, or a negative code. */
int64_t keto_tree_json(const keto_snapshot* s, const keto_tree_arena* a, uint32_t i, char* buf, uint64_t cap);
/* Every tree of the arena as JSON on host threads (the REST Expand response body of each root,
 * internal/expand/handler.go:77-91, h.d.Writer().Write of the
 * BuildTree result, via Tree.MarshalJSON): offsets[n+1], tree i = buf[offsets[i],
 * offsets[i+1]) -- keto_tree_json's text for a tree, "null" for a nil tree, empty for the roots
 * keto_tree_json reports as errors (KETO_EXPAND_NOT_FOUND / KETO_EXPAND_UNDECIDED).  buf is written
 * only if cap >= the total, which is returned (call with buf = NULL to size it).  A sizing call
 * keeps its encodings in the arena until the filling call (or keto_tree_arena_free), so the pair
 * encodes once; keto_tree_proto_all does the same. */
int64_t keto_tree_json_all(const keto_snapshot* s, const keto_tree_arena* a, char* buf, uint64_t cap,
                           uint64_t* offsets);

/* Tree i as acl.SubjectTree protobuf bytes, exactly as proto.Marshal(Tree.ToProto())
 * (internal/expand/tree.go:165-188; proto/ory/keto/acl/v1alpha1/expand_service.proto): the
 * gRPC Expand response's `tree`.  Writes min(cap, size) bytes, returns the size (0 for a nil tree,
 * which the reference sends as an unset field), or a negative code. */
int64_t keto_tree_proto(const keto_snapshot* s, const keto_tree_arena* a, uint32_t i, uint8_t* buf, uint64_t cap);
/* Every tree of the arena encoded on host threads: offsets[n+1] (tree i = buf[offsets[i],
 * offsets[i+1]), empty for nil / error trees); buf is written only if cap >= the total, which is
 * returned (call with buf = NULL to size it). */
int64_t keto_tree_proto_all(const keto_snapshot* s, const keto_tree_arena* a, uint8_t* buf, uint64_t cap,
                            uint64_t* offsets);
/* keto_tree_proto_all encoded on the GPU from the arena's nodes and the snapshot's strings (uploaded
 * to the snapshot's device on first use): the same bytes and offsets.  offsets
 * is always written; buf only when cap >= the returned total (call with buf = NULL to size it).
 * The call's device buffers stay with the snapshot for the next call (freed with its device
 * state); a pinned (hipHostMalloc'd) buf takes one DMA, a pageable one two pinned bounce chunks. */
int64_t keto_tree_proto_all_device(keto_snapshot* s, const keto_tree_arena* a, uint8_t* buf, uint64_t cap,
                                   uint64_t* offsets);

/* The fields of subject references as keto_tree_node.subject holds them, for building expand.Tree
 * values (internal/expand/tree.go:26-30: relationtuple.SubjectID / SubjectSet,
 * internal/relationtuple/definitions.go:40-42,102-117) straight from the node arena without a text
 * codec.  a: the arena the references come from (its batch-local wildcard roots and subject ids the
 * snapshot does not know), or NULL.  Reference i: lens_out[3i..3i+2] = (id length, 0, 0) for a subject
 * id, (namespace, object, relation lengths) for a subject set; the strings follow one another in buf
 * in that order.  buf is written only if cap >= the total byte count, which is returned (call with
 * buf = NULL to size it; the count of a reference never changes, so a size-then-fill pair agrees
 * even across keto_snapshot_apply). */
int64_t keto_subject_fields(const keto_snapshot* s, const keto_tree_arena* a, const uint32_t* subjects, uint64_t n,
                            char* buf, uint64_t cap, uint32_t* lens_out);

/* String of a subject reference used in keto_tree_node.subject (Subject.String(), definitions.go:163-169). */
int64_t keto_subject_string(const keto_snapshot* s, uint32_t subject, char* buf, uint64_t cap);

#ifdef __cplusplus
}
#endif

#endif /* KETO_MI355X_H */
