// Internal snapshot representation shared by the host builder (snapshot.cpp), the device
// engine (engine.hip) and the C-ABI (capi.cpp).
//
// Host tables: rows (RowRec: edge range, flags, effective set / id counts), edges (bit31 = subject
// set, bits 0..30 = target row id; else a subject id = string id), row_pp (first poisoned page,
// expand only) and coll (visit ids of colliding Subject.String() keys).  The device arena built
// from them is described at HDR_WORDS below.
//
// A "normal" row stores its effective (check) edges as [subject sets in ORDER BY order]
// [subject ids sorted by string id == byte order], so a check finds the requested subject id by
// membership.  A ROW_SEQ row (materialized wildcard query, or a row holding an edge whose
// Subject.String() collides with another subject's) keeps the exact ORDER BY sequence and is
// walked edge by edge with full visited semantics.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <type_traits>
#include <utility>
#include <unordered_map>
#include <vector>

#include "../../include/keto_mi355x.h"

#if defined(__HIP__)
#define KETO_HD __host__ __device__
#else
#define KETO_HD
#endif

namespace keto {

constexpr uint32_t EDGE_SET = 0x80000000u;
constexpr uint32_t EDGE_VAL = 0x7FFFFFFFu;
constexpr uint32_t EDGE_POISON = 0x7FFFFFFFu;   // a row whose toInternal fails; never traversed
constexpr uint32_t NO_PAGE = 0xFFFFFFFFu;
constexpr uint32_t NO_UNIT = 0xFFFFFFFFu;         // row not on this device (edge partitioning)
constexpr uint32_t ANY = 0xFFFFFFFFu;           // wildcard field of a row key
constexpr int64_t ANY_NS = INT64_MIN;
constexpr uint32_t ROW_SEQ = 1u;                // flag bit (in RowRec.y bits 8..15)
constexpr uint32_t VID_CLASS = 0x80000000u;     // visit ids of colliding keys live above all row ids
// keto_check_ids.flags bit of the engine's own top-level items (reach.hip; not part of the C-ABI,
// honoured only for the work arrays reach.hip builds)
constexpr uint32_t KETO_ITEM_FLAG = 2u;
// keto_check_ids.flags bit of a migrating batch's requests for one top-level tuple of a wildcard
// query (comm.cpp routed_check): enter `row` as the walk does after the hop from that tuple, the map
// holding the tuple's visit key (bits 8..31: its collision class + 1, or 0 for the row's own key).
// Honoured only where comm.cpp builds them (mig_begin(..., child_entries = true)).
constexpr uint32_t KETO_CHILD_FLAG = 4u;

// Device arena (one u32 array per device).  Row r occupies
//   [subject-id table, 2^hlog2 words of 16-B buckets, for rows whose ids do not all fit in the
//    window (n_ids > 0 and n_sets + n_ids > WINDOW_WORDS)]
//   [closure filter (CF_WORDS) + child signatures (SIG_WORDS): CB_WORDS words, only for rows
//    some subject set points at (HDR_CLOSURE)]
//   [16-B header: n_sets, n_ids, flags | hlog2 << 8 | bloom, bloom]   <- handle = word / 4
//   [edges in ORDER BY order; subject sets hold the target's handle]  padded to 16 B
// A row visit reads the header and the window (the first 4 edge words) -- and, entering a subject
// set, one word of its closure filter -- from one 128-B line: closure filter, header and window
// never straddle a line, and a row that fits in a line is placed in a single line, so its id table
// is in the line the header came in with.
constexpr uint32_t HDR_WORDS = 4;
constexpr uint32_t WINDOW_WORDS = 4;            // edge words read together with the header
constexpr uint32_t LINE_WORDS = 32;             // 128-B cache line
constexpr uint32_t BUCKET_WORDS = 4;            // id tables are probed one 16-B bucket at a time
// The arena is segments of 2^32 words (16 GiB each, up to four in a narrow layout, 64 GiB in all); no
// row (id table to last edge) crosses from one to the next, so a position inside a row is a 32-bit
// word index within its segment.  A narrow handle (a 16-B unit, 32 bits) lies in segment
// handle >> SEG_SHIFT; a wide one in segment hword(handle, g) >> 32.
//
// Edges hold a subject set's handle in 31 bits, so every row some subject set points at (a
// target) has a handle below 2^31 (the first 32 GiB); root rows -- rows no subject set points at,
// reached only as a request's row -- may lie anywhere below 2^32 - 16.  The layout puts targets
// first anyway (hottest first, roots last); when the arena outgrows 2^33 words it leaves a reserve
// for the targets later writes add between the targets and the roots ("split" layout:
// [0, tgt_tail) targets, [tgt_tail, tgt_end) reserve, [roots_at >= tgt_end, ...) roots).
constexpr uint32_t SEG_SHIFT = 30;
constexpr uint32_t SEG_MASK = (1u << SEG_SHIFT) - 1u;
constexpr uint64_t NARROW_MAX_WORDS = 1ull << 34;     // every handle a 16-B unit: up to 64 GiB
constexpr uint64_t TARGET_MAX_WORDS = 1ull << 33;     // target rows' headers lie below this word
constexpr uint32_t HANDLE_MAX = 0xFFFFFFF0u;          // handles (and overlay handles) stay below
// Wide arenas (past 64 GiB, round 6): a handle below 2^31 is still a 16-B unit (every target, and the
// roots laid out below word 2^33), but a handle h >= 2^31 names a root row whose header lies at word
// 2^33 + ((h - 2^31) << (2 + g)): root rows past 32 GiB are addressed in units of 16 << g bytes (their
// headers aligned so), g = Snapshot::root_g in 1..ROOT_G_MAX, the smallest that gives every root a
// handle.  Only a request's own row (the top frame of a search, or a tree's root) is ever a root, so
// only the request start decodes such a handle; g = 0 is the narrow layout (hword(h, 0) = 4 h).
// Segments stay 2^32 words (no row crosses one); up to 18 of them.
constexpr uint32_t ROOT_G_MAX = 3;
constexpr uint64_t ARENA_MAX_WORDS = TARGET_MAX_WORDS + (1ull << (33 + ROOT_G_MAX));   // 288 GiB
KETO_HD inline uint64_t hword(uint32_t h, uint32_t g) {
    return h < 0x80000000u ? (uint64_t)h * 4u : TARGET_MAX_WORDS + ((uint64_t)(h - 0x80000000u) << (2u + g));
}
// the handle of a header at word w (w a multiple of 4 below 2^33, else of 4 << g past it)
KETO_HD inline uint64_t handle_at_word(uint64_t w, uint32_t g) {
    return w < TARGET_MAX_WORDS || g == 0 ? w / 4u : 0x80000000ull + ((w - TARGET_MAX_WORDS) >> (2u + g));
}
// the first handle past an arena of w words (every header of it has a smaller one)
KETO_HD inline uint64_t handle_end(uint64_t w, uint32_t g) {
    return w <= TARGET_MAX_WORDS || g == 0 ? (w + 3u) / 4u
                                           : 0x80000000ull + ((w - TARGET_MAX_WORDS + (4ull << g) - 1u) >> (2u + g));
}
// header word 2: bits 0..7 flags, 8..12 hlog2, 13..31 bloom bits 32..50; word 3: bloom bits 0..31.
// The 51-bit bloom filter (2 bits per subject id) summarizes the ids of a row with an id table,
// so most absent ids are rejected with the header and the table is never probed for them.
constexpr uint32_t HDR_SEQ = 1u;                // walked edge by edge (ROW_SEQ)
constexpr uint32_t HDR_POISON = 2u;             // some page fails toInternal (expand: error)
constexpr uint32_t HDR_POISON0 = 4u;            // the first page fails (check: empty row)
constexpr uint32_t HDR_CLOSURE = 8u;            // a closure filter precedes the header
// A row rewritten by a write that no longer fits its place (delta.cpp / device_apply) lives at the
// arena's tail; its identity header (whose handle every subject set holds, and whose closure filter
// stays in front of it) becomes a forward: word 0 = handle of the row's current header.
constexpr uint32_t HDR_FWD = 16u;
// Migrating partition (PART_MIGRATE): a stub stands for a row another part owns that some set edge
// of this part points at.  It is a closure block (the remote row's closure filter, filled in by
// the filter exchange) and a header {owner part, handle on the owner, HDR_REMOTE | HDR_CLOSURE, 0}
// with no edges; a walk that enters it continues on the owner (migrate.hip).
constexpr uint32_t HDR_REMOTE = 32u;
// upload modes of an edge-partitioned snapshot (keto_snapshot_upload_part_mode)
constexpr int PART_SHARED = 0;    // rows some set points at on every part, root rows by hash
constexpr int PART_MIGRATE = 1;   // every row on one part by hash, stubs for remote set targets
constexpr uint32_t MIG_MAX_PARTS = 30;   // visit-id part field: 0..29 parts, 30 replicated rows, 31 classes
// Closure filter of a row some subject set points at: a 704-bit, one-hash bloom filter of every
// subject id reachable from the row through any number of subject sets (its own ids included).  A
// check entering such a row for a requested id the filter rules out skips the row: every node the
// skipped search would have marked visited lies inside that closure, which never reaches the
// requested id, so no answer changes (rows whose closure holds a colliding visit key, ROW_SEQ,
// have all bits set).  Built on the device at upload (closure_pass).
//
// Child signatures (the last SIG_WORDS words in front of a closure row's header): for each of the
// row's 4 window slots, the 16-bit OR-fold of the closure filter of the subject set in that slot
// (fold bit b = some filter bit p with p % 16 == b is set; all ones for a slot holding no subject
// set).  T sits at filter bit p, so fold bit p % 16 clear means the child's own filter rules T out:
// a walk inside this row skips that child without loading its line, exactly as the child's filter
// word would have.  Stored transposed so one word serves all 4 slots: word (b >> 3) bit
// ((b & 7) * 4 + slot) = fold bit b of that slot.  Built on the device after the filters are
// closed (sig_pass); all ones until then (no skip).
constexpr uint32_t CF_WORDS = 22;               // closure filter: 704 bits
constexpr uint32_t SIG_WORDS = 2;
constexpr uint32_t CB_WORDS = CF_WORDS + SIG_WORDS;   // in front of a closure row's header
KETO_HD inline void closure_bit(uint32_t id, uint32_t& word, uint32_t& bit) {
    uint32_t h = id * 0x85EBCA77u + 0x165667B1u;
    h ^= h >> 13;
    h *= 0xC2B2AE3Du;
    h ^= h >> 16;
    const uint32_t p = (uint32_t)(((uint64_t)h * (CF_WORDS * 32u)) >> 32);
    word = p >> 5;
    bit = p & 31u;
}
constexpr uint32_t BLOOM_BITS = 51;
KETO_HD inline void bloom_bits(uint32_t id, uint32_t& b1, uint32_t& b2) {
    uint32_t h = id * 0x9E3779B1u + 0x7F4A7C15u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    h *= 0x297A2D39u;
    h ^= h >> 15;
    b1 = (h & 0xFFFFu) % BLOOM_BITS;
    b2 = (h >> 16) % BLOOM_BITS;
}
// is bit b of the (word2, word3) bloom set?
KETO_HD inline bool bloom_has(uint32_t w2, uint32_t w3, uint32_t b) {
    return b < 32 ? ((w3 >> b) & 1u) : ((w2 >> (b - 32 + 13)) & 1u);
}

struct RowRec {          // 16 B
    uint32_t edge_lo;    // edge begin, low 32 bits
    uint32_t hi_flags;   // bits 0..7 edge begin bits 32..39; bits 8..15 flags
    uint32_t n_sets;     // normal: effective subject sets; ROW_SEQ: effective edge count
    uint32_t n_ids;      // normal: effective subject ids;  ROW_SEQ: 0
};
static_assert(sizeof(RowRec) == 16, "RowRec must be 16 bytes");

struct RowKey {          // (namespace id | ANY, object string | ANY, relation string | ANY)
    int64_t ns;
    uint32_t obj, rel;
    bool operator==(const RowKey& o) const { return ns == o.ns && obj == o.obj && rel == o.rel; }
};
struct RowKeyHash {
    size_t operator()(const RowKey& k) const {
        uint64_t h = (uint64_t)k.ns * 0x9E3779B97F4A7C15ull;
        h ^= (uint64_t)k.obj * 0xC2B2AE3D27D4EB4Full + (h << 6) + (h >> 2);
        h ^= (uint64_t)k.rel * 0x165667B19E3779F9ull + (h << 6) + (h >> 2);
        return (size_t)h;
    }
};

struct DeviceState;      // engine.hip
struct DeviceStateDeleter {
    void operator()(DeviceState* d) const;   // engine.hip
};
struct MigState;         // migrate.hip
struct MigStateDeleter {
    void operator()(MigState* m) const;      // migrate.hip
};
struct ProtoState;       // proto.hip
struct ProtoStateDeleter {
    void operator()(ProtoState* p) const;    // proto.hip
};
struct ReachState;       // reach.hip
struct ReachStateDeleter {
    void operator()(ReachState* r) const;    // reach.hip
};
struct RDevState;        // resolve_dev.hip
struct RDevStateDeleter {
    void operator()(RDevState* r) const;     // resolve_dev.hip
};

uint64_t next_snapshot_uid();   // snapshot.cpp: a process-wide counter

// The snapshot's reader / writer lock, writer-preferring: a waiting writer holds the turnstile
// every reader passes before it takes the lock shared, so a stream of overlapping batches cannot
// keep keto_snapshot_apply waiting forever (std::shared_mutex on glibc lets readers in while a writer
// waits).  A thread never takes it shared twice, and never waits for another thread's call on the
// same snapshot while it holds it.
struct RwGate {
    std::shared_mutex m;
    std::mutex gate;
    void lock() {
        std::lock_guard<std::mutex> g(gate);
        m.lock();
    }
    bool try_lock() { return m.try_lock(); }
    void unlock() { m.unlock(); }
    void lock_shared() {
        { std::lock_guard<std::mutex> g(gate); }
        m.lock_shared();
    }
    bool try_lock_shared() { return m.try_lock_shared(); }
    void unlock_shared() { m.unlock_shared(); }
};

// A table that grows without moving its elements: fixed chunks of 2^SHIFT, so appending under the
// snapshot's exclusive lock costs the appended elements (and a new chunk now and then), never a copy
// of the whole table -- a std::vector of the 1B-tuple graph's ~220M strings moved 7 GB on the first
// write that added a string, blocking every batch for ~2 s (profiles/r05aj_apply_1b_readers.log).
template <class T, unsigned SHIFT = 16>
struct Chunked {
    static constexpr uint64_t CH = 1ull << SHIFT;
    Chunked() = default;
    Chunked(const Chunked& o) { *this = o; }
    Chunked(Chunked&&) noexcept = default;
    Chunked& operator=(Chunked&&) noexcept = default;
    Chunked& operator=(const Chunked& o) {
        if (this == &o) return *this;
        resize(0);
        resize(o.n);
        for (uint64_t c = 0; c < o.chunks.size(); ++c)
            std::copy(o.chunks[c].get(), o.chunks[c].get() + std::min(CH, o.n - c * CH), chunks[c].get());
        return *this;
    }
    uint64_t size() const { return n; }
    bool empty() const { return n == 0; }
    T& operator[](uint64_t i) { return chunks[i >> SHIFT][i & (CH - 1)]; }
    const T& operator[](uint64_t i) const { return chunks[i >> SHIFT][i & (CH - 1)]; }
    void resize(uint64_t m) {
        for (uint64_t i = m; i < n && (i & (CH - 1)); ++i) (*this)[i] = T();   // the kept chunk's tail
        chunks.resize((m + CH - 1) >> SHIFT);
        for (auto& c : chunks)
            if (!c) c.reset(new T[CH]());
        n = m;
    }
    void push_back(T&& x) {
        if (n == chunks.size() * CH) chunks.emplace_back(new T[CH]());
        (*this)[n++] = std::move(x);
    }

   private:
    std::vector<std::unique_ptr<T[]>> chunks;
    uint64_t n = 0;
};

struct Snapshot {
    const uint64_t uid = next_snapshot_uid();   // never reused (caches keyed by snapshot use it, not its address)
    // ---- config
    std::vector<int32_t> ns_ids;
    std::vector<std::string> ns_names;
    std::unordered_map<std::string, int> ns_by_name;   // name -> config index
    std::unordered_map<int32_t, int> ns_by_id;         // id   -> config index
    uint32_t page_size = 100;

    // ---- strings (byte order == id order)
    Chunked<std::string> strs;
    uint32_t empty_str = ANY;                                // id of "" if present

    // ---- rows
    uint32_t n_real_rows = 0;
    uint32_t n_wild_rows = 0;
    std::vector<uint32_t> wild_rows;                         // the wildcard rows (keys with an ANY field)
    std::vector<RowKey> row_key;                             // per row
    std::unordered_map<RowKey, uint32_t, RowKeyHash> row_of; // real + empty + wildcard rows
    std::vector<RowRec> rows;
    std::vector<uint32_t> row_pp;
    std::vector<uint32_t> edges;
    std::vector<uint8_t> row_has_coll;

    // ---- visit-key collisions
    std::unordered_map<uint32_t, uint32_t> coll;             // edge value -> visit id
    uint32_t n_coll_keys = 0;
    bool coll_dirty = false;                                 // a write added classes: the device table follows

    uint64_t n_tuples = 0;
    uint32_t n_poisoned_rows = 0;
    uint32_t n_seq_rows = 0;

    // ---- device arena layout (compute_layout): handle of each row, total arena units (16 B)
    std::vector<uint32_t> unit_of_row;    // NO_UNIT: a root row another part owns (not on this device)
    std::vector<uint32_t> rows_by_unit;   // rows in arena order (most-referenced first)
    std::vector<uint32_t> layout_units;   // their units, increasing
    // split layout (arenas past 2^33 words, see SEG_SHIFT): the target reserve [tgt_tail, tgt_end)
    // in words, filled by writes from tgt_tail up, and the first root row's word roots_at (>=
    // tgt_end); tgt_end == 0: not split
    uint64_t tgt_tail = 0, tgt_end = 0, roots_at = 0;
    // edge partitioning (keto_snapshot_upload_part): rows that are some subject set's target are
    // kept on every part; root rows (never a subject set) only on part hash(ns, object) % n_parts
    std::vector<uint8_t> is_root;
    uint32_t part = 0, n_parts = 1;
    int part_mode = PART_SHARED;
    uint32_t root_owner(uint32_t r, uint32_t parts) const;   // hash(namespace id, object) % parts
    // owner of row r under this snapshot's partitioning: -1 = on every part (PART_SHARED non-root rows)
    int32_t row_owner(uint32_t r, uint32_t parts) const {
        return (part_mode == PART_MIGRATE || is_root[r]) ? (int32_t)root_owner(r, parts) : -1;
    }
    // PART_MIGRATE: stub[r] = r is another part's row with a stub here; g_handle[r] = r's handle on its
    // owner part (every row), for the request translation of set targets and for the stubs
    std::vector<uint8_t> stub;
    std::vector<uint32_t> g_handle;
    uint64_t n_stubs = 0;
    // PART_MIGRATE: the rows most subject sets point at are replicated on every part, hottest first, up
    // to hot_bytes of arena; they form the identical prefix [0, hot_units) of every part's arena
    uint64_t hot_bytes = 0;
    uint32_t hot_units = 0;
    uint64_t hot_rows = 0;
    // PART_MIGRATE: closure filters final (part_closure_done, or one part); atomic: read by batches under
    // the shared lock while a filter exchange (exclusive lock) or a write resets it
    std::atomic<bool> mig_ready{false};
    // r is held by this device (owned, or on every part); stubs are not rows of this part
    bool present(uint32_t r) const { return unit_of_row[r] != NO_UNIT && (stub.empty() || !stub[r]); }
    bool mapped(uint32_t r) const { return unit_of_row[r] != NO_UNIT; }   // a row or a stub here
    uint64_t n_units = 0;                 // handle end: every row's handle is below (overlay handles start here)
    uint64_t n_words = 0;                 // arena words laid out (== 4 n_units in a narrow layout)
    uint32_t root_g = 0;                  // wide layouts: root handles past 2^31 count 16 << root_g bytes (hword)
    uint64_t hdr_word(uint32_t h) const { return hword(h, root_g); }
    uint64_t shared_words = 0;            // arena words of the rows every part keeps (non-root rows)
    uint32_t handle(uint32_t row) const { return unit_of_row[row]; }
    int64_t row_of_handle(uint32_t unit) const;   // -1 if not a row header
    uint32_t row_hlog2(uint32_t r) const;         // 0 = no id table

    // ---- lifecycle (delta.cpp): writes applied since the build
    RwGate rw;                                 // calls read the host tables shared; keto_snapshot_apply exclusive
    std::mutex apply_mu;                       // one keto_snapshot_apply at a time (it stages under rw shared)
    std::atomic<uint64_t> version{0};          // bumped by every keto_snapshot_apply (read without the lock)
    uint32_t n_sorted_strs = 0;                // strs[0, n) are in byte order (id = rank); later ones were added
    std::unordered_map<std::string, uint32_t> added_str;
    uint32_t n_base_rows = 0;                  // rows of the build; rows >= n_base_rows were added by writes
    std::unordered_map<uint32_t, std::vector<uint32_t>> row_over;   // current edges of rows changed by writes
    std::vector<uint8_t> row_cb;               // the row's identity handle has a closure filter in front of it
    struct RowPlace {                          // where a changed row's content is (device arenas)
        uint32_t unit;                         // its header (== identity handle unless forwarded)
        uint32_t hlog2;
        uint64_t edge_cap;                     // edge words the place holds
        bool cb;                               // a closure filter precedes that header
    };
    std::unordered_map<uint32_t, RowPlace> row_place;
    std::vector<uint32_t> dirty;               // rows the last apply changed (device_apply's work list)
    std::vector<uint32_t> needs_cb;            // of them: rows that became subject-set targets without a filter
    std::vector<std::shared_ptr<void>> retired;   // tables a commit replaced: freed after the exclusive lock
    // edges of row r in ORDER BY order (row-id encoded), whether or not a write changed it
    std::pair<const uint32_t*, uint64_t> row_edges(uint32_t r) const {
        auto it = row_over.find(r);
        if (it != row_over.end()) return {it->second.data(), it->second.size()};
        if (r >= n_base_rows) return {nullptr, 0};
        const uint64_t b = row_begin(r), e = r + 1 < n_base_rows ? row_begin(r + 1) : edges.size();
        return {edges.data() + b, e - b};
    }
    int str_cmp(uint32_t a, uint32_t b) const;    // byte order of two string ids
    int key_cmp_bytes(const RowKey& a, const RowKey& b) const;   // (namespace id, object bytes, relation bytes)
    // rows a (wildcard) RelationQuery k returns, in the reference ORDER BY (relationtuples.go:250)
    std::vector<uint32_t> rows_in_key_order(const RowKey& k) const;

    std::atomic<float> last_resolve_ms{0};     // keto_check_batch: name resolution of the last batch (diagnostic)

    // ---- device
    int device = -1;
    std::unique_ptr<DeviceState, DeviceStateDeleter> dev;
    std::unique_ptr<MigState, MigStateDeleter> mig;      // migrating-partition batches (migrate.hip)
    std::unique_ptr<ProtoState, ProtoStateDeleter> proto; // strings on the device for tree encoding (proto.hip)
    std::unique_ptr<ReachState, ReachStateDeleter> reach; // reverse / postings index of deep batches (reach.hip)
    std::unique_ptr<RDevState, RDevStateDeleter> rdev;    // string / row indexes on the device (resolve_dev.hip)
    std::mutex mu;

    ~Snapshot();

    uint64_t row_begin(uint32_t r) const {
        return (uint64_t)rows[r].edge_lo | ((uint64_t)(rows[r].hi_flags & 0xFFu) << 32);
    }
    uint32_t row_flags(uint32_t r) const { return (rows[r].hi_flags >> 8) & 0xFFu; }
    uint32_t n_rows() const { return (uint32_t)rows.size(); }

    // ---- request resolution (resolve.cpp): flat open-addressing indexes over the build's strings
    // (byte-order ids, strs[0, n_sorted_strs)) and its real rows (row_key[0, n_real_rows)), both fixed
    // after the build, so they are built once, on the first lookup; writes add strings and rows to
    // added_str / row_of, which the lookups consult after the index.  16-B slots carry what verifies a
    // hit (a string's length and first 11 bytes, a row's whole key), so a short string or a row is
    // matched without reading strs / row_key; tables are huge-page mappings (one TLB entry per 2 MB).
    struct HugeBuf {                                // anonymous zero-filled mapping, THP requested
        void* p = nullptr;
        uint64_t bytes = 0;
        HugeBuf() = default;
        HugeBuf(const HugeBuf&) = delete;
        HugeBuf& operator=(const HugeBuf&) = delete;
        ~HugeBuf();
        void alloc(uint64_t bytes);
    };
    struct StrSlot {                                // id + 1 (0 = empty), length (255: >= 255), leading bytes
        uint32_t id1;
        uint8_t n;
        char b[11];
    };
    struct RowSlot {                                // the row's key and row + 1 (0 = empty)
        int32_t ns;
        uint32_t obj, rel, row1;
    };
    mutable HugeBuf str_idx, row_idx;
    mutable uint64_t str_mask = 0, row_mask = 0;
    mutable std::once_flag idx_once;
    void ensure_index() const;
    std::unordered_map<std::string_view, int> ns_view;   // name -> config index (views into ns_names)
    int ns_index(std::string_view name) const;           // config index, -1 if unknown
    int64_t real_row(const RowKey& k) const;             // real row of a complete key, -1 if none
    // lookups used by request resolution
    int64_t lookup_str(std::string_view s) const;                      // -1 if absent
    // RelationQuery (namespace name, object, relation) -> row, per whereQuery; returns
    //  >=0 row id, -1 no such row (empty result), -2 unknown namespace (NotFound),
    //  -3 a wildcard query no stored subject set materialized (*key_out is set)
    int64_t resolve_query(std::string_view ns, std::string_view obj, std::string_view rel,
                          RowKey* key_out = nullptr) const;
    // visit id of a Subject.String() key that names no snapshot row: the row sharing the key
    // (if any), else 0xFFFFFFF0 (no snapshot subject has it)
    uint32_t vid_of_key(std::string_view key) const;
    // the rows (subject sets) whose Subject.String() is `key` ("ns:obj#rel"; fields may contain ':'
    // and '#', so every split is tried against the namespaces, strings and row indexes)
    std::vector<uint32_t> rows_of_string(std::string_view key) const;
    uint32_t vid_of_row(uint32_t row) const;
    std::string subject_string(uint32_t subject_ref) const;
    std::string row_field_ns(uint32_t row) const;
    std::string row_field(uint32_t row, int which) const;               // 1 obj, 2 rel
};

// builders (snapshot.cpp); throw keto::Error
struct Error {
    int code;
    std::string msg;
};

// named check requests [b, e) -> device form (resolve.cpp; the role of whereQuery,
// internal/persistence/sql/relationtuples.go:178-198): out[i], status[i] (KETO_CHECK_*), and for a
// wildcard query that no stored subject set materialized an entry {i, its key} appended to `wild`
// (out[i].row is then KETO_NO_ROW until the caller gives it a batch-local row).  Throws
// KETO_E_INVALID for a top-level row another part owns.  by_row: rows (and subject-set targets)
// by row id instead of this device's handles, for requests routed to the part owning their row
// (comm.cpp); no ownership check.
struct WildReq {
    uint32_t i;
    RowKey key;
};
void resolve_checks(const Snapshot& S, const keto_check_req* q, uint64_t b, uint64_t e, keto_check_ids* out,
                    uint8_t* status, std::vector<WildReq>& wild, bool by_row = false);

std::unique_ptr<Snapshot> build_snapshot(const keto_namespace* ns, uint32_t n_ns, const keto_tuple* t, uint64_t n,
                                         uint32_t page_size);
std::unique_ptr<Snapshot> build_snapshot_csr(const keto_namespace* ns, uint32_t n_ns, uint32_t n_rows,
                                             const int32_t* row_ns, const uint32_t* row_obj,
                                             const uint32_t* row_rel, const uint64_t* row_ptr,
                                             const uint32_t* edges, const keto_str* strings, uint32_t n_strings,
                                             uint32_t page_size);

// host copy of an unpartitioned snapshot at its current version, laid out afresh (snapshot.cpp)
std::unique_ptr<Snapshot> clone_host(const Snapshot& s);
// persist.cpp: the host tables of an unpartitioned snapshot to / from one file (keto_snapshot_save /
// keto_snapshot_load); the loaded snapshot is laid out afresh, as a clone is
void save_snapshot(const Snapshot& s, const char* path, uint64_t tag);
std::unique_ptr<Snapshot> load_snapshot(const char* path, uint64_t* tag_out);

// Batch-local rows for wildcard requests that no stored subject set materialized: they can only
// be top-level (check) or root (expand) rows, never edge targets.  Row ids >= base.
struct Overlay {
    uint32_t base = 0;                 // row ids >= base are overlay rows (host side)
    std::vector<RowRec> rows;
    std::vector<uint32_t> pp;
    std::vector<uint32_t> edges;       // row-id encoded like Snapshot::edges
    std::vector<RowKey> keys;
    std::unordered_map<RowKey, uint32_t, RowKeyHash> map;
    std::vector<uint32_t> unit;        // overlay-local arena unit of each overlay row
    uint64_t n_units = 0;
    bool empty() const { return rows.empty(); }
};
// materialize the wildcard query k (ns ANY / obj ANY / rel ANY) into the overlay; returns row id
uint32_t overlay_row(const Snapshot& s, Overlay& ov, const RowKey& k);
// device handle of a row id that may be an overlay row (handles >= s.n_units are overlay rows)
uint32_t handle_of(const Snapshot& s, const Overlay* ov, uint32_t row);
// arena layout of every row (called by the builders)
void compute_layout(Snapshot& s);
// arena placement of one row (compute_layout, device_apply): the first word at or after w where a
// row of `table` id-table words, `cb` closure-block words and n_edges edges keeps the line and
// segment rules; total = the row's words from there
uint64_t arena_fit(uint64_t w, uint64_t table, uint64_t cb, uint64_t n_edges, uint64_t& total);
// the same, with a wide layout's header alignment past word 2^33 (root_g = g, see hword)
uint64_t arena_fit_g(uint64_t w, uint64_t table, uint64_t cb, uint64_t n_edges, uint64_t& total, uint32_t g);
// snapshot lifecycle (delta.cpp): apply an insert / delete transaction to the host tables
// (TransactRelationTuples, internal/persistence/sql/relationtuples.go:289-297); throws KETO_E_REBUILD
// for writes outside the delta path; device_apply then patches the device arena
// commit: called once the transaction is staged (every check passed, nothing of the snapshot changed
// yet) and before it changes anything; keto_snapshot_apply stages under the shared lock and takes the
// exclusive one there, so batches run while a write is staged
void apply_writes(Snapshot& s, const keto_tuple* ins, uint64_t n_ins, const keto_tuple* del, uint64_t n_del,
                  const std::function<void()>& commit = {});
void device_apply(Snapshot& s);

// device engine (engine.hip)
void device_upload(Snapshot& s, int device);
void device_release(Snapshot& s);
uint64_t device_bytes(const Snapshot& s);
// device-resident requests and decisions, enqueued on `stream` (NULL: the snapshot's own)
void device_check(Snapshot& s, const keto_check_ids* d_reqs, uint32_t n, int32_t gmd, uint8_t* d_allowed, void* stream,
                  uint64_t* work_out = nullptr, uint32_t* d_steps = nullptr);
// host buffers: pipelined chunks (H2D / check / D2H overlapped); form FORM_* (keto_check_ids by
// handle or by row id, 8-B keto_check_pair by row id with one request depth); ov = batch-local
// wildcard rows
constexpr int FORM_HANDLES = 0, FORM_ROWS = 1, FORM_PAIRS = 2;
void device_check_host(Snapshot& s, const void* reqs, uint32_t n, int32_t gmd, uint8_t* allowed, int form,
                       int32_t pair_depth, const Overlay* ov);
keto_batch_timing device_last_timing(const Snapshot& s);
// requests with row ids (not handles) resident on the device: translated, then checked.  rows_valid:
// every row id is one this part holds (the packed path's own resolution on an unpartitioned
// snapshot), so the misrouted-row count is not read back (a host round trip fewer)
void device_check_rows(Snapshot& s, const keto_check_ids* d_reqs, uint32_t n, int32_t gmd, uint8_t* d_allowed,
                       void* stream, bool rows_valid = false);
// requests already in the handle form, checked without a host round trip: enqueued after `ready`,
// `done` recorded when the decisions are in d_allowed; d_counts[0]: tier-0 overflows (> 0: check the
// batch again with device_check_rows).  false: not taken (deep batch or a partitioned snapshot)
bool device_check_rows_async(Snapshot& s, const keto_check_ids* d_handles, uint32_t n, int32_t gmd,
                             uint8_t* d_allowed, uint32_t* d_counts, void* ready_event, void* done_event);
// the device row id -> handle map (NO_UNIT: a row this part does not hold); valid while the caller
// holds the snapshot lock
const uint32_t* device_row_handle_map(Snapshot& s);
const char* device_check_kernel_name(int32_t gmd);
// deep batches (reach.hip): requests split into top-level items, items pretested by hop-bounded
// reachability; engine.hip checks the kept work requests, then reach_merge folds their decisions
// into the requests' (allowed if an item is, else undecided if one is, else denied)
struct ItemWork {
    keto_check_ids* work = nullptr;   // device: kept work requests (items, and requests checked whole)
    uint32_t* owner = nullptr;        // device: the request each belongs to
    uint32_t n_work = 0;              // kept work requests
    uint32_t n_entries = 0;           // work requests before the pretest
    uint32_t* acc = nullptr;          // device: per request, what its items decided
    uint8_t* dec = nullptr;           // device: decisions of the work requests
    uint32_t* wsteps = nullptr;       // device: loop iterations per work request (instrumented), or NULL
    uint32_t* undecided = nullptr;    // device: requests left undecided
    float split_ms = 0;               // split + pretest + compaction
    float index_ms = 0;               // index rebuilt first (host + upload), 0 if it was current
};
bool reach_enabled(const Snapshot& s);
bool reach_split(Snapshot& s, const keto_check_ids* d_reqs, uint32_t n, int32_t gmd, uint8_t* d_allowed,
                 uint32_t ov_base, void* stream, bool steps, ItemWork& out);
void reach_merge(Snapshot& s, const ItemWork& w, uint32_t n, uint8_t* d_allowed, uint32_t* d_steps, void* stream,
                 uint32_t* undecided);
float reach_build_ms(const Snapshot& s);
void* host_alloc(uint64_t bytes);    // pinned host memory (hipHostMalloc)
void host_free(void* p);
// partitioned-batch routing (route.hip): stable counting sort of row-id requests by owner part
uint64_t route_work_bytes(uint32_t n, uint32_t n_parts);
void route_rows(const keto_check_ids* d_reqs, uint32_t n, const int16_t* d_owner, uint32_t n_rows, uint32_t self_part,
                uint32_t n_parts, void* d_work, uint64_t work_len, keto_check_ids* d_send, uint32_t* d_order,
                uint32_t* counts_out, void* stream);
void unroute_rows(const uint8_t* d_back, const uint32_t* d_order, uint32_t n, uint8_t* d_out, void* stream);
// migrating partition (engine.hip): closure-filter exchange between parts.  part_filters copies the
// closure filters (CF_WORDS words each) of this part's rows; part_close ORs the owners' filters into
// the stubs of `rows`, re-closes this part's filters and returns how many filters changed;
// part_closure_done finishes the filters (signatures) or, when the exchange did not converge, sets
// every filter to all ones (no pruning, still exact)
void part_filters(Snapshot& s, const uint32_t* rows, uint64_t n, uint32_t* out);
uint64_t part_close(Snapshot& s, const uint32_t* rows, uint64_t n, const uint32_t* filters);
void part_closure_done(Snapshot& s, bool converged);
struct DevView {             // what migrate.hip needs of a device snapshot
    const uint32_t* arena;
    uint64_t arena_words;
    const uint64_t* coll;
    uint32_t coll_mask;
    int device;
    void* stream;
};
DevView device_view(const Snapshot& s);
// migrating-partition check batches (migrate.hip); see keto_mig_begin / keto_mig_round
struct MigOut {
    uint64_t units[MIG_MAX_PARTS];
    uint32_t records[MIG_MAX_PARTS];
    const void* d_buf;
    const uint32_t* d_off;
    uint32_t decided, undecided, processed, reruns;
};
void mig_begin(Snapshot& s, const keto_check_ids* d_reqs, uint32_t n, int32_t gmd, uint8_t* d_allowed, void* stream,
               MigOut& out, bool child_entries = false);
void mig_round(Snapshot& s, const void* d_in, const uint32_t* d_in_off, const uint32_t* in_records,
               const uint64_t* in_units, void* stream, MigOut& out);
void mig_release(Snapshot& s);
// acl.SubjectTree bytes of trees (pre-order nodes, tree t = nodes[tree_off[t], tree_off[t+1])) encoded
// on the device (proto.hip): offsets[n_trees + 1] always; buf written when cap >= the total returned
uint64_t device_tree_proto(Snapshot& s, const keto_tree_node* nodes, uint64_t n_nodes, const uint64_t* tree_off,
                           uint32_t n_trees, uint32_t ov_base, const std::vector<RowKey>& ov_keys, uint32_t extra_base,
                           const std::vector<std::string>& extra, uint8_t* buf, uint64_t cap, uint64_t* offsets);
void device_copy(void* dst, const void* src, uint64_t bytes, void* stream);   // D2D, synchronous
void device_memory(int device, uint64_t& free_bytes, uint64_t& total_bytes);
// packed string requests resolved and checked on the device (resolve_dev.hip); the indexes of the
// requests left to the host (wildcard queries) are appended to `host`
void device_check_packed(Snapshot& s, const uint8_t* blob, uint64_t blob_len, const keto_check_packed* reqs, uint32_t n,
                         int32_t gmd, uint8_t* allowed, uint8_t* status, std::vector<uint32_t>& host);
void rdev_release(Snapshot& s);
// a packed batch resolved on the device into row-id requests (the routed path, comm.cpp): d_out on
// the device, statuses to the host; host_idx = the requests left to the host (wildcard queries)
void device_resolve_packed_rows(Snapshot& s, const uint8_t* blob, uint64_t blob_len, const keto_check_packed* reqs,
                                uint32_t n, keto_check_ids* d_out, uint8_t* status_out, std::vector<uint32_t>& host_idx,
                                void* stream);
// d[idx[k]] = vals[k] for k < m (device arrays)
void scatter_ids(keto_check_ids* d, const uint32_t* d_idx, const keto_check_ids* d_vals, uint32_t m, void* stream);
// up to COPY_SEGMENTS device-to-device copies in one launch (route.hip)
constexpr uint32_t COPY_SEGMENTS = 64;
struct CopySegments {
    const void* src[COPY_SEGMENTS];
    void* dst[COPY_SEGMENTS];
    uint64_t bytes[COPY_SEGMENTS];
    uint32_t n;
};
void copy_segments(const CopySegments& s, void* stream);
// An allocator whose resize() leaves new elements default-initialized (no zero fill): the expand
// node arena is sized, then overwritten by one D2H copy.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
    template <class U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
        ::new ((void*)p) U;
    }
};

// Page-locked host memory for expand node arenas (engine.hip): blocks are recycled across arenas,
// so the arena's D2H is one DMA at the link's rate without a hipHostMalloc per call.  Falls back to
// malloc when no pinned memory can be had.
// tooling (KETO_TRACE_LOCKS=1): one stderr line per lock / phase step of the calls that share a
// snapshot (apply, packed batches), with the thread: where each thread waits when a run hangs
void lock_trace(const char* what);
void* pinned_take(size_t bytes);
void pinned_give(void* p) noexcept;
template <class T>
struct PinnedAlloc : NoInitAlloc<T> {
    using value_type = T;
    template <class U>
    struct rebind {
        using other = PinnedAlloc<U>;
    };
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U>&) noexcept {}
    T* allocate(size_t n) { return static_cast<T*>(pinned_take(n * sizeof(T))); }
    void deallocate(T* p, size_t) noexcept { pinned_give(p); }
};
template <class T, class U>
bool operator==(const PinnedAlloc<T>&, const PinnedAlloc<U>&) noexcept { return true; }
template <class T, class U>
bool operator!=(const PinnedAlloc<T>&, const PinnedAlloc<U>&) noexcept { return false; }

struct ExpandResult {
    std::vector<uint8_t> status;
    std::vector<uint64_t> offset;          // n+1
    std::vector<keto_tree_node, PinnedAlloc<keto_tree_node>> nodes;
};
// roots: row handles (root_flags bit0 = subject set) or string ids; out.nodes carry row ids.  On a
// migrating part, remote_roots lists the roots (index, row id) whose rows this part does not hold
// (their root / vid entries are ignored).  root_rows: each subject-set root's row id (any other
// entry ignored), which an arena whose roots lie past 2^31 units needs: such a root's handle does
// not fit a tree node, so its node takes the row from here
void device_expand(Snapshot& s, const std::vector<uint32_t>& root, const std::vector<uint32_t>& root_flags,
                   const std::vector<uint32_t>& root_vid, const std::vector<int32_t>& depth, int32_t gmd,
                   const Overlay* ov, ExpandResult& out,
                   const std::vector<std::pair<uint32_t, uint32_t>>* remote_roots = nullptr,
                   const std::vector<uint32_t>* root_rows = nullptr);

}  // namespace keto
