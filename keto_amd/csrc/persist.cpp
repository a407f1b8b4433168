// Persisted snapshots (keto_snapshot_save / keto_snapshot_load): the host tables a snapshot is
// built into, written to one file, so that a restarting server uploads its graph again instead of
// scanning and sorting the whole table (the reference reads every tuple back through
// internal/persistence/sql/relationtuples.go:249-251 on each query; a GPU server's snapshot is
// built from that scan once, SURVEY 8(f) row 2 names an optional on-disk CSR).
//
// What is saved is exactly what keto_snapshot_clone copies (clone_host, snapshot.cpp): the config,
// the strings, the rows with their keys, page cuts and edges, the collision classes, and the state
// writes added (added strings, rows' current edges, the version).  The arena layout, the resolution
// indexes and every device structure are derived and are recomputed on load, as for a clone.
//
// File: a 64-B header (magic, format, the caller's tag, the version, section count), then sections,
// each a 24-B prefix {id, bytes, hash} and its payload padded to 8 B.  The hash is a 64-bit mix over
// 1-MiB blocks (hashed in parallel, folded in order); a truncated or damaged file fails the load
// with KETO_E_INVALID naming the section.  Large sections are written and read with positional I/O
// on the builder's threads.  The file is written under <path>.tmp and renamed, so a crash during
// save leaves the previous file intact.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>

#include "parallel.hpp"
#include "snapshot.hpp"

namespace keto {

namespace {

constexpr char MAGIC[8] = {'K', 'E', 'T', 'O', 'S', 'N', 'A', 'P'};
constexpr uint32_t FORMAT = 1;
constexpr uint64_t BLOCK = 1ull << 20;

struct FileHeader {        // 64 B
    char magic[8];
    uint32_t format;
    uint32_t abi;
    uint64_t tag;          // the caller's (e.g. the table's last commit when the snapshot was built)
    uint64_t version;
    uint64_t n_sections;
    uint64_t reserved[3];
};
static_assert(sizeof(FileHeader) == 64, "header is 64 bytes");

struct SecHeader {         // 24 B
    uint64_t id, bytes, hash;
};

struct Scalars {
    uint32_t page_size, empty_str, n_real_rows, n_wild_rows;
    uint32_t n_coll_keys, n_poisoned_rows, n_seq_rows, n_sorted_strs;
    uint32_t n_base_rows, n_ns, pad0, pad1;
    uint64_t n_tuples, version;
};

enum : uint64_t {
    S_SCALARS = 1, S_NS_IDS, S_NS_OFF, S_NS_BLOB, S_STR_OFF, S_STR_BLOB, S_WILD, S_ROW_KEY, S_ROW_OF,
    S_ROWS, S_ROW_PP, S_EDGES, S_COLL, S_ADDED_OFF, S_ADDED_BLOB, S_ADDED_ID, S_OVER_ROW, S_OVER_OFF,
    S_OVER_EDGES, S_END
};

uint64_t block_hash(const char* p, uint64_t n, uint64_t seed) {
    uint64_t h = seed ^ (n * 0x9E3779B97F4A7C15ull), i = 0;
    for (; i + 32 <= n; i += 32) {                                   // four independent lanes
        uint64_t a = load64(p + i), b = load64(p + i + 8), c = load64(p + i + 16), d = load64(p + i + 24);
        h = mix64(h ^ a) + mix64(b ^ 0x632BE59BD9B4E019ull) + mix64(c + h) + mix64(d ^ (h >> 17));
    }
    for (; i + 8 <= n; i += 8) h = mix64(h ^ load64(p + i));
    uint64_t t = 0;
    if (i < n) std::memcpy(&t, p + i, n - i);
    return mix64(h ^ t ^ 0xD6E8FEB86659FD93ull);
}

uint64_t section_hash(const void* data, uint64_t n, unsigned threads) {
    const char* p = static_cast<const char*>(data);
    const uint64_t nb = (n + BLOCK - 1) / BLOCK;
    std::vector<uint64_t> hb(nb);
    par_chunks(nb, nb >= 16 ? threads : 1u, 4, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t k = b; k < e; ++k) hb[k] = block_hash(p + k * BLOCK, std::min(BLOCK, n - k * BLOCK), k);
    });
    uint64_t h = mix64(n + 1);
    for (uint64_t x : hb) h = mix64(h ^ x) * 0x94D049BB133111EBull;
    return h;
}

struct Fd {
    int fd = -1;
    ~Fd() { if (fd >= 0) ::close(fd); }
};

void io_all(int fd, char* p, uint64_t n, uint64_t off, bool write, const std::string& what) {
    while (n) {
        const size_t step = (size_t)std::min<uint64_t>(n, 1ull << 30);
        const ssize_t r = write ? ::pwrite(fd, p, step, (off_t)off) : ::pread(fd, p, step, (off_t)off);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0)
            throw Error{KETO_E_INVALID, std::string(write ? "write" : "read") + " of " + what + " failed: " +
                                            (r < 0 ? std::strerror(errno) : "unexpected end of file")};
        p += r;
        n -= (uint64_t)r;
        off += (uint64_t)r;
    }
}

// positional I/O of one buffer on several threads (64-MiB pieces)
void io_par(int fd, char* p, uint64_t n, uint64_t off, bool write, unsigned threads, const std::string& what) {
    constexpr uint64_t PIECE = 64ull << 20;
    const uint64_t np = (n + PIECE - 1) / PIECE;
    std::atomic<bool> failed{false};
    Error first{KETO_OK, ""};
    std::mutex mu;
    par_chunks(np, np >= 2 ? threads : 1u, 1, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t k = b; k < e && !failed; ++k) {
            try {
                io_all(fd, p + k * PIECE, std::min(PIECE, n - k * PIECE), off + k * PIECE, write, what);
            } catch (const Error& x) {
                std::lock_guard<std::mutex> lk(mu);
                if (!failed.exchange(true)) first = x;
            }
        }
    });
    if (failed) throw first;
}

struct Writer {
    int fd;
    unsigned threads;
    uint64_t off = sizeof(FileHeader);
    uint64_t n_sections = 0;
    void section(uint64_t id, const void* data, uint64_t bytes) {
        SecHeader h{id, bytes, section_hash(data, bytes, threads)};
        io_all(fd, reinterpret_cast<char*>(&h), sizeof h, off, true, "a section header");
        off += sizeof h;
        if (bytes) io_par(fd, const_cast<char*>(static_cast<const char*>(data)), bytes, off, true, threads,
                          "section " + std::to_string(id));
        off += (bytes + 7) & ~7ull;
        ++n_sections;
    }
    template <class V>
    void vec(uint64_t id, const V& v) { section(id, v.data(), v.size() * sizeof(v[0])); }
};

struct Reader {
    int fd;
    unsigned threads;
    uint64_t size;
    uint64_t off = sizeof(FileHeader);
    // the next section, which must be `id`; its payload read into out (resized to fit)
    template <class T>
    void vec(uint64_t id, std::vector<T>& out) {
        SecHeader h;
        if (off + sizeof h > size) throw Error{KETO_E_INVALID, "snapshot file truncated before section " + std::to_string(id)};
        io_all(fd, reinterpret_cast<char*>(&h), sizeof h, off, false, "a section header");
        off += sizeof h;
        if (h.id != id) throw Error{KETO_E_INVALID, "snapshot file: section " + std::to_string(id) + " expected, found " + std::to_string(h.id)};
        if (h.bytes > size || h.bytes % sizeof(T) || off + h.bytes > size)
            throw Error{KETO_E_INVALID, "snapshot file: section " + std::to_string(id) + " has a bad size"};
        out.resize(h.bytes / sizeof(T));
        if (h.bytes) io_par(fd, reinterpret_cast<char*>(out.data()), h.bytes, off, false, threads, "section " + std::to_string(id));
        if (section_hash(out.data(), h.bytes, threads) != h.hash)
            throw Error{KETO_E_INVALID, "snapshot file: section " + std::to_string(id) + " is damaged (hash mismatch)"};
        off += (h.bytes + 7) & ~7ull;
    }
};

// KETO_BUILD_TRACE=1: load phase times on stderr (tooling)
struct LoadClock {
    bool on = getenv("KETO_BUILD_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char* what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "[keto load] %-28s %8.3f s\n", what, std::chrono::duration<double>(n - t).count());
        t = n;
    }
};

struct RowOfRec {
    RowKey k;
    uint32_t row, pad;
};
static_assert(sizeof(RowOfRec) == 24, "row_of record is 24 bytes");

// strings as offsets (n + 1) and one byte blob
template <class Get>
void pack_strings(uint64_t n, Get get, std::vector<uint64_t>& off, std::vector<char>& blob, unsigned threads) {
    off.assign(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) off[i + 1] = off[i] + get(i).size();
    blob.resize(off[n]);
    par_chunks(n, n >= par_min() ? threads : 1u, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t i = b; i < e; ++i) {
            const std::string_view s = get(i);
            if (!s.empty()) std::memcpy(blob.data() + off[i], s.data(), s.size());
        }
    });
}

template <class Out>   // std::vector<std::string> or Chunked<std::string>
void unpack_strings(const std::vector<uint64_t>& off, const std::vector<char>& blob, Out& out,
                    unsigned threads, const char* what) {
    if (off.empty()) throw Error{KETO_E_INVALID, std::string("snapshot file: no offsets for ") + what};
    const uint64_t n = off.size() - 1;
    for (uint64_t i = 0; i < n; ++i)
        if (off[i] > off[i + 1]) throw Error{KETO_E_INVALID, std::string("snapshot file: bad offsets for ") + what};
    if (off[n] != blob.size()) throw Error{KETO_E_INVALID, std::string("snapshot file: bad blob size for ") + what};
    out.resize(n);
    par_chunks(n, n >= par_min() ? threads : 1u, 1 << 14, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t i = b; i < e; ++i) out[i].assign(blob.data() + off[i], off[i + 1] - off[i]);
    });
}

}  // namespace

void save_snapshot(const Snapshot& S, const char* path, uint64_t tag) {
    if (!path || !*path) throw Error{KETO_E_INVALID, "path is empty"};
    if (S.n_parts > 1) throw Error{KETO_E_INVALID, "a part of a partitioned snapshot cannot be saved"};
    const unsigned th = build_threads();
    const std::string tmp = std::string(path) + ".tmp";
    Fd f;
    f.fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (f.fd < 0) throw Error{KETO_E_INVALID, "cannot create " + tmp + ": " + std::strerror(errno)};
    Writer w{f.fd, th};

    Scalars sc{};
    sc.page_size = S.page_size;
    sc.empty_str = S.empty_str;
    sc.n_real_rows = S.n_real_rows;
    sc.n_wild_rows = S.n_wild_rows;
    sc.n_coll_keys = S.n_coll_keys;
    sc.n_poisoned_rows = S.n_poisoned_rows;
    sc.n_seq_rows = S.n_seq_rows;
    sc.n_sorted_strs = S.n_sorted_strs;
    sc.n_base_rows = S.n_base_rows;
    sc.n_ns = (uint32_t)S.ns_ids.size();
    sc.n_tuples = S.n_tuples;
    sc.version = S.version;
    w.section(S_SCALARS, &sc, sizeof sc);
    w.vec(S_NS_IDS, S.ns_ids);
    {
        std::vector<uint64_t> off;
        std::vector<char> blob;
        pack_strings(S.ns_names.size(), [&](uint64_t i) { return std::string_view(S.ns_names[i]); }, off, blob, 1);
        w.vec(S_NS_OFF, off);
        w.vec(S_NS_BLOB, blob);
    }
    {
        std::vector<uint64_t> off;
        std::vector<char> blob;
        pack_strings(S.strs.size(), [&](uint64_t i) { return std::string_view(S.strs[i]); }, off, blob, th);
        w.vec(S_STR_OFF, off);
        w.vec(S_STR_BLOB, blob);
    }
    w.vec(S_WILD, S.wild_rows);
    w.vec(S_ROW_KEY, S.row_key);
    {
        std::vector<RowOfRec> ro;
        ro.reserve(S.row_of.size());
        for (const auto& kv : S.row_of) ro.push_back(RowOfRec{kv.first, kv.second, 0});
        std::sort(ro.begin(), ro.end(), [](const RowOfRec& a, const RowOfRec& b) { return a.row < b.row; });
        w.vec(S_ROW_OF, ro);
    }
    w.vec(S_ROWS, S.rows);
    w.vec(S_ROW_PP, S.row_pp);
    w.vec(S_EDGES, S.edges);
    {
        std::vector<uint32_t> cl;
        cl.reserve(2 * S.coll.size());
        for (const auto& kv : S.coll) { cl.push_back(kv.first); cl.push_back(kv.second); }
        w.vec(S_COLL, cl);
    }
    {
        std::vector<std::pair<std::string_view, uint32_t>> ad(S.added_str.begin(), S.added_str.end());
        std::sort(ad.begin(), ad.end(), [](const auto& a, const auto& b) { return a.second < b.second; });
        std::vector<uint64_t> off;
        std::vector<char> blob;
        pack_strings(ad.size(), [&](uint64_t i) { return ad[i].first; }, off, blob, 1);
        std::vector<uint32_t> ids(ad.size());
        for (size_t i = 0; i < ad.size(); ++i) ids[i] = ad[i].second;
        w.vec(S_ADDED_OFF, off);
        w.vec(S_ADDED_BLOB, blob);
        w.vec(S_ADDED_ID, ids);
    }
    {
        std::vector<uint32_t> rows;
        rows.reserve(S.row_over.size());
        for (const auto& kv : S.row_over) rows.push_back(kv.first);
        std::sort(rows.begin(), rows.end());
        std::vector<uint64_t> off(1, 0);
        std::vector<uint32_t> ed;
        for (uint32_t r : rows) {
            const auto& v = S.row_over.at(r);
            ed.insert(ed.end(), v.begin(), v.end());
            off.push_back(ed.size());
        }
        w.vec(S_OVER_ROW, rows);
        w.vec(S_OVER_OFF, off);
        w.vec(S_OVER_EDGES, ed);
    }
    w.section(S_END, nullptr, 0);

    FileHeader fh{};
    std::memcpy(fh.magic, MAGIC, 8);
    fh.format = FORMAT;
    fh.abi = KETO_ABI_VERSION;
    fh.tag = tag;
    fh.version = S.version;
    fh.n_sections = w.n_sections;
    io_all(f.fd, reinterpret_cast<char*>(&fh), sizeof fh, 0, true, "the header");
    if (::fsync(f.fd) != 0) throw Error{KETO_E_INVALID, "fsync of " + tmp + " failed: " + std::strerror(errno)};
    ::close(f.fd);
    f.fd = -1;
    if (::rename(tmp.c_str(), path) != 0)
        throw Error{KETO_E_INVALID, "rename " + tmp + " -> " + path + " failed: " + std::strerror(errno)};
}

std::unique_ptr<Snapshot> load_snapshot(const char* path, uint64_t* tag_out) {
    if (!path || !*path) throw Error{KETO_E_INVALID, "path is empty"};
    const unsigned th = build_threads();
    Fd f;
    f.fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (f.fd < 0) throw Error{KETO_E_INVALID, std::string("cannot open ") + path + ": " + std::strerror(errno)};
    struct stat st;
    if (::fstat(f.fd, &st) != 0) throw Error{KETO_E_INVALID, std::string("cannot stat ") + path};
    FileHeader fh;
    if ((uint64_t)st.st_size < sizeof fh) throw Error{KETO_E_INVALID, std::string(path) + " is not a snapshot file"};
    io_all(f.fd, reinterpret_cast<char*>(&fh), sizeof fh, 0, false, "the header");
    if (std::memcmp(fh.magic, MAGIC, 8) != 0) throw Error{KETO_E_INVALID, std::string(path) + " is not a snapshot file"};
    if (fh.format != FORMAT)
        throw Error{KETO_E_INVALID, "snapshot file format " + std::to_string(fh.format) + " (this library reads " +
                                        std::to_string(FORMAT) + ")"};
    // a file from a newer library may carry records this one lays out differently
    if (fh.abi > (uint32_t)KETO_ABI_VERSION)
        throw Error{KETO_E_INVALID, "snapshot file written by library ABI " + std::to_string(fh.abi) + " (this is " +
                                        std::to_string(KETO_ABI_VERSION) + ")"};
    Reader rd{f.fd, th, (uint64_t)st.st_size};

    LoadClock clk;
    auto Sp = std::make_unique<Snapshot>();
    Snapshot& S = *Sp;
    std::vector<Scalars> sc;
    rd.vec(S_SCALARS, sc);
    if (sc.size() != 1) throw Error{KETO_E_INVALID, "snapshot file: bad scalars"};
    const Scalars& c = sc[0];
    rd.vec(S_NS_IDS, S.ns_ids);
    {
        std::vector<uint64_t> off;
        std::vector<char> blob;
        rd.vec(S_NS_OFF, off);
        rd.vec(S_NS_BLOB, blob);
        unpack_strings(off, blob, S.ns_names, 1, "namespaces");
        if (S.ns_names.size() != S.ns_ids.size() || S.ns_ids.size() != c.n_ns)
            throw Error{KETO_E_INVALID, "snapshot file: namespace tables disagree"};
        for (uint32_t i = 0; i < c.n_ns; ++i) {
            S.ns_by_id[S.ns_ids[i]] = (int)i;
            S.ns_by_name[S.ns_names[i]] = (int)i;
        }
        for (uint32_t i = 0; i < c.n_ns; ++i) S.ns_view.emplace(S.ns_names[i], (int)i);
    }
    {
        std::vector<uint64_t> off;
        std::vector<char> blob;
        rd.vec(S_STR_OFF, off);
        rd.vec(S_STR_BLOB, blob);
        clk.lap("strings read");
        unpack_strings(off, blob, S.strs, th, "strings");
        clk.lap("strings unpacked");
    }
    S.page_size = c.page_size;
    S.empty_str = c.empty_str;
    S.n_real_rows = c.n_real_rows;
    S.n_wild_rows = c.n_wild_rows;
    S.n_coll_keys = c.n_coll_keys;
    S.n_poisoned_rows = c.n_poisoned_rows;
    S.n_seq_rows = c.n_seq_rows;
    S.n_sorted_strs = c.n_sorted_strs;
    S.n_base_rows = c.n_base_rows;
    S.n_tuples = c.n_tuples;
    S.version = c.version;
    rd.vec(S_WILD, S.wild_rows);
    rd.vec(S_ROW_KEY, S.row_key);
    {
        std::vector<RowOfRec> ro;
        rd.vec(S_ROW_OF, ro);
        S.row_of.reserve(ro.size());
        for (const RowOfRec& x : ro) S.row_of.emplace(x.k, x.row);
    }
    rd.vec(S_ROWS, S.rows);
    rd.vec(S_ROW_PP, S.row_pp);
    rd.vec(S_EDGES, S.edges);
    {
        std::vector<uint32_t> cl;
        rd.vec(S_COLL, cl);
        if (cl.size() % 2) throw Error{KETO_E_INVALID, "snapshot file: bad collision table"};
        S.coll.reserve(cl.size() / 2);
        for (size_t i = 0; i < cl.size(); i += 2) S.coll.emplace(cl[i], cl[i + 1]);
    }
    {
        std::vector<uint64_t> off;
        std::vector<char> blob;
        std::vector<uint32_t> ids;
        std::vector<std::string> ad;
        rd.vec(S_ADDED_OFF, off);
        rd.vec(S_ADDED_BLOB, blob);
        rd.vec(S_ADDED_ID, ids);
        unpack_strings(off, blob, ad, 1, "added strings");
        if (ids.size() != ad.size()) throw Error{KETO_E_INVALID, "snapshot file: added strings disagree"};
        for (size_t i = 0; i < ad.size(); ++i) S.added_str.emplace(std::move(ad[i]), ids[i]);
    }
    {
        std::vector<uint32_t> rows, ed;
        std::vector<uint64_t> off;
        rd.vec(S_OVER_ROW, rows);
        rd.vec(S_OVER_OFF, off);
        rd.vec(S_OVER_EDGES, ed);
        if (off.size() != rows.size() + 1 || off.back() != ed.size())
            throw Error{KETO_E_INVALID, "snapshot file: bad changed-row table"};
        for (size_t i = 0; i < rows.size(); ++i) {
            if (off[i] > off[i + 1]) throw Error{KETO_E_INVALID, "snapshot file: bad changed-row table"};
            S.row_over.emplace(rows[i], std::vector<uint32_t>(ed.begin() + off[i], ed.begin() + off[i + 1]));
        }
    }
    {
        std::vector<char> end;
        rd.vec(S_END, end);
    }
    clk.lap("tables read");
    // the tables must agree with each other before anything indexes with them
    const uint64_t R = S.row_key.size();
    if (S.rows.size() != R || S.row_pp.size() != R || R >= EDGE_VAL || S.n_real_rows > R || S.n_base_rows > R ||
        S.n_sorted_strs > S.strs.size())
        throw Error{KETO_E_INVALID, "snapshot file: row tables disagree"};
    for (uint32_t r : S.wild_rows)
        if (r >= R) throw Error{KETO_E_INVALID, "snapshot file: wildcard row out of range"};
    for (const auto& kv : S.row_of)
        if (kv.second >= R) throw Error{KETO_E_INVALID, "snapshot file: row out of range"};
    for (uint32_t r = 0; r < S.n_base_rows; ++r) {
        const uint64_t b = S.row_begin(r), e = r + 1 < S.n_base_rows ? S.row_begin(r + 1) : S.edges.size();
        if (b > e || e > S.edges.size()) throw Error{KETO_E_INVALID, "snapshot file: edge offsets out of range"};
    }
    std::atomic<bool> bad{false};
    // strings writes added are appended to strs; a CSR snapshot loaded without a string table
    // (keto_snapshot_from_csr, strings == NULL) has subject ids that name no string
    const uint64_t n_str = S.strs.empty() ? EDGE_VAL : S.strs.size();
    par_chunks(S.edges.size(), th, 1 << 20, [&](uint64_t b, uint64_t e, unsigned) {
        for (uint64_t i = b; i < e; ++i) {
            const uint32_t x = S.edges[i];
            if (x == EDGE_POISON) continue;
            if ((x & EDGE_SET) ? (x & ~EDGE_SET) >= R : x >= n_str) { bad = true; return; }
        }
    });
    for (const auto& kv : S.row_over) {
        if (kv.first >= R) bad = true;
        for (uint32_t x : kv.second)
            if (x != EDGE_POISON && ((x & EDGE_SET) ? (x & ~EDGE_SET) >= R : x >= n_str)) bad = true;
    }
    if (bad) throw Error{KETO_E_INVALID, "snapshot file: an edge names a row or string out of range"};
    // the scalars and ids compute_layout and the kernels index with (a damaged or foreign file must
    // fail here, not index out of range later)
    if (S.page_size == 0 || S.n_wild_rows != S.wild_rows.size() || S.n_seq_rows > R || S.n_poisoned_rows > R ||
        (S.empty_str != ANY && S.empty_str >= n_str))
        throw Error{KETO_E_INVALID, "snapshot file: bad scalars"};
    for (uint64_t r = 0; r < R; ++r) {
        const RowKey& k = S.row_key[r];
        if ((k.obj != ANY && k.obj >= n_str) || (k.rel != ANY && k.rel >= n_str))
            throw Error{KETO_E_INVALID, "snapshot file: a row key names a string out of range"};
    }
    for (const auto& kv : S.coll) {
        const uint32_t key = kv.first, v = kv.second;
        const bool key_ok = (key & EDGE_SET) ? (key & ~EDGE_SET) < R : key < n_str;
        if (!key_ok || !(v & VID_CLASS) || (v & ~VID_CLASS) >= std::max<uint64_t>(S.n_coll_keys, S.coll.size()))
            throw Error{KETO_E_INVALID, "snapshot file: bad collision class"};
    }
    for (const auto& kv : S.added_str)
        if (kv.second < S.n_sorted_strs || kv.second >= S.strs.size())
            throw Error{KETO_E_INVALID, "snapshot file: an added string's id is out of range"};
    clk.lap("tables checked");
    if (tag_out) *tag_out = fh.tag;
    compute_layout(S);
    clk.lap("layout");
    return Sp;
}

}  // namespace keto
