//go:build keto_gpu
// +build keto_gpu

// Package gpu binds Keto's read engines to the MI355X engine (libketo_mi355x.so, C-ABI
// include/keto_mi355x.h).  Drop this directory into the Keto tree as internal/gpu and build with
// `-tags sqlite,keto_gpu`.  Written for the reference's toolchain, Go 1.17 (go.mod:221): no generics,
// no runtime.Pinner, no unsafe.StringData.
//
// cgo pointer rules: the C side keeps no pointer after a call returns (keto_mi355x.h), and every
// array handed to it lives in C memory (one C.malloc'd block of structs plus one of string bytes
// per call, or a large packed batch's page-locked arena from keto_host_alloc), so no Go pointer is
// ever passed inside a struct.
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/include
#cgo LDFLAGS: -lketo_mi355x
#include <stdlib.h>
#include "keto_mi355x.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"sync"
	"unsafe"

	"github.com/ory/keto/internal/namespace"
	"github.com/ory/keto/internal/relationtuple"
)

// This package must not import internal/expand, internal/check or internal/driver: those import it
// (engine_gpu.go, registry_gpu.go).  Trees therefore come back as pre-order Nodes, and
// internal/expand builds its *Tree values from them.

// Decision statuses of CheckBatch (KETO_CHECK_*).
const (
	StatusOK               = uint8(C.KETO_CHECK_OK)
	StatusUnknownNamespace = uint8(C.KETO_CHECK_UNKNOWN_NAMESPACE)
	StatusUndecided        = uint8(C.KETO_CHECK_UNDECIDED) // ask the SQL engine for this one request
)

var (
	// ErrNotFound mirrors herodot.ErrNotFound for expand roots in unknown namespaces
	// (internal/expand/handler_test.go:48-59); the caller maps it to its herodot error.
	ErrNotFound = errors.New("gpu: unknown namespace")
	// ErrUndecided: the tree exceeds the engine's limits; fall back to the SQL engine.
	ErrUndecided = errors.New("gpu: tree exceeds the engine's limits")
)

// Error is a negative KETO_E_* code with the library's thread-local message.
type Error struct {
	Code int
	Msg  string
}

func (e *Error) Error() string { return fmt.Sprintf("keto_mi355x error %d: %s", e.Code, e.Msg) }

func lastErr(rc C.int) error {
	if rc == C.KETO_OK {
		return nil
	}
	return &Error{Code: int(rc), Msg: C.GoString(C.keto_last_error())}
}

// cmem is one call's C memory: an arena of string bytes and the struct arrays, freed together.
type cmem struct {
	blocks []unsafe.Pointer
	str    unsafe.Pointer
	used   int
}

func (m *cmem) alloc(n int) unsafe.Pointer {
	if n < 1 {
		n = 1
	}
	p := C.malloc(C.size_t(n))
	if p == nil {
		panic("gpu: C.malloc failed")
	}
	m.blocks = append(m.blocks, p)
	return p
}

// strings reserves the byte arena for every string the call will pass.
func (m *cmem) strings(total int) { m.str = m.alloc(total) }

func (m *cmem) s(v string) C.keto_str {
	if len(v) == 0 {
		return C.keto_str{}
	}
	dst := unsafe.Add(m.str, m.used)
	copy(unsafe.Slice((*byte)(dst), len(v)), v)
	m.used += len(v)
	return C.keto_str{p: (*C.char)(dst), n: C.uint32_t(len(v))}
}

func (m *cmem) free() {
	for _, p := range m.blocks {
		C.free(p)
	}
	m.blocks = nil
}

// Row is one row of keto_relation_tuples (internal/persistence/sql/relationtuples.go:19-31).
// Rows are passed in commit order: ties of the reference ORDER BY keep that order.
type Row struct {
	NamespaceID    int32
	Object         string
	Relation       string
	SubjectID      *string // nil -> subject set
	SetNamespaceID int32
	SetObject      string
	SetRelation    string
}

// Snapshot is a device-resident snapshot of the tuple table, patched in place by Apply.
type Snapshot struct {
	h       *C.keto_snapshot
	Version uint64 // bumped by every Apply (snapshot lifecycle, see apply.go)
	device  int    // HIP device of its arena, -1: host only
	arenas  arenaPool
}

// pinnedArena is a snapshot's page-locked buffer for large packed batches (keto_host_alloc), reused
// from call to call and grown when a batch needs more.  keto_check_batch_packed uploads a batch from
// it asynchronously, piece by piece under the resolution and check of earlier pieces; from C.malloc'd
// memory the runtime stages every copy through its own bounce buffers, synchronously.  Pinning maps
// and locks every page, so it is paid once per size, not per call.
type pinnedArena struct {
	mu sync.Mutex
	p  unsafe.Pointer
	n  int
}

// pinMin is the smallest packed batch (bytes of strings, records and outputs) that uses the arena.
const pinMin = 1 << 20

// get locks the arena and returns it with at least n bytes; ok = false (and unlocked) when pinning
// failed, and the caller uses C memory instead.
func (a *pinnedArena) get(n int) (unsafe.Pointer, bool) {
	a.mu.Lock()
	if n > a.n {
		if a.p != nil {
			C.keto_host_free(a.p)
			a.p, a.n = nil, 0
		}
		grow := n + n/4
		var p unsafe.Pointer
		if rc := C.keto_host_alloc(C.uint64_t(grow), &p); rc != C.KETO_OK || p == nil {
			a.mu.Unlock()
			return nil, false
		}
		a.p, a.n = p, grow
	}
	return a.p, true
}

func (a *pinnedArena) put() { a.mu.Unlock() }

// arenaPool holds one pinned arena per packed batch a snapshot keeps in flight (InflightFromEnv):
// the library runs one batch's upload and resolution while another's check runs
// (keto_check_batch_packed, KETO_PACKED_SLOTS), so two batches must not share staging memory.
type arenaPool struct {
	once sync.Once
	free chan *pinnedArena
	all  []*pinnedArena
}

func (p *arenaPool) init() {
	p.once.Do(func() {
		n := InflightFromEnv()
		p.free = make(chan *pinnedArena, n)
		for i := 0; i < n; i++ {
			a := &pinnedArena{}
			p.all = append(p.all, a)
			p.free <- a
		}
	})
}

// get takes a free arena with at least n bytes (waiting for one); ok = false when pinning failed
// (the arena is returned, and the caller uses C memory instead).
func (p *arenaPool) get(n int) (*pinnedArena, unsafe.Pointer, bool) {
	p.init()
	a := <-p.free
	base, ok := a.get(n)
	if !ok {
		p.free <- a
		return nil, nil, false
	}
	return a, base, true
}

func (p *arenaPool) put(a *pinnedArena) {
	a.put()
	p.free <- a
}

func (p *arenaPool) freeAll() {
	p.init()
	for _, a := range p.all {
		a.free()
	}
}

func (a *pinnedArena) free() {
	a.mu.Lock()
	if a.p != nil {
		C.keto_host_free(a.p)
		a.p, a.n = nil, 0
	}
	a.mu.Unlock()
}

// rowsLen is the string bytes of rows (one arena per call).
func rowsLen(rows []Row) int {
	total := 0
	for i := range rows {
		r := &rows[i]
		total += len(r.Object) + len(r.Relation) + len(r.SetObject) + len(r.SetRelation)
		if r.SubjectID != nil {
			total += len(*r.SubjectID)
		}
	}
	return total
}

// tuples copies rows into C memory as keto_tuple structs (nil for none).
func (m *cmem) tuples(rows []Row) *C.keto_tuple {
	if len(rows) == 0 {
		return nil
	}
	ct := (*C.keto_tuple)(m.alloc(len(rows) * int(C.sizeof_keto_tuple)))
	s := unsafe.Slice(ct, len(rows))
	for i := range rows {
		r := &rows[i]
		t := C.keto_tuple{namespace_id: C.int32_t(r.NamespaceID), object: m.s(r.Object), relation: m.s(r.Relation)}
		if r.SubjectID != nil {
			t.subject_kind = 0
			t.subject_id = m.s(*r.SubjectID)
		} else {
			t.subject_kind = 1
			t.set_namespace_id = C.int32_t(r.SetNamespaceID)
			t.set_object = m.s(r.SetObject)
			t.set_relation = m.s(r.SetRelation)
		}
		s[i] = t
	}
	return ct
}

// Build sorts the rows with the reference ORDER BY (relationtuples.go:250) and uploads the
// snapshot to HIP device `device` (-1: host only).
func Build(nss []*namespace.Namespace, rows []Row, device int) (*Snapshot, error) {
	var m cmem
	defer m.free()
	total := rowsLen(rows)
	for _, n := range nss {
		total += len(n.Name)
	}
	m.strings(total)
	var cns *C.keto_namespace
	if len(nss) > 0 {
		cns = (*C.keto_namespace)(m.alloc(len(nss) * int(C.sizeof_keto_namespace)))
		s := unsafe.Slice(cns, len(nss))
		for i, n := range nss {
			s[i] = C.keto_namespace{id: C.int32_t(n.ID), name: m.s(n.Name)}
		}
	}
	ct := m.tuples(rows)
	opts := C.keto_snapshot_opts{page_size: 100, device: C.int32_t(device)}
	var h *C.keto_snapshot
	if rc := C.keto_snapshot_build(cns, C.uint32_t(len(nss)), ct, C.uint64_t(len(rows)), &opts, &h); rc != C.KETO_OK {
		return nil, lastErr(rc)
	}
	return &Snapshot{h: h, device: device}, nil
}

// Clone makes a replica of the snapshot at its current version on another HIP device
// (keto_snapshot_clone): the host tables are copied and uploaded, nothing is scanned or sorted again.
func (s *Snapshot) Clone(device int) (*Snapshot, error) {
	var h *C.keto_snapshot
	if rc := C.keto_snapshot_clone(s.h, C.int32_t(device), &h); rc != C.KETO_OK {
		return nil, lastErr(rc)
	}
	return &Snapshot{h: h, Version: s.Version, device: device}, nil
}

// Save writes the snapshot's host tables at its current version to path (keto_snapshot_save),
// with the caller's tag: typically the table's last commit the snapshot covers, so that a restarting
// server loads the file and replays only the transactions committed after it instead of scanning
// and sorting the whole table again (internal/persistence/sql/relationtuples.go:249-251).
func (s *Snapshot) Save(path string, tag uint64) error {
	cp := C.CString(path)
	defer C.free(unsafe.Pointer(cp))
	if rc := C.keto_snapshot_save(s.h, cp, C.uint64_t(tag)); rc != C.KETO_OK {
		return lastErr(rc)
	}
	return nil
}

// Load reads a snapshot written by Save and uploads it to HIP device `device` (-1: host only);
// it returns the snapshot and the tag it was saved with.  A damaged, truncated or foreign file is
// an error (the caller rebuilds from the table).
func Load(path string, device int) (*Snapshot, uint64, error) {
	cp := C.CString(path)
	defer C.free(unsafe.Pointer(cp))
	var h *C.keto_snapshot
	var tag C.uint64_t
	if rc := C.keto_snapshot_load(cp, C.int32_t(device), &h, &tag); rc != C.KETO_OK {
		return nil, 0, lastErr(rc)
	}
	return &Snapshot{h: h, Version: uint64(C.keto_snapshot_version(h)), device: device}, uint64(tag), nil
}

// BuildReplicas builds one snapshot per device of a node (one server process driving every GPU):
// the rows are sorted and uploaded once by Build on devices[0], the other devices get clones.
func BuildReplicas(nss []*namespace.Namespace, rows []Row, devices []int) ([]*Snapshot, error) {
	if len(devices) == 0 {
		return nil, errors.New("gpu: no device")
	}
	first, err := Build(nss, rows, devices[0])
	if err != nil {
		return nil, err
	}
	out := []*Snapshot{first}
	for _, d := range devices[1:] {
		c, err := first.Clone(d)
		if err != nil {
			CloseAll(out)
			return nil, err
		}
		out = append(out, c)
	}
	return out, nil
}

// CloseAll closes every snapshot of a replica set.
func CloseAll(snaps []*Snapshot) {
	for _, s := range snaps {
		s.Close()
	}
}

// ApplyAll applies one transaction to every replica (see Apply).  An error from any replica leaves
// the set inconsistent: the caller rebuilds it (gpu.ErrRebuild or a device error alike).
func ApplyAll(snaps []*Snapshot, inserts, deletes []Row) error {
	for _, s := range snaps {
		if err := s.Apply(inserts, deletes); err != nil {
			return err
		}
	}
	return nil
}

// Close releases the host tables and the device arena.
func (s *Snapshot) Close() {
	if s.h != nil {
		C.keto_snapshot_release(s.h)
		s.h = nil
	}
	s.arenas.freeAll()
}

func subjectLen(sub relationtuple.Subject) int {
	switch v := sub.(type) {
	case *relationtuple.SubjectID:
		return len(v.ID)
	case *relationtuple.SubjectSet:
		return len(v.Namespace) + len(v.Object) + len(v.Relation)
	}
	return 0
}

func (m *cmem) subject(sub relationtuple.Subject) C.keto_subject {
	switch v := sub.(type) {
	case *relationtuple.SubjectID:
		return C.keto_subject{kind: 0, id: m.s(v.ID)}
	case *relationtuple.SubjectSet:
		return C.keto_subject{kind: 1, set_namespace: m.s(v.Namespace), set_object: m.s(v.Object),
			set_relation: m.s(v.Relation)}
	}
	return C.keto_subject{kind: 0} // nil subject: matches nothing
}

// CheckBatch = check.(*Engine).SubjectIsAllowed (internal/check/engine.go:116-123) for many
// requests: allowed[i] and status[i] (StatusUndecided: ask the SQL engine for request i).  The
// batch's strings go to the library packed back to back in one C buffer and are resolved on the GPU
// (keto_check_batch_packed); a batch holding a field longer than 65535 bytes takes keto_check_batch,
// which resolves on host threads.
func (s *Snapshot) CheckBatch(reqs []*relationtuple.InternalRelationTuple, depths []int, globalMax int) ([]bool, []uint8, error) {
	if out, st, ok, err := s.checkPacked(reqs, depths, globalMax); ok {
		return out, st, err
	}
	return checkWith(reqs, depths, false, func(cr *C.keto_check_req, n C.uint32_t, allowed, status *C.uint8_t) C.int {
		return C.keto_check_batch(s.h, cr, n, C.int32_t(globalMax), allowed, status)
	})
}

// packedFields are a request's fields in keto_check_packed order: namespace, object, relation, then
// the subject id or the subject set's namespace, object and relation.
func packedFields(r *relationtuple.InternalRelationTuple) ([6]string, int, uint8) {
	f := [6]string{r.Namespace, r.Object, r.Relation}
	switch v := r.Subject.(type) {
	case *relationtuple.SubjectID:
		f[3] = v.ID
		return f, 4, 0
	case *relationtuple.SubjectSet:
		f[3], f[4], f[5] = v.Namespace, v.Object, v.Relation
		return f, 6, 1
	}
	return f, 4, 0 // nil subject: an empty subject id, which matches nothing
}

// checkPacked runs the batch through keto_check_batch_packed; ok = false when a field does not fit
// a record (then nothing ran).
func (s *Snapshot) checkPacked(reqs []*relationtuple.InternalRelationTuple, depths []int, globalMax int) ([]bool, []uint8, bool, error) {
	n := len(reqs)
	if n == 0 {
		return nil, nil, true, nil
	}
	if len(depths) != n {
		return nil, nil, true, fmt.Errorf("gpu: %d requests, %d depths", n, len(depths))
	}
	total := 0
	for _, r := range reqs {
		f, k, _ := packedFields(r)
		for j := 0; j < k; j++ {
			if len(f[j]) > 65535 {
				return nil, nil, false, nil
			}
			total += len(f[j])
		}
	}
	if total >= 1<<32 {
		return nil, nil, false, nil
	}
	var m cmem
	defer m.free()
	// strings, records (8-B aligned), decisions and statuses: one pinned arena for a large batch
	strBytes := (total + 7) &^ 7
	recBytes := n * int(C.sizeof_keto_check_packed)
	var rec *C.keto_check_packed
	var allowed, status *C.uint8_t
	if size := strBytes + recBytes + 2*n; size >= pinMin {
		if a, base, ok := s.arenas.get(size); ok {
			defer s.arenas.put(a)
			m.str = base
			rec = (*C.keto_check_packed)(unsafe.Add(base, strBytes))
			allowed = (*C.uint8_t)(unsafe.Add(base, strBytes+recBytes))
			status = (*C.uint8_t)(unsafe.Add(base, strBytes+recBytes+n))
		}
	}
	if rec == nil {
		m.strings(total)
		rec = (*C.keto_check_packed)(m.alloc(recBytes))
		allowed = (*C.uint8_t)(m.alloc(n))
		status = (*C.uint8_t)(m.alloc(n))
	}
	rs := unsafe.Slice(rec, n)
	for i, r := range reqs {
		f, k, kind := packedFields(r)
		p := C.keto_check_packed{off: C.uint32_t(m.used), kind: C.uint8_t(kind), max_depth: C.int32_t(depths[i])}
		for j := 0; j < k; j++ {
			p.len[j] = C.uint16_t(len(f[j]))
			m.s(f[j])
		}
		rs[i] = p
	}
	if rc := C.keto_check_batch_packed(s.h, (*C.char)(m.str), C.uint64_t(m.used), rec, C.uint32_t(n),
		C.int32_t(globalMax), allowed, status); rc != C.KETO_OK {
		return nil, nil, true, lastErr(rc)
	}
	out := make([]bool, n)
	st := make([]uint8, n)
	as, ss := unsafe.Slice(allowed, n), unsafe.Slice(status, n)
	for i := range out {
		out[i] = as[i] == 1
		st[i] = uint8(ss[i])
	}
	return out, st, true, nil
}

// checkWith marshals the requests into C memory, runs call (one of the keto_check_batch* entry
// points taking keto_check_req) and unpacks its decisions and statuses.  collective: the call is a
// collective one (comm.go) and is made even for an empty batch, since the other ranks wait for it.
func checkWith(reqs []*relationtuple.InternalRelationTuple, depths []int, collective bool,
	call func(cr *C.keto_check_req, n C.uint32_t, allowed, status *C.uint8_t) C.int) ([]bool, []uint8, error) {
	n := len(reqs)
	if n == 0 && !collective {
		return nil, nil, nil
	}
	if len(depths) != n {
		return nil, nil, fmt.Errorf("gpu: %d requests, %d depths", n, len(depths))
	}
	var m cmem
	defer m.free()
	total := 0
	for _, r := range reqs {
		total += len(r.Namespace) + len(r.Object) + len(r.Relation) + subjectLen(r.Subject)
	}
	m.strings(total)
	cr := (*C.keto_check_req)(m.alloc(n * int(C.sizeof_keto_check_req)))
	cs := unsafe.Slice(cr, n)
	for i, r := range reqs {
		cs[i] = C.keto_check_req{namespace_: m.s(r.Namespace), object: m.s(r.Object), relation: m.s(r.Relation),
			subject: m.subject(r.Subject), max_depth: C.int32_t(depths[i])}
	}
	allowed := (*C.uint8_t)(m.alloc(n))
	status := (*C.uint8_t)(m.alloc(n))
	if rc := call(cr, C.uint32_t(n), allowed, status); rc != C.KETO_OK {
		return nil, nil, lastErr(rc)
	}
	out := make([]bool, n)
	st := make([]uint8, n)
	as, ss := unsafe.Slice(allowed, n), unsafe.Slice(status, n)
	for i := range out {
		out[i] = as[i] == 1
		st[i] = uint8(ss[i])
	}
	return out, st, nil
}

// Node is one node of an expand tree in pre-order (keto_tree_node): a leaf, or a union whose next
// Children subtrees follow it (internal/expand/tree.go:26-30; only union and leaf are produced).
type Node struct {
	Leaf     bool
	Children int
	Subject  relationtuple.Subject
}

// ExpandBatch = expand.(*Engine).BuildTree (internal/expand/engine.go:33-102) for many roots.
// trees[i] holds root i's nodes in pre-order (nil for a nil tree, JSON null); errs[i] is ErrNotFound /
// ErrUndecided per root.  Subjects are built from the node arena and keto_subject_fields: no text
// codec on the way.
func (s *Snapshot) ExpandBatch(subs []relationtuple.Subject, depths []int, globalMax int) ([][]Node, []error, error) {
	if len(subs) == 0 {
		return nil, nil, nil
	}
	return s.expandWith(subs, depths, func(cr *C.keto_expand_req, n C.uint32_t, a **C.keto_tree_arena) C.int {
		return C.keto_expand_batch(s.h, cr, n, C.int32_t(globalMax), a)
	})
}

// expandWith runs one expand entry point over the roots and reads its arena (an empty batch still
// makes the call: the routed form is collective).
func (s *Snapshot) expandWith(subs []relationtuple.Subject, depths []int,
	run func(cr *C.keto_expand_req, n C.uint32_t, a **C.keto_tree_arena) C.int) ([][]Node, []error, error) {
	n := len(subs)
	if len(depths) != n {
		return nil, nil, fmt.Errorf("gpu: %d roots, %d depths", n, len(depths))
	}
	var m cmem
	defer m.free()
	total := 0
	for _, sub := range subs {
		total += subjectLen(sub)
	}
	m.strings(total)
	cr := (*C.keto_expand_req)(m.alloc((n + 1) * int(C.sizeof_keto_expand_req)))
	cs := unsafe.Slice(cr, n)
	for i, sub := range subs {
		cs[i] = C.keto_expand_req{subject: m.subject(sub), max_depth: C.int32_t(depths[i])}
	}
	var a *C.keto_tree_arena
	if rc := run(cr, C.uint32_t(n), &a); rc != C.KETO_OK {
		return nil, nil, lastErr(rc)
	}
	defer C.keto_tree_arena_free(a)

	// the arena's nodes, tree by tree, and every distinct subject reference they hold
	type span struct{ nodes []C.keto_tree_node }
	spans := make([]span, n)
	errs := make([]error, n)
	refIdx := make(map[uint32]int)
	var refs []uint32
	for i := 0; i < n; i++ {
		switch C.keto_tree_status(a, C.uint32_t(i)) {
		case C.KETO_EXPAND_NIL:
			continue
		case C.KETO_EXPAND_NOT_FOUND:
			errs[i] = ErrNotFound
			continue
		case C.KETO_EXPAND_UNDECIDED:
			errs[i] = ErrUndecided
			continue
		}
		var nn C.uint64_t
		p := C.keto_tree_nodes(a, C.uint32_t(i), &nn)
		if p == nil || nn == 0 {
			continue
		}
		nodes := unsafe.Slice(p, int(nn)) // arena memory: read before keto_tree_arena_free
		spans[i].nodes = nodes
		for _, x := range nodes {
			ref := uint32(x.subject)
			if _, ok := refIdx[ref]; !ok {
				refIdx[ref] = len(refs)
				refs = append(refs, ref)
			}
		}
	}
	subjects, err := s.subjects(a, refs, &m)
	if err != nil {
		return nil, nil, err
	}
	trees := make([][]Node, n)
	for i := range spans {
		if spans[i].nodes == nil {
			continue
		}
		out := make([]Node, len(spans[i].nodes))
		for k, x := range spans[i].nodes {
			info := uint32(x.info)
			out[k] = Node{Leaf: info&0x80000000 != 0, Children: int(info & 0x7FFFFFFF),
				Subject: subjects[refIdx[uint32(x.subject)]]}
		}
		trees[i] = out
	}
	return trees, errs, nil
}

// subjects resolves subject references of arena a (keto_tree_node.subject) to Subjects with one
// keto_subject_fields sizing call and one filling call; a reference's strings never change, so the
// pair agrees even if a write lands in between (the fill is retried on a larger total regardless).
func (s *Snapshot) subjects(a *C.keto_tree_arena, refs []uint32, m *cmem) ([]relationtuple.Subject, error) {
	k := len(refs)
	if k == 0 {
		return nil, nil
	}
	cref := (*C.uint32_t)(m.alloc(k * 4))
	copy(unsafe.Slice((*uint32)(unsafe.Pointer(cref)), k), refs)
	lens := (*C.uint32_t)(m.alloc(3 * k * 4))
	total := C.keto_subject_fields(s.h, a, cref, C.uint64_t(k), nil, 0, lens)
	for {
		if total < 0 {
			return nil, lastErr(C.int(total))
		}
		buf := (*C.char)(m.alloc(int(total) + 1))
		got := C.keto_subject_fields(s.h, a, cref, C.uint64_t(k), buf, C.uint64_t(total), lens)
		if got < 0 {
			return nil, lastErr(C.int(got))
		}
		if got > total { // cannot happen (see above); size again rather than misread
			total = got
			continue
		}
		text := C.GoStringN(buf, C.int(got)) // one Go string; the fields are substrings of it
		ls := unsafe.Slice((*uint32)(unsafe.Pointer(lens)), 3*k)
		out := make([]relationtuple.Subject, k)
		at := 0
		take := func(n uint32) string {
			v := text[at : at+int(n)]
			at += int(n)
			return v
		}
		for i, ref := range refs {
			if ref&0x80000000 == 0 {
				out[i] = &relationtuple.SubjectID{ID: take(ls[3*i])}
				continue
			}
			ns := take(ls[3*i])
			obj := take(ls[3*i+1])
			out[i] = &relationtuple.SubjectSet{Namespace: ns, Object: obj, Relation: take(ls[3*i+2])}
		}
		return out, nil
	}
}
