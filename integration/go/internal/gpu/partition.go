//go:build keto_gpu
// +build keto_gpu

package gpu

/*
#include "keto_mi355x.h"
*/
import "C"

import (
	"crypto/rand"
	"errors"
	"sync"

	"github.com/ory/keto/internal/relationtuple"
)

// Engine is what the check and expand batchers deal a batch to: one snapshot replica on one GPU, or
// a whole partition over several GPUs.  Apply follows one committed write transaction; Close
// releases it.
type Engine interface {
	CheckBatch(reqs []*relationtuple.InternalRelationTuple, depths []int, globalMax int) ([]bool, []uint8, error)
	ExpandBatch(subs []relationtuple.Subject, depths []int, globalMax int) ([][]Node, []error, error)
	Apply(inserts, deletes []Row) error
	Footprint() map[int]uint64
	Close()
}

// Footprint is the device memory the snapshot's arena and tables hold, by HIP device
// (keto_snapshot_get_stats; empty for a host-only snapshot).
func (s *Snapshot) Footprint() map[int]uint64 {
	out := map[int]uint64{}
	var st C.keto_snapshot_stats
	if s.device >= 0 && C.keto_snapshot_get_stats(s.h, &st) == C.KETO_OK {
		out[s.device] = uint64(st.device_bytes)
	}
	return out
}

// Footprint of a partition: its parts' device memory, by device.
func (p *Partition) Footprint() map[int]uint64 {
	out := map[int]uint64{}
	for _, s := range p.parts {
		for d, b := range s.Footprint() {
			out[d] += b
		}
	}
	return out
}

// FootprintOf sums the device memory an engine set holds, by device: what a rebuild's placement
// credits back while the outgoing set is still on the devices (PlaceWith).
func FootprintOf(es []Engine) map[int]uint64 {
	out := map[int]uint64{}
	for _, e := range es {
		for d, b := range e.Footprint() {
			out[d] += b
		}
	}
	return out
}

// Engines views a replica set as engines.
func Engines(snaps []*Snapshot) []Engine {
	out := make([]Engine, len(snaps))
	for i, s := range snaps {
		out[i] = s
	}
	return out
}

// DeviceMemory is the free and total memory of HIP device d (keto_device_memory).
func DeviceMemory(d int) (free, total uint64, err error) {
	var f, t C.uint64_t
	if rc := C.keto_device_memory(C.int32_t(d), &f, &t); rc != C.KETO_OK {
		return 0, 0, lastErr(rc)
	}
	return uint64(f), uint64(t), nil
}

// PartArenaBytes is the device arena part `part` of nParts shared-rows parts of this host-only
// snapshot would take (keto_snapshot_part_stats_mode); nParts = 1 is the replicated arena.
func (s *Snapshot) PartArenaBytes(part, nParts int) (uint64, error) {
	var st C.keto_part_stats
	if rc := C.keto_snapshot_part_stats_mode(s.h, C.uint32_t(part), C.uint32_t(nParts), C.KETO_PART_SHARED, &st); rc != C.KETO_OK {
		return 0, lastErr(rc)
	}
	return uint64(st.arena_bytes), nil
}

// PartStats is what part `part` of nParts shared-rows parts of this host-only snapshot would take on
// a device: its arena, and of it the rows every part keeps (the subject-set targets).
func (s *Snapshot) PartStats(part, nParts int) (arena, shared uint64, err error) {
	var st C.keto_part_stats
	if rc := C.keto_snapshot_part_stats_mode(s.h, C.uint32_t(part), C.uint32_t(nParts), C.KETO_PART_SHARED, &st); rc != C.KETO_OK {
		return 0, 0, lastErr(rc)
	}
	return uint64(st.arena_bytes), uint64(st.shared_bytes), nil
}

// UploadPart uploads this host-only snapshot as part `part` of nParts shared-rows parts on HIP
// device `device` (keto_snapshot_upload_part_mode, KETO_PART_SHARED): the rows subject sets point at
// on every part, each root row on the part hash(namespace, object) picks.
func (s *Snapshot) UploadPart(part, nParts, device int) error {
	if rc := C.keto_snapshot_upload_part_mode(s.h, C.uint32_t(part), C.uint32_t(nParts), C.int32_t(device), C.KETO_PART_SHARED); rc != C.KETO_OK {
		return lastErr(rc)
	}
	s.device = device
	return nil
}

// workspaceBytes is what a device keeps beside its arena for the engine's tiers, visited tables,
// expand staging and request buffers (the deep tiers and the expand staging pool take the most).
const workspaceBytes = 12 << 30

// placementFree is the memory of device d a placement may count on: what is free now plus what
// `resident` (an outgoing engine set that a rebuild replaces) holds there, so that the placement
// depends on the graph and the devices, not on whether the previous set is still loaded.
func placementFree(d int, resident map[int]uint64) (uint64, error) {
	free, total, err := DeviceMemory(d)
	if err != nil {
		return 0, err
	}
	free += resident[d]
	if free > total {
		free = total
	}
	return free, nil
}

// Fits reports whether an arena of `arena` bytes and the engine's workspaces fit on every device.
func Fits(arena uint64, devices []int) (bool, error) { return fitsWith(arena, devices, nil) }

func fitsWith(arena uint64, devices []int, resident map[int]uint64) (bool, error) {
	for _, d := range devices {
		free, err := placementFree(d, resident)
		if err != nil {
			return false, err
		}
		if arena+arena/8+workspaceBytes > free { // + room for the rows writes add
			return false, nil
		}
	}
	return true, nil
}

// Partition is a graph too large for one replica, edge-partitioned over the devices of the server
// process: shared-rows parts (subject-set targets on every part, root rows by hash), one or more per
// device (PlanParts), and one in-process communicator rank per part (keto_comm_init_local).  It answers batches like a
// snapshot does: a batch is split over the ranks and every rank calls the collective routed entry
// point with its slice -- an empty slice too -- on its own goroutine, so each request travels to
// the part owning its row and its decision (or tree) comes back.  Batches run one at a time; every
// write transaction is applied to every part (each holds the whole graph's host tables).
type Partition struct {
	mu    sync.Mutex
	parts []*Snapshot
	comms []*Comm
}

// NewPartition partitions the host-only snapshot base over devices, one part per entry (a device
// may appear more than once: its parts are separate ranks on it); base becomes part 0 (the partition
// owns it), the other parts are host-only clones of it.
func NewPartition(base *Snapshot, devices []int) (*Partition, error) {
	if len(devices) == 0 {
		return nil, errors.New("gpu: no device")
	}
	p := &Partition{parts: []*Snapshot{base}}
	for range devices[1:] {
		c, err := base.Clone(-1)
		if err != nil {
			p.Close()
			return nil, err
		}
		p.parts = append(p.parts, c)
	}
	for k, d := range devices {
		if err := p.parts[k].UploadPart(k, len(devices), d); err != nil {
			p.Close()
			return nil, err
		}
	}
	id := make([]byte, C.KETO_COMM_ID_BYTES)
	if _, err := rand.Read(id); err != nil {
		p.Close()
		return nil, err
	}
	p.comms = make([]*Comm, len(devices))
	errs := p.ranks(func(k int) error {
		c, err := NewLocalComm(id, len(devices), k, devices[k])
		p.comms[k] = c
		return err
	})
	if err := firstErr(errs); err != nil {
		p.Close()
		return nil, err
	}
	return p, nil
}

// ranks runs fn(k) for every rank at once, each on its own goroutine (a collective call blocks its
// OS thread until every rank has arrived), and returns each rank's error.
func (p *Partition) ranks(fn func(k int) error) []error {
	errs := make([]error, len(p.parts))
	var wg sync.WaitGroup
	for k := range p.parts {
		wg.Add(1)
		go func(k int) {
			defer wg.Done()
			errs[k] = fn(k)
		}(k)
	}
	wg.Wait()
	return errs
}

func firstErr(errs []error) error {
	for _, e := range errs {
		if e != nil {
			return e
		}
	}
	return nil
}

// slice bounds of rank k's share of n requests
func share(n, k, ranks int) (int, int) { return n * k / ranks, n * (k + 1) / ranks }

// CheckBatch = SubjectIsAllowed for many requests over the partition (keto_check_batch_routed).
func (p *Partition) CheckBatch(reqs []*relationtuple.InternalRelationTuple, depths []int, globalMax int) ([]bool, []uint8, error) {
	p.mu.Lock()
	defer p.mu.Unlock()
	allowed := make([]bool, len(reqs))
	status := make([]uint8, len(reqs))
	// resolved on every rank's device when every request fits a packed record (the same choice on
	// every rank: one collective call), else on host threads by name
	packed := packedFits(reqs)
	errs := p.ranks(func(k int) error {
		lo, hi := share(len(reqs), k, len(p.parts))
		call := p.comms[k].CheckBatchRouted
		if packed {
			call = p.comms[k].CheckBatchRoutedPacked
		}
		a, st, err := call(p.parts[k], reqs[lo:hi], depths[lo:hi], globalMax)
		if err != nil {
			return err
		}
		copy(allowed[lo:hi], a)
		copy(status[lo:hi], st)
		return nil
	})
	if err := firstErr(errs); err != nil { // agreed: every rank returned the failing rank's code
		return nil, nil, err
	}
	return allowed, status, nil
}

// ExpandBatch = BuildTree for many roots over the partition (keto_expand_batch_routed).
func (p *Partition) ExpandBatch(subs []relationtuple.Subject, depths []int, globalMax int) ([][]Node, []error, error) {
	p.mu.Lock()
	defer p.mu.Unlock()
	trees := make([][]Node, len(subs))
	terrs := make([]error, len(subs))
	errs := p.ranks(func(k int) error {
		lo, hi := share(len(subs), k, len(p.parts))
		t, e, err := p.comms[k].ExpandBatchRouted(p.parts[k], subs[lo:hi], depths[lo:hi], globalMax)
		if err != nil {
			return err
		}
		copy(trees[lo:hi], t)
		copy(terrs[lo:hi], e)
		return nil
	})
	if err := firstErr(errs); err != nil {
		return nil, nil, err
	}
	return trees, terrs, nil
}

// Apply follows one committed write transaction on every part (see Snapshot.Apply).  An error
// leaves the parts inconsistent: the caller rebuilds the partition.
func (p *Partition) Apply(inserts, deletes []Row) error {
	p.mu.Lock()
	defer p.mu.Unlock()
	// the parts are independent snapshots: each applies the transaction on its own goroutine (a
	// migrating part lays itself out afresh, seconds at the 1B-tuple scale, so serially P times that)
	return firstErr(p.ranks(func(k int) error { return p.parts[k].Apply(inserts, deletes) }))
}

// Close releases the communicators and the parts.
func (p *Partition) Close() {
	for _, c := range p.comms {
		if c != nil {
			c.Close()
		}
	}
	for _, s := range p.parts {
		s.Close()
	}
	p.comms, p.parts = nil, nil
}

// arenaCap is the largest arena a replica or a part takes on a device (KETO_ARENA_MAX_BYTES: handles
// are 32-bit counts of 16-byte units, or of up to 128-byte units for the root rows past 32 GiB).
const arenaCap = uint64(C.KETO_ARENA_MAX_BYTES)

// maxParts bounds the partitions PlanParts tries (every part holds all the subject-set targets).
const maxParts = 64

// PlanParts picks the shared-rows parts of a snapshot that does not fit a replica, and the device of
// each: the fewest parts -- at least one per device, dealt to the devices in turn, so a device may
// hold several -- such that every part's arena stays within arenaCap and each device's parts fit its
// free memory.  Part sizes are estimated from the one-part statistics (every part keeps the targets,
// the root rows split by hash; an eighth of margin), and the first plan the estimate admits is then
// checked part by part.  A graph whose arena passes 288 GiB is so served from one GPU too.
func PlanParts(base *Snapshot, devices []int) ([]int, error) { return planPartsWith(base, devices, nil) }

func planPartsWith(base *Snapshot, devices []int, resident map[int]uint64) ([]int, error) {
	if len(devices) == 0 {
		return nil, errors.New("gpu: no device")
	}
	total, shared, err := base.PartStats(0, 1)
	if err != nil {
		return nil, err
	}
	free := make([]uint64, len(devices))
	for i, d := range devices {
		if free[i], err = placementFree(d, resident); err != nil {
			return nil, err
		}
	}
	roots := uint64(0)
	if total > shared {
		roots = total - shared
	}
	fits := func(P int, arena func(k int) (uint64, error)) (bool, error) {
		load := make([]uint64, len(devices))
		for k := 0; k < P; k++ {
			a, err := arena(k)
			if err != nil {
				return false, err
			}
			if a > arenaCap {
				return false, nil
			}
			load[k%len(devices)] += a + a/8 + workspaceBytes // + room for the rows writes add
		}
		for i := range devices {
			if load[i] > free[i] {
				return false, nil
			}
		}
		return true, nil
	}
	for P := len(devices); P <= maxParts; P++ {
		est := func(int) (uint64, error) { return shared + roots/uint64(P) + roots/uint64(8*P), nil }
		ok, err := fits(P, est)
		if err != nil {
			return nil, err
		}
		if !ok {
			continue
		}
		if ok, err = fits(P, func(k int) (uint64, error) { return base.PartArenaBytes(k, P) }); err != nil {
			return nil, err
		}
		if ok {
			plan := make([]int, P)
			for k := range plan {
				plan[k] = devices[k%len(devices)]
			}
			return plan, nil
		}
	}
	return nil, errors.New("gpu: no partition of the snapshot fits the devices")
}

// Place builds the engines for a host-only snapshot base (consumed) on devices: replicas -- base
// cloned to every device -- when the replicated arena is within arenaCap and fits each of them (mode
// "" or "auto") or when mode is "replicate"; else (or with mode "partition") one Partition over the
// parts PlanParts picks (one per device, or more when a part would pass arenaCap).
func Place(base *Snapshot, devices []int, mode string) ([]Engine, error) {
	return PlaceWith(base, devices, mode, nil)
}

// PlaceWith is Place for a rebuild: resident is the device memory the outgoing engine set still
// holds (FootprintOf), counted as free, so the new set is placed as the graph requires (replicas or a
// partition) and not pushed into a partition by the set it replaces.
func PlaceWith(base *Snapshot, devices []int, mode string, resident map[int]uint64) ([]Engine, error) {
	if len(devices) == 0 {
		base.Close()
		return nil, errors.New("gpu: no device")
	}
	replicate := mode == "replicate"
	if mode == "" || mode == "auto" {
		arena, err := base.PartArenaBytes(0, 1)
		if err != nil {
			base.Close()
			return nil, err
		}
		if replicate, err = fitsWith(arena, devices, resident); err != nil {
			base.Close()
			return nil, err
		}
		replicate = replicate && arena <= arenaCap
	}
	if !replicate {
		plan, err := planPartsWith(base, devices, resident)
		if err != nil {
			base.Close()
			return nil, err
		}
		p, err := NewPartition(base, plan)
		if err != nil {
			return nil, err
		}
		return []Engine{p}, nil
	}
	var out []*Snapshot
	for _, d := range devices {
		c, err := base.Clone(d)
		if err != nil {
			CloseAll(out)
			base.Close()
			return nil, err
		}
		out = append(out, c)
	}
	base.Close()
	return Engines(out), nil
}

// ApplyEngines applies one transaction to every engine of a set (see Snapshot.Apply).  An error
// leaves the set inconsistent: the caller rebuilds it (gpu.ErrRebuild or a device error alike).
func ApplyEngines(es []Engine, inserts, deletes []Row) error {
	for _, e := range es {
		if err := e.Apply(inserts, deletes); err != nil {
			return err
		}
	}
	return nil
}

// CloseEngines closes every engine of a set.
func CloseEngines(es []Engine) {
	for _, e := range es {
		e.Close()
	}
}

// Fingerprint identifies the table's contents for a persisted snapshot (Snapshot.Save's tag): an
// order-independent hash of the multiset of rows (a sum of per-row hashes) mixed with their count.
// Any committed write changes it -- an insert adds a row's hash, a delete removes one (duplicates
// included) -- whatever the rows' commit_time (the reference sets it from the app clock,
// relationtuples.go:137, and a MySQL TIMESTAMP keeps whole seconds only), so a restarting server
// never loads a file whose contents differ from the table's.
func Fingerprint(rows []Row) uint64 {
	var sum uint64
	for i := range rows {
		r := &rows[i]
		h := uint64(1469598103934665603)
		add := func(b string) {
			for k := 0; k < len(b); k++ {
				h = (h ^ uint64(b[k])) * 1099511628211
			}
			h = (h ^ uint64(len(b))) * 1099511628211 // field boundaries: "ab","c" != "a","bc"
		}
		h = (h ^ uint64(uint32(r.NamespaceID))) * 1099511628211
		add(r.Object)
		add(r.Relation)
		if r.SubjectID != nil {
			h = (h ^ 1) * 1099511628211
			add(*r.SubjectID)
		} else {
			h = (h ^ 2 ^ uint64(uint32(r.SetNamespaceID))<<8) * 1099511628211
			add(r.SetObject)
			add(r.SetRelation)
		}
		sum += mix64(h)
	}
	return mix64(sum ^ mix64(uint64(len(rows))+0x9E3779B97F4A7C15))
}

func mix64(x uint64) uint64 {
	x ^= x >> 31
	x *= 0xBF58476D1CE4E5B9
	x ^= x >> 29
	x *= 0x94D049BB133111EB
	return x ^ x>>32
}

