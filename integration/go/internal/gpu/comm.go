//go:build keto_gpu
// +build keto_gpu

package gpu

/*
#include <stdlib.h>
#include "keto_mi355x.h"
*/
import "C"

import (
	"fmt"
	"unsafe"

	"github.com/ory/keto/internal/relationtuple"
)

// Comm is the library's communicator (keto_comm, include/keto_mi355x.h): over RCCL between processes
// (NewComm, one process per GPU), or between goroutines of one server process (NewLocalComm; the
// reference serves from one process, internal/driver/daemon.go:62-69).  Every method is collective:
// all ranks call it, an empty batch included; an error on one rank is returned by every rank.
type Comm struct {
	h *C.keto_comm
}

// NewCommID makes a communicator id on one rank (keto_comm_id); send its bytes to every rank over
// the deployment's own channel, then every rank calls NewComm with them.
func NewCommID() ([]byte, error) {
	buf := (*C.uint8_t)(C.malloc(C.KETO_COMM_ID_BYTES))
	defer C.free(unsafe.Pointer(buf))
	if rc := C.keto_comm_id(buf); rc != C.KETO_OK {
		return nil, lastErr(rc)
	}
	return C.GoBytes(unsafe.Pointer(buf), C.KETO_COMM_ID_BYTES), nil
}

// NewComm joins the communicator as rank of ranks, on GPU device (keto_comm_init).
func NewComm(id []byte, ranks, rank, device int) (*Comm, error) {
	if len(id) != C.KETO_COMM_ID_BYTES {
		return nil, fmt.Errorf("gpu: communicator id of %d bytes, want %d", len(id), C.KETO_COMM_ID_BYTES)
	}
	cid := C.CBytes(id)
	defer C.free(cid)
	var h *C.keto_comm
	if rc := C.keto_comm_init((*C.uint8_t)(cid), C.int32_t(ranks), C.int32_t(rank), C.int32_t(device), &h); rc != C.KETO_OK {
		return nil, lastErr(rc)
	}
	return &Comm{h: h}, nil
}

// NewLocalComm joins an in-process communicator (keto_comm_init_local): the ranks are goroutines of
// this one server process, each rank's collective calls made from its own goroutine (a blocked cgo
// call holds its own OS thread) and driving its own part of an edge-partitioned snapshot on GPU
// device; the exchanges are device copies (peer copies over xGMI).
// id is any KETO_COMM_ID_BYTES the process chooses, the same for every rank.
func NewLocalComm(id []byte, ranks, rank, device int) (*Comm, error) {
	if len(id) != C.KETO_COMM_ID_BYTES {
		return nil, fmt.Errorf("gpu: communicator id of %d bytes, want %d", len(id), C.KETO_COMM_ID_BYTES)
	}
	cid := C.CBytes(id)
	defer C.free(cid)
	var h *C.keto_comm
	if rc := C.keto_comm_init_local((*C.uint8_t)(cid), C.int32_t(ranks), C.int32_t(rank), C.int32_t(device), &h); rc != C.KETO_OK {
		return nil, lastErr(rc)
	}
	return &Comm{h: h}, nil
}

// Close frees the communicator (keto_comm_free).
func (c *Comm) Close() {
	if c.h != nil {
		C.keto_comm_free(c.h)
		c.h = nil
	}
}

// CheckBatchSharded decides a batch every rank passes identically on a replicated snapshot: each
// rank checks its contiguous shard, one all-gather returns every decision to every rank
// (keto_check_batch_sharded).
func (c *Comm) CheckBatchSharded(s *Snapshot, reqs []*relationtuple.InternalRelationTuple, depths []int, globalMax int) ([]bool, []uint8, error) {
	return checkWith(reqs, depths, true, func(cr *C.keto_check_req, n C.uint32_t, allowed, status *C.uint8_t) C.int {
		return C.keto_check_batch_sharded(c.h, s.h, cr, n, C.int32_t(globalMax), allowed, status)
	})
}

// CheckBatchRouted decides this rank's own batch on an edge-partitioned snapshot: requests travel
// to the parts owning their rows and their decisions come back (keto_check_batch_routed).
func (c *Comm) CheckBatchRouted(s *Snapshot, reqs []*relationtuple.InternalRelationTuple, depths []int, globalMax int) ([]bool, []uint8, error) {
	return checkWith(reqs, depths, true, func(cr *C.keto_check_req, n C.uint32_t, allowed, status *C.uint8_t) C.int {
		return C.keto_check_batch_routed(c.h, s.h, cr, n, C.int32_t(globalMax), allowed, status)
	})
}

// packedFits reports whether every request of a batch fits a keto_check_packed record (fields of
// at most 65,535 bytes, strings below 4 GiB): a partitioned batch then goes packed on every rank
// (CheckBatchRoutedPacked), else by name on every rank -- the ranks of one collective call agree.
func packedFits(reqs []*relationtuple.InternalRelationTuple) bool {
	total := 0
	for _, r := range reqs {
		f, k, _ := packedFields(r)
		for j := 0; j < k; j++ {
			if len(f[j]) > 65535 {
				return false
			}
			total += len(f[j])
		}
	}
	return total < 1<<32
}

// CheckBatchRoutedPacked is CheckBatchRouted with the batch packed into one string blob and 24-B
// records and resolved on this rank's device (keto_check_batch_routed_packed) instead of on host
// threads.  Collective: every rank calls it, with an empty batch too; every request must fit a
// record (packedFits).
func (c *Comm) CheckBatchRoutedPacked(s *Snapshot, reqs []*relationtuple.InternalRelationTuple, depths []int, globalMax int) ([]bool, []uint8, error) {
	n := len(reqs)
	if len(depths) != n {
		return nil, nil, fmt.Errorf("gpu: %d requests, %d depths", n, len(depths))
	}
	var m cmem
	defer m.free()
	total := 0
	for _, r := range reqs {
		f, k, _ := packedFields(r)
		for j := 0; j < k; j++ {
			total += len(f[j])
		}
	}
	m.strings(total)
	rec := (*C.keto_check_packed)(m.alloc(n * int(C.sizeof_keto_check_packed)))
	allowed := (*C.uint8_t)(m.alloc(n))
	status := (*C.uint8_t)(m.alloc(n))
	if n > 0 {
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
	}
	if rc := C.keto_check_batch_routed_packed(c.h, s.h, (*C.char)(m.str), C.uint64_t(m.used), rec, C.uint32_t(n),
		C.int32_t(globalMax), allowed, status); rc != C.KETO_OK {
		return nil, nil, lastErr(rc)
	}
	out := make([]bool, n)
	st := make([]uint8, n)
	if n > 0 {
		as, ss := unsafe.Slice(allowed, n), unsafe.Slice(status, n)
		for i := range out {
			out[i] = as[i] == 1
			st[i] = uint8(ss[i])
		}
	}
	return out, st, nil
}

// ExpandBatchRouted is BuildTree (internal/expand/engine.go:33-102) for this rank's roots over an
// edge-partitioned snapshot of shared-rows parts (keto_expand_batch_routed): a root row another
// part owns is expanded there.  Collective: every rank calls it, with an empty batch too.
func (c *Comm) ExpandBatchRouted(s *Snapshot, subs []relationtuple.Subject, depths []int, globalMax int) ([][]Node, []error, error) {
	return s.expandWith(subs, depths, func(cr *C.keto_expand_req, n C.uint32_t, a **C.keto_tree_arena) C.int {
		return C.keto_expand_batch_routed(c.h, s.h, cr, n, C.int32_t(globalMax), a)
	})
}

// CloseFilters runs a migrating partition's closure-filter exchange once after upload
// (keto_comm_close_filters); it returns the rounds it took.
func (c *Comm) CloseFilters(s *Snapshot) (int, error) {
	var rounds C.uint32_t
	if rc := C.keto_comm_close_filters(c.h, s.h, &rounds); rc != C.KETO_OK {
		return 0, lastErr(rc)
	}
	return int(rounds), nil
}
