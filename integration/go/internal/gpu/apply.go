//go:build keto_gpu
// +build keto_gpu

package gpu

/*
#include "keto_mi355x.h"
*/
import "C"

import (
	"context"
	"errors"

	"github.com/ory/keto/internal/namespace"
	"github.com/ory/keto/internal/relationtuple"
)

// ErrRebuild: the write touches a poisoned row (a tuple of an unconfigured namespace) or a wildcard
// row that matches one.  The snapshot is unchanged; build a new one from the table
// (keto_snapshot_apply, KETO_E_REBUILD).  New Subject.String() collisions, wildcard subject sets and
// writes to a shared-rows part of an edge-partitioned snapshot are applied in place.
var ErrRebuild = errors.New("keto_mi355x: write needs a snapshot rebuild")

// Apply patches the snapshot with one transaction of TransactRelationTuples
// (internal/persistence/sql/relationtuples.go:279-297): inserts land after the equal tuples already
// in their row (commit order), deletes remove every equal tuple.  The library takes the snapshot's
// lock exclusively, so running batches finish on the old version first.  Version is the snaptoken
// the reference leaves "not yet implemented" (internal/check/handler.go:182).
func (s *Snapshot) Apply(inserts, deletes []Row) error {
	var m cmem
	defer m.free()
	m.strings(rowsLen(inserts) + rowsLen(deletes))
	ci := m.tuples(inserts)
	cd := m.tuples(deletes)
	var v C.uint64_t
	rc := C.keto_snapshot_apply(s.h, ci, C.uint64_t(len(inserts)), cd, C.uint64_t(len(deletes)), &v)
	if rc == C.KETO_E_REBUILD {
		return ErrRebuild
	}
	if rc != C.KETO_OK {
		return lastErr(rc)
	}
	s.Version = uint64(v)
	return nil
}

// RowsOf maps the tuples of one TransactRelationTuples call to table rows with the namespace name ->
// id lookups RelationTuple.FromInternal / insertSubject make before the SQL insert
// (internal/persistence/sql/relationtuples.go:82-130).  The persister calls Apply with them after
// its transaction commits, so the snapshot follows the table one transaction at a time.
func RowsOf(ctx context.Context, nm namespace.Manager, ts []*relationtuple.InternalRelationTuple) ([]Row, error) {
	rows := make([]Row, 0, len(ts))
	for _, t := range ts {
		n, err := nm.GetNamespaceByName(ctx, t.Namespace)
		if err != nil {
			return nil, err
		}
		r := Row{NamespaceID: n.ID, Object: t.Object, Relation: t.Relation}
		switch s := t.Subject.(type) {
		case *relationtuple.SubjectID:
			id := s.ID
			r.SubjectID = &id
		case *relationtuple.SubjectSet:
			sn, err := nm.GetNamespaceByName(ctx, s.Namespace)
			if err != nil {
				return nil, err
			}
			r.SetNamespaceID, r.SetObject, r.SetRelation = sn.ID, s.Object, s.Relation
		}
		rows = append(rows, r)
	}
	return rows, nil
}
