//go:build keto_gpu
// +build keto_gpu

package sql

import (
	"context"

	"github.com/ory/x/sqlcon"

	"github.com/ory/keto/internal/gpu"
)

// snapshotChunk is the page size of the full scan (keyset pagination, so the scan stays linear).
const snapshotChunk = 1 << 20

// SnapshotRows reads this network's rows of keto_relation_tuples in commit order, the one full
// scan the GPU snapshot is built from instead of the per-node paged queries of GetRelationTuples
// (relationtuples.go:238-277).  Ties of the reference ORDER BY (relationtuples.go:250) end in
// commit_time, so commit order is all the builder needs; it sorts the rest itself.  Rows whose
// namespace id is not configured are kept: they are the poisoned pages the engines must reproduce.
func (p *Persister) SnapshotRows(ctx context.Context) ([]gpu.Row, error) {
	var out []gpu.Row
	var last *RelationTuple
	for {
		q := p.QueryWithNetwork(ctx).Order("commit_time, shard_id").Limit(snapshotChunk)
		if last != nil {
			q = q.Where("(commit_time > ?) OR (commit_time = ? AND shard_id > ?)", last.CommitTime, last.CommitTime, last.ID)
		}
		var res relationTuples
		if err := q.All(&res); err != nil {
			return nil, sqlcon.HandleError(err)
		}
		for _, r := range res {
			row := gpu.Row{NamespaceID: r.NamespaceID, Object: r.Object, Relation: r.Relation}
			if r.SubjectID.Valid {
				id := r.SubjectID.String
				row.SubjectID = &id
			} else {
				row.SetNamespaceID = r.SubjectSetNamespaceID.Int32
				row.SetObject = r.SubjectSetObject.String
				row.SetRelation = r.SubjectSetRelation.String
			}
			out = append(out, row)
		}
		if len(res) < snapshotChunk {
			return out, nil
		}
		last = res[len(res)-1]
	}
}
