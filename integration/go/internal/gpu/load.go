//go:build keto_gpu
// +build keto_gpu

package gpu

import (
	"context"
	"database/sql"

	"github.com/gofrs/uuid"

	"github.com/ory/keto/internal/namespace"
)

// LoadRows reads network nid's rows of keto_relation_tuples in commit order (ties of the reference
// ORDER BY, relationtuples.go:250, are broken by commit_time; the snapshot builder sorts the rest).
// One full scan replaces the per-node paged queries of GetRelationTuples (relationtuples.go:238-277).
func LoadRows(ctx context.Context, db *sql.DB, nid uuid.UUID) ([]Row, error) {
	rs, err := db.QueryContext(ctx, `SELECT namespace_id, object, relation, subject_id, subject_set_namespace_id,
		subject_set_object, subject_set_relation FROM keto_relation_tuples WHERE nid = ? ORDER BY commit_time`, nid)
	if err != nil {
		return nil, err
	}
	defer rs.Close()
	var rows []Row
	for rs.Next() {
		var r Row
		var sid, sobj, srel sql.NullString
		var sns sql.NullInt32
		if err := rs.Scan(&r.NamespaceID, &r.Object, &r.Relation, &sid, &sns, &sobj, &srel); err != nil {
			return nil, err
		}
		if sid.Valid {
			v := sid.String
			r.SubjectID = &v
		} else {
			r.SetNamespaceID, r.SetObject, r.SetRelation = sns.Int32, sobj.String, srel.String
		}
		rows = append(rows, r)
	}
	return rows, rs.Err()
}

// BuildFromDB is what the registry runs once after Init (internal/driver/registry_default.go:241-262):
// namespaces in config order (config.NamespaceManager, internal/driver/config/provider.go:190-218).
func BuildFromDB(ctx context.Context, db *sql.DB, nid uuid.UUID, nss []*namespace.Namespace, device int) (*Snapshot, error) {
	rows, err := LoadRows(ctx, db, nid)
	if err != nil {
		return nil, err
	}
	return Build(nss, rows, device)
}
