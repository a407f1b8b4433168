//go:build keto_gpu
// +build keto_gpu

package check

import (
	"context"

	"github.com/ory/keto/internal/gpu"
	"github.com/ory/keto/internal/relationtuple"
)

// GPUProvider is implemented by the registry once a GPU snapshot is loaded
// (internal/driver/registry_default.go:159-164 constructs the engine; registry_gpu.go's EnableGPU
// builds the snapshot after Init, :241-262).  A nil batcher means "no current snapshot" (none loaded,
// or one behind the table while it is rebuilt): the SQL path runs.
type GPUProvider interface {
	GPUCheckBatcher() *gpu.Batcher
}

// SubjectIsAllowed dispatch, the one change to internal/check/engine.go:116-123: the existing
// body is renamed subjectIsAllowedSQL (its depth clamp and checkOneIndirectionFurther call stay as
// they are) and becomes the batcher's fallback for requests the GPU leaves undecided.
//
//	func (e *Engine) SubjectIsAllowed(ctx context.Context, r *relationtuple.InternalRelationTuple, restDepth int) (bool, error) {
//		if b := e.gpuBatcher(); b != nil {
//			return b.Check(ctx, r, restDepth)
//		}
//		return e.subjectIsAllowedSQL(ctx, r, restDepth)
//	}
func (e *Engine) gpuBatcher() *gpu.Batcher {
	if p, ok := e.d.(GPUProvider); ok {
		return p.GPUCheckBatcher()
	}
	return nil
}

// Fallback for gpu.NewBatcher: the reference engine on its own goroutine.
func (e *Engine) Fallback() gpu.Fallback {
	return func(ctx context.Context, r *relationtuple.InternalRelationTuple, restDepth int) (bool, error) {
		return e.subjectIsAllowedSQL(ctx, r, restDepth)
	}
}
