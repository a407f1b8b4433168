//go:build keto_gpu
// +build keto_gpu

package expand

import (
	"context"
	"errors"

	"github.com/ory/keto/internal/gpu"
	"github.com/ory/keto/internal/relationtuple"
)

// GPUProvider is implemented by the registry once a GPU snapshot is loaded
// (internal/driver/registry_default.go:166-171 constructs the engine; registry_gpu.go implements
// it).  A nil batcher means "no current snapshot": the SQL path runs.
type GPUProvider interface {
	GPUExpandBatcher() *gpu.ExpandBatcher
}

// BuildTree dispatch, the one change to internal/expand/engine.go:33: the existing body is renamed
// buildTreeSQL (its depth clamp, visited map and page loop stay as they are) and answers every root
// the GPU does not:
//
//	func (e *Engine) BuildTree(ctx context.Context, subject relationtuple.Subject, restDepth int) (*Tree, error) {
//		if t, ok, err := e.buildTreeGPU(ctx, subject, restDepth); ok {
//			return t, err
//		}
//		return e.buildTreeSQL(ctx, subject, restDepth)
//	}
//
// The recursion inside buildTreeSQL keeps calling e.BuildTree for children, so only top-level calls
// (the handlers, internal/expand/handler.go:84,98) should reach the GPU: buildTreeSQL's recursive call
// is renamed too, to e.buildTreeSQL.
func (e *Engine) buildTreeGPU(ctx context.Context, subject relationtuple.Subject, restDepth int) (*Tree, bool, error) {
	p, ok := e.d.(GPUProvider)
	if !ok {
		return nil, false, nil
	}
	b := p.GPUExpandBatcher()
	if b == nil {
		return nil, false, nil
	}
	nodes, err := b.Expand(ctx, subject, restDepth)
	switch {
	case err == nil:
		return TreeFromNodes(nodes), true, nil
	case errors.Is(err, gpu.ErrNotFound):
		// the root's namespace is unknown, or a page below it names an unknown namespace: the SQL path
		// returns the error the reference returns.  For the root that is the persister's namespace
		// lookup (whereQuery, internal/persistence/sql/relationtuples.go:179-185), made here directly.
		if us, isSet := subject.(*relationtuple.SubjectSet); isSet && us.Namespace != "" {
			nm, err := e.d.Config().NamespaceManager()
			if err != nil {
				return nil, true, err
			}
			if _, err := nm.GetNamespaceByName(ctx, us.Namespace); err != nil {
				return nil, true, err // herodot.ErrNotFound: 404 (internal/expand/handler_test.go:48-59)
			}
		}
		return nil, false, nil
	case errors.Is(err, context.Canceled), errors.Is(err, context.DeadlineExceeded):
		return nil, true, err
	default: // ErrUndecided, ErrBatchFailed, ErrClosed: the reference engine answers
		return nil, false, nil
	}
}

// TreeFromNodes builds the *Tree of one root from its pre-order nodes (nil for a nil tree), without
// recursion: a tree is as deep as its max-depth allows.
func TreeFromNodes(nodes []gpu.Node) *Tree {
	if len(nodes) == 0 {
		return nil
	}
	type open struct {
		t    *Tree
		left int
	}
	var stack []open
	var root *Tree
	for _, n := range nodes {
		t := &Tree{Type: Union, Subject: n.Subject}
		if n.Leaf {
			t.Type = Leaf
		}
		if len(stack) == 0 {
			root = t
		} else {
			top := &stack[len(stack)-1]
			top.t.Children = append(top.t.Children, t)
			top.left--
		}
		if !n.Leaf && n.Children > 0 {
			t.Children = make([]*Tree, 0, n.Children)
			stack = append(stack, open{t, n.Children})
		}
		for len(stack) > 0 && stack[len(stack)-1].left == 0 {
			stack = stack[:len(stack)-1]
		}
	}
	return root
}
