//go:build keto_gpu
// +build keto_gpu

package gpu

import (
	"context"
	"sync"
	"time"

	"github.com/ory/keto/internal/relationtuple"
)

// Fallback answers one check on the reference engine (the SQL path of
// check.(*Engine).SubjectIsAllowed, internal/check/engine.go:116-123): used for requests the GPU
// leaves KETO_CHECK_UNDECIDED and when a batch fails as a whole (no device, snapshot gone).
type Fallback func(ctx context.Context, r *relationtuple.InternalRelationTuple, restDepth int) (bool, error)

// Batcher coalesces concurrent SubjectIsAllowed calls (one goroutine per gRPC / REST request,
// internal/check/handler.go:108,154,174) into keto_check_batch calls: a batch is flushed when
// MaxBatch requests are queued or MaxWait after its first request, whichever comes first.
type Batcher struct {
	mu        sync.RWMutex
	snap      *Snapshot
	GlobalMax func() int // config.ReadAPIMaxDepth (internal/driver/config/provider.go:143-145)
	Fallback  Fallback
	MaxBatch  int
	MaxWait   time.Duration
	queue     chan *pending
	stop      chan struct{}
}

type pending struct {
	ctx   context.Context
	r     *relationtuple.InternalRelationTuple
	depth int
	done  chan result
}

type result struct {
	allowed bool
	err     error
}

// NewBatcher starts the flush loop.  Defaults: 65,536 requests or 200 µs per batch.
func NewBatcher(s *Snapshot, globalMax func() int, fb Fallback) *Batcher {
	b := &Batcher{snap: s, GlobalMax: globalMax, Fallback: fb, MaxBatch: 1 << 16, MaxWait: 200 * time.Microsecond,
		queue: make(chan *pending, 1<<16), stop: make(chan struct{})}
	go b.loop()
	return b
}

// Swap installs a new snapshot version (Apply / rebuild); batches already running keep theirs.
func (b *Batcher) Swap(s *Snapshot) *Snapshot {
	b.mu.Lock()
	defer b.mu.Unlock()
	old := b.snap
	b.snap = s
	return old
}

// Close stops the loop; queued requests are answered by the fallback.
func (b *Batcher) Close() { close(b.stop) }

// Check = SubjectIsAllowed through the GPU batch path.
func (b *Batcher) Check(ctx context.Context, r *relationtuple.InternalRelationTuple, restDepth int) (bool, error) {
	p := &pending{ctx: ctx, r: r, depth: restDepth, done: make(chan result, 1)}
	select {
	case b.queue <- p:
	case <-ctx.Done():
		return false, ctx.Err()
	case <-b.stop:
		return b.Fallback(ctx, r, restDepth)
	}
	select {
	case res := <-p.done:
		return res.allowed, res.err
	case <-ctx.Done():
		return false, ctx.Err()
	}
}

func (b *Batcher) loop() {
	for {
		var first *pending
		select {
		case first = <-b.queue:
		case <-b.stop:
			return
		}
		batch := []*pending{first}
		timer := time.NewTimer(b.MaxWait)
	fill:
		for len(batch) < b.MaxBatch {
			select {
			case p := <-b.queue:
				batch = append(batch, p)
			case <-timer.C:
				break fill
			}
		}
		timer.Stop()
		b.flush(batch)
	}
}

func (b *Batcher) flush(batch []*pending) {
	reqs := make([]*relationtuple.InternalRelationTuple, len(batch))
	depths := make([]int, len(batch))
	for i, p := range batch {
		reqs[i], depths[i] = p.r, p.depth
	}
	b.mu.RLock()
	allowed, status, err := b.snap.CheckBatch(reqs, depths, b.GlobalMax())
	b.mu.RUnlock()
	for i, p := range batch {
		if err != nil || status[i] == StatusUndecided {
			// one request (or, on a batch error, each) goes to the reference engine on its own goroutine
			go func(p *pending) {
				a, e := b.Fallback(p.ctx, p.r, p.depth)
				p.done <- result{a, e}
			}(p)
			continue
		}
		// StatusUnknownNamespace is allowed = false, nil like the reference (engine.go:98-100)
		p.done <- result{allowed[i], nil}
	}
}
