//go:build keto_gpu
// +build keto_gpu

package gpu

import (
	"context"
	"errors"
	"fmt"
	"os"
	"strconv"
	"sync"
	"time"

	"github.com/ory/keto/internal/relationtuple"
)

var (
	// ErrClosed: the batcher was closed; the caller answers on the SQL engine.
	ErrClosed = errors.New("gpu: batcher closed")
	// ErrBatchFailed wraps the error of a whole batch (no device, snapshot gone): every request of
	// the batch goes to the SQL engine.
	ErrBatchFailed = errors.New("gpu: batch failed")
)

// coalescer gathers concurrent requests (one goroutine per gRPC / REST request,
// internal/check/handler.go:108,154,174, internal/expand/handler.go:84,98) into batches: a batch is
// flushed when maxBatch requests are queued or maxWait after its first request.  Close answers every
// request still queued through drain, and later calls get ErrClosed without queueing.
type coalescer struct {
	maxBatch int
	maxWait  time.Duration
	queue    chan *pending
	stop     chan struct{}
	done     chan struct{}
	closeMu  sync.RWMutex // held shared while enqueueing, exclusively by Close
	closed   bool
	flush    func([]*pending) // answers every request of a batch
	drain    func([]*pending) // answers the requests left at Close
}

type pending struct {
	ctx  context.Context
	req  interface{}
	done chan result
}

type result struct {
	val interface{}
	err error
}

func newCoalescer(maxBatch int, maxWait time.Duration, flush, drain func([]*pending)) *coalescer {
	c := &coalescer{maxBatch: maxBatch, maxWait: maxWait, queue: make(chan *pending, maxBatch),
		stop: make(chan struct{}), done: make(chan struct{}), flush: flush, drain: drain}
	go c.loop()
	return c
}

// submit queues one request and waits for its answer (or ctx).  After Close it returns ErrClosed.
func (c *coalescer) submit(ctx context.Context, req interface{}) (interface{}, error) {
	p := &pending{ctx: ctx, req: req, done: make(chan result, 1)}
	c.closeMu.RLock()
	if c.closed {
		c.closeMu.RUnlock()
		return nil, ErrClosed
	}
	select {
	case c.queue <- p: // the loop runs until Close, which waits for this lock: it will be read
	case <-ctx.Done():
		c.closeMu.RUnlock()
		return nil, ctx.Err()
	}
	c.closeMu.RUnlock()
	select {
	case res := <-p.done:
		return res.val, res.err
	case <-ctx.Done():
		return nil, ctx.Err()
	}
}

// close stops the loop after it has answered (drain) every queued request.
func (c *coalescer) close() {
	c.closeMu.Lock()
	if c.closed {
		c.closeMu.Unlock()
		<-c.done
		return
	}
	c.closed = true
	close(c.stop)
	c.closeMu.Unlock()
	<-c.done
}

func (c *coalescer) loop() {
	defer close(c.done)
	for {
		var first *pending
		select {
		case first = <-c.queue:
		case <-c.stop:
			// closed: nothing can be enqueued any more (Close held the lock); answer what is left
			var left []*pending
			for {
				select {
				case p := <-c.queue:
					left = append(left, p)
				default:
					if len(left) > 0 {
						c.drain(left)
					}
					return
				}
			}
		}
		batch := []*pending{first}
		timer := time.NewTimer(c.maxWait)
	fill:
		for len(batch) < c.maxBatch {
			select {
			case p := <-c.queue:
				batch = append(batch, p)
			case <-timer.C:
				break fill
			}
		}
		timer.Stop()
		c.flush(batch)
	}
}

// Fallback answers one check on the reference engine (the SQL path of
// check.(*Engine).SubjectIsAllowed, internal/check/engine.go:116-123): used for requests the GPU
// leaves KETO_CHECK_UNDECIDED, when a batch fails as a whole (no device, snapshot gone) and for the
// requests still queued when the batcher closes.
type Fallback func(ctx context.Context, r *relationtuple.InternalRelationTuple, restDepth int) (bool, error)

// replicas deals batches to the engines of a set: one snapshot replica per GPU (BuildReplicas), or
// one Partition over all of them (a graph past one GPU's memory).  A batch goes to an engine with
// fewer than InflightFromEnv batches in flight, so the GPUs of a node work on consecutive batches at
// once, each overlapping two of them, and the dealing follows their load; when every engine is full
// the flush loop waits (back-pressure).
type replicas struct {
	mu  sync.RWMutex // held shared by a running batch (from dealing to its end), exclusively by swap
	cur *engineSet
}

type engineSet struct {
	snaps []Engine
	idle  chan int // one token per batch an engine may take more: InflightFromEnv tokens per engine
}

// InflightFromEnv is the number of batches the batchers keep in flight per engine,
// KETO_GPU_INFLIGHT (default 2, at most 8): the library overlaps one packed batch's upload and
// resolution with another's check on the same device (keto_check_batch_packed keeps that many
// in flight, KETO_PACKED_SLOTS), so at the 65,536-request flush the GPU is not idle between batches.
// A Partition serializes its own batches.
func InflightFromEnv() int {
	if v, err := strconv.Atoi(os.Getenv("KETO_GPU_INFLIGHT")); err == nil && v > 0 {
		if v > 8 {
			v = 8
		}
		return v
	}
	return 2
}

func newEngineSet(snaps []Engine) *engineSet {
	per := InflightFromEnv()
	s := &engineSet{snaps: snaps, idle: make(chan int, per*len(snaps))}
	for j := 0; j < per; j++ { // engine k's tokens interleaved, so batches spread over the GPUs first
		for k := range snaps {
			s.idle <- k
		}
	}
	return s
}

func newReplicas(snaps []Engine) *replicas { return &replicas{cur: newEngineSet(snaps)} }

// run takes an idle engine of the current set, then runs fn on it in its own goroutine.  The shared
// lock is held from here until fn returns (another goroutine may release it), so a swap waits for
// the batches in flight and no batch sees two sets.
func (r *replicas) run(fn func(s Engine)) {
	r.mu.RLock()
	set := r.cur
	k := <-set.idle
	go func() {
		defer r.mu.RUnlock()
		defer func() { set.idle <- k }()
		fn(set.snaps[k])
	}()
}

// swap installs a new engine set (a rebuild, which may also change the placement: replicas <-> a
// partition); it returns the old one once no batch uses it.
func (r *replicas) swap(snaps []Engine) []Engine {
	r.mu.Lock()
	defer r.mu.Unlock()
	old := r.cur.snaps
	r.cur = newEngineSet(snaps)
	return old
}

// Batcher coalesces concurrent SubjectIsAllowed calls into keto_check_batch calls (defaults: 65,536
// requests or 200 µs per batch), dealt over the replica set's GPUs.
type Batcher struct {
	rep       *replicas
	GlobalMax func() int // config.ReadAPIMaxDepth (internal/driver/config/provider.go:143-145)
	Fallback  Fallback
	c         *coalescer
}

type checkReq struct {
	r     *relationtuple.InternalRelationTuple
	depth int
}

// CheckFlushFromEnv is the check batcher's flush size, KETO_GPU_CHECK_BATCH requests (default 65,536,
// at most 2^24).  Larger batches trade latency for throughput: on the 1B-tuple graph a packed batch
// of 65,536 requests takes 0.34 ms (~190 M checks/s per GPU), one of 1M 1.66 ms (~600 M checks/s),
// profiles/r05as_packed_*.log.
func CheckFlushFromEnv() int {
	if v, err := strconv.Atoi(os.Getenv("KETO_GPU_CHECK_BATCH")); err == nil && v > 0 {
		if v > 1<<24 {
			v = 1 << 24
		}
		return v
	}
	return 1 << 16
}

// NewBatcher starts the flush loop over the engines (one snapshot per GPU, or a partition).
func NewBatcher(snaps []Engine, globalMax func() int, fb Fallback) *Batcher {
	b := &Batcher{rep: newReplicas(snaps), GlobalMax: globalMax, Fallback: fb}
	b.c = newCoalescer(CheckFlushFromEnv(), 200*time.Microsecond, b.flush, b.fallbackAll)
	return b
}

// Swap installs a new engine set (a rebuild); it returns the old one once no batch uses it.
func (b *Batcher) Swap(snaps []Engine) []Engine { return b.rep.swap(snaps) }

// Close stops the loop; queued requests are answered by the fallback, later ones too.
func (b *Batcher) Close() { b.c.close() }

// Check = SubjectIsAllowed through the GPU batch path.
func (b *Batcher) Check(ctx context.Context, r *relationtuple.InternalRelationTuple, restDepth int) (bool, error) {
	v, err := b.c.submit(ctx, checkReq{r, restDepth})
	if errors.Is(err, ErrClosed) {
		return b.Fallback(ctx, r, restDepth)
	}
	if err != nil {
		return false, err
	}
	return v.(bool), nil
}

func (b *Batcher) fallbackAll(ps []*pending) {
	for _, p := range ps {
		go func(p *pending) {
			q := p.req.(checkReq)
			a, e := b.Fallback(p.ctx, q.r, q.depth)
			p.done <- result{a, e}
		}(p)
	}
}

func (b *Batcher) flush(batch []*pending) {
	reqs := make([]*relationtuple.InternalRelationTuple, len(batch))
	depths := make([]int, len(batch))
	for i, p := range batch {
		q := p.req.(checkReq)
		reqs[i], depths[i] = q.r, q.depth
	}
	globalMax := b.GlobalMax()
	b.rep.run(func(s Engine) {
		allowed, status, err := s.CheckBatch(reqs, depths, globalMax)
		if err != nil {
			b.fallbackAll(batch)
			return
		}
		var undecided []*pending
		for i, p := range batch {
			if status[i] == StatusUndecided {
				undecided = append(undecided, p) // this one request goes to the reference engine
				continue
			}
			// StatusUnknownNamespace is allowed = false, nil like the reference (engine.go:98-100)
			p.done <- result{allowed[i], nil}
		}
		b.fallbackAll(undecided)
	})
}

// ExpandBatcher coalesces concurrent BuildTree calls into keto_expand_batch calls (defaults: 4,096
// roots or 200 µs per batch), dealt over the replica set's GPUs.  Trees come back as pre-order Nodes;
// errors per root are ErrNotFound, ErrUndecided, a wrapped ErrBatchFailed or ErrClosed (the last
// three: answer on the SQL engine).
type ExpandBatcher struct {
	rep       *replicas
	GlobalMax func() int
	c         *coalescer
}

type expandReq struct {
	sub   relationtuple.Subject
	depth int
}

// NewExpandBatcher starts the flush loop over the engines (one snapshot per GPU, or a partition).
func NewExpandBatcher(snaps []Engine, globalMax func() int) *ExpandBatcher {
	b := &ExpandBatcher{rep: newReplicas(snaps), GlobalMax: globalMax}
	b.c = newCoalescer(1<<12, 200*time.Microsecond, b.flush, func(ps []*pending) {
		for _, p := range ps {
			p.done <- result{nil, ErrClosed}
		}
	})
	return b
}

// Swap installs a new engine set; it returns the old one once no batch uses it.
func (b *ExpandBatcher) Swap(snaps []Engine) []Engine { return b.rep.swap(snaps) }

// Close stops the loop; queued and later requests get ErrClosed.
func (b *ExpandBatcher) Close() { b.c.close() }

// Expand = BuildTree through the GPU batch path: root's nodes in pre-order (nil: a nil tree).
func (b *ExpandBatcher) Expand(ctx context.Context, sub relationtuple.Subject, restDepth int) ([]Node, error) {
	v, err := b.c.submit(ctx, expandReq{sub, restDepth})
	if err != nil {
		return nil, err
	}
	nodes, _ := v.([]Node)
	return nodes, nil
}

func (b *ExpandBatcher) flush(batch []*pending) {
	subs := make([]relationtuple.Subject, len(batch))
	depths := make([]int, len(batch))
	for i, p := range batch {
		q := p.req.(expandReq)
		subs[i], depths[i] = q.sub, q.depth
	}
	globalMax := b.GlobalMax()
	b.rep.run(func(s Engine) {
		trees, errs, err := s.ExpandBatch(subs, depths, globalMax)
		for i, p := range batch {
			switch {
			case err != nil:
				p.done <- result{nil, fmt.Errorf("%w: %v", ErrBatchFailed, err)}
			case errs[i] != nil:
				p.done <- result{nil, errs[i]}
			default:
				p.done <- result{trees[i], nil}
			}
		}
	})
}
