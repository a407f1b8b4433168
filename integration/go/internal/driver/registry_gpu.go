//go:build keto_gpu
// +build keto_gpu

package driver

import (
	"context"
	"errors"
	"os"
	"strconv"
	"strings"
	"sync"

	"github.com/ory/keto/internal/gpu"
	"github.com/ory/keto/internal/persistence"
	"github.com/ory/keto/internal/relationtuple"
)

// The registry side of the GPU path.  After Init (internal/driver/registry_default.go:241-262) the
// server calls EnableGPU once, the one change to cmd/server/serve.go:45-55:
//
//	reg, err := driver.NewDefaultRegistry(cmd.Context(), cmd.Flags(), false)
//	...
//	if err := driver.EnableGPU(cmd.Context(), reg, driver.GPUDevicesFromEnv()); err != nil {
//		return err
//	}
//	return reg.ServeAllSQA(cmd)
//
// The server stays one process (internal/driver/daemon.go:62-69) and drives every GPU of the node
// itself: EnableGPU builds the snapshot from one full scan of the table (sorted once, host-only) and
// places it (gpu.Place): one replica per device while the replicated arena fits each of them (and the
// 288 GiB arena cap), else one edge-partitioned snapshot over all of them (gpu.Partition: shared-rows
// parts, one in-process communicator rank per part, several parts per device when a part would pass
// the cap), so a table of any size is served from this one process, as the
// reference serves it.  It starts the check and expand batchers, which deal each batch to an engine
// with no batch in flight, and wraps the persister so that every committed write transaction is
// applied to every replica or part before the write returns.  The engines find the batchers through GPUCheckBatcher /
// GPUExpandBatcher (internal/check/engine_gpu.go, internal/expand/engine_gpu.go) and answer on SQL
// whenever those return nil: no GPU, or a snapshot that is behind the table while it is rebuilt.

// GPUDevicesFromEnv is the HIP devices of the GPU path: KETO_GPU_DEVICES, a comma-separated list
// ("0,1,2,3,4,5,6,7"), or the single KETO_GPU_DEVICE; unset, empty or negative: off (nil).
func GPUDevicesFromEnv() []int {
	v := os.Getenv("KETO_GPU_DEVICES")
	if v == "" {
		v = os.Getenv("KETO_GPU_DEVICE")
	}
	var out []int
	for _, f := range strings.Split(v, ",") {
		d, err := strconv.Atoi(strings.TrimSpace(f))
		if err != nil || d < 0 {
			continue
		}
		out = append(out, d)
	}
	return out
}

// gpuRowSource is the persister's full scan (internal/persistence/sql/snapshot_gpu.go).
type gpuRowSource interface {
	SnapshotRows(ctx context.Context) ([]gpu.Row, error)
}

// GPUPlacementFromEnv is how the snapshot is placed on the devices (KETO_GPU_PLACEMENT): "auto" (the
// default: replicas while the replicated arena fits every device, else a partition), "replicate" or
// "partition".
func GPUPlacementFromEnv() string { return os.Getenv("KETO_GPU_PLACEMENT") }

// GPUSnapshotFileFromEnv is where the GPU path keeps its persisted snapshot (KETO_GPU_SNAPSHOT_FILE;
// empty: none).  A server that starts with a file saved under the table's current fingerprint loads
// it (gpu.Load: about 15 s for 1B tuples) instead of sorting the table; every build writes the file
// again.  The fingerprint is a hash of the scanned rows' contents (gpu.Fingerprint), so the scan
// still runs; what the file saves is the sort, the interning and the layout.
func GPUSnapshotFileFromEnv() string { return os.Getenv("KETO_GPU_SNAPSHOT_FILE") }

type gpuState struct {
	r       *RegistryDefault
	devices []int
	check   *gpu.Batcher
	expand  *gpu.ExpandBatcher

	mu      sync.RWMutex
	engines []gpu.Engine // one replica per device, or one partition over them, at one version
	stale   bool         // the engines are behind the table: SQL answers until the rebuild lands

	wmu        sync.Mutex // one write transaction (SQL commit + Apply) at a time; the rebuild's scan holds it too
	rebuilding bool
	pending    [][2][]gpu.Row // writes committed after the rebuild's scan, applied to the new snapshot
	rescan     bool           // a write during the rebuild cannot be replayed: scan the table again
}

// one state per registry (RegistryDefault's fields are in registry_default.go)
var gpuStates sync.Map // *RegistryDefault -> *gpuState

func gpuOf(r *RegistryDefault) *gpuState {
	if v, ok := gpuStates.Load(r); ok {
		return v.(*gpuState)
	}
	return nil
}

// EnableGPU loads the snapshot onto the HIP devices of `devices` (none: leave the registry on SQL).
func EnableGPU(ctx context.Context, reg Registry, devices []int) error {
	r, ok := reg.(*RegistryDefault)
	if !ok || len(devices) == 0 {
		return nil
	}
	if err := r.Init(ctx); err != nil {
		return err
	}
	st := &gpuState{r: r, devices: append([]int(nil), devices...)}
	engines, err := st.build(ctx)
	if err != nil {
		return err
	}
	st.engines = engines
	globalMax := func() int { return r.Config().ReadAPIMaxDepth() }
	st.check = gpu.NewBatcher(engines, globalMax, r.PermissionEngine().Fallback())
	st.expand = gpu.NewExpandBatcher(engines, globalMax)
	r.p = &gpuPersister{Persister: r.p, g: st}
	gpuStates.Store(r, st)
	return nil
}

// GPUCheckBatcher implements check.GPUProvider (nil: answer on SQL).
func (r *RegistryDefault) GPUCheckBatcher() *gpu.Batcher {
	st := gpuOf(r)
	if st == nil {
		return nil
	}
	st.mu.RLock()
	defer st.mu.RUnlock()
	if st.stale {
		return nil
	}
	return st.check
}

// GPUExpandBatcher implements expand.GPUProvider (nil: answer on SQL).
func (r *RegistryDefault) GPUExpandBatcher() *gpu.ExpandBatcher {
	st := gpuOf(r)
	if st == nil {
		return nil
	}
	st.mu.RLock()
	defer st.mu.RUnlock()
	if st.stale {
		return nil
	}
	return st.expand
}

// build scans the table (caller holds wmu when it must be consistent with writes) and places the
// snapshot: from the persisted file when it was saved from these exact rows, else built from them.
func (g *gpuState) build(ctx context.Context) ([]gpu.Engine, error) {
	src, ok := g.r.p.(gpuRowSource) // EnableGPU builds before it wraps the persister
	if !ok {
		return nil, errors.New("gpu: the persister has no full-scan source")
	}
	rows, err := src.SnapshotRows(ctx)
	if err != nil {
		return nil, err
	}
	if path := GPUSnapshotFileFromEnv(); path != "" {
		if es, ok := g.loadFile(path, gpu.Fingerprint(rows)); ok {
			return es, nil
		}
	}
	return g.buildFrom(ctx, rows)
}

// loadFile: the persisted snapshot at path, if it was saved under fingerprint fp, loaded host-only
// and placed on the devices; ok is false (and nothing is kept) otherwise.
func (g *gpuState) loadFile(path string, fp uint64) ([]gpu.Engine, bool) {
	base, tag, err := gpu.Load(path, -1)
	if err != nil {
		return nil, false
	}
	if tag != fp {
		base.Close()
		return nil, false
	}
	es, err := gpu.Place(base, g.devices, GPUPlacementFromEnv())
	if err != nil {
		return nil, false
	}
	return es, true
}

// buildFrom sorts the rows once, host-only, saves the persisted file (best effort: without it the
// next start sorts again) and places the snapshot on the devices.
func (g *gpuState) buildFrom(ctx context.Context, rows []gpu.Row) ([]gpu.Engine, error) {
	nm, err := g.r.Config().NamespaceManager()
	if err != nil {
		return nil, err
	}
	nss, err := nm.Namespaces(ctx) // config order: the builder maps names to ids with it
	if err != nil {
		return nil, err
	}
	base, err := gpu.Build(nss, rows, -1)
	if err != nil {
		return nil, err
	}
	if path := GPUSnapshotFileFromEnv(); path != "" {
		_ = base.Save(path, gpu.Fingerprint(rows))
	}
	// a rebuild places the new set while the outgoing one is still on the devices: credit its memory
	g.mu.RLock()
	resident := gpu.FootprintOf(g.engines)
	g.mu.RUnlock()
	return gpu.PlaceWith(base, g.devices, GPUPlacementFromEnv(), resident)
}

// applyLocked runs after a write committed, with wmu held: every replica follows the table one
// transaction at a time, or the set goes stale and is rebuilt.
func (g *gpuState) applyLocked(ctx context.Context, ins, del []*relationtuple.InternalRelationTuple) {
	nm, err := g.r.Config().NamespaceManager()
	var iRows, dRows []gpu.Row
	if err == nil {
		iRows, err = gpu.RowsOf(ctx, nm, ins)
	}
	if err == nil {
		dRows, err = gpu.RowsOf(ctx, nm, del)
	}
	if g.rebuilding {
		if err != nil { // cannot replay this write: the rebuild scans the table again
			g.rescan = true
			return
		}
		g.pending = append(g.pending, [2][]gpu.Row{iRows, dRows})
		return
	}
	g.mu.RLock()
	engines, stale := g.engines, g.stale
	g.mu.RUnlock()
	if stale { // an earlier rebuild failed: the replicas are behind, try again
		g.startRebuildLocked()
		return
	}
	if err == nil {
		err = gpu.ApplyEngines(engines, iRows, dRows)
	}
	if err != nil { // gpu.ErrRebuild (or a failed write to a device): serve SQL until rebuilt
		g.startRebuildLocked()
	}
}

// startRebuildLocked (wmu held): mark the snapshot stale and rebuild it in the background.
func (g *gpuState) startRebuildLocked() {
	g.mu.Lock()
	g.stale = true
	g.mu.Unlock()
	if g.rebuilding {
		return
	}
	g.rebuilding = true
	go g.rebuild()
}

// rebuild: scan the table under wmu (so the scan sees every committed write and none is half
// applied), build without it, replay the writes that committed meanwhile, swap the new snapshot into
// the batchers and serve from the GPU again.
func (g *gpuState) rebuild() {
	ctx := context.Background()
	for {
		g.wmu.Lock()
		g.pending = nil
		g.rescan = false
		var src gpuRowSource
		if w, ok := g.r.p.(*gpuPersister); ok {
			src, _ = w.Persister.(gpuRowSource)
		}
		var rows []gpu.Row
		var err error
		if src == nil {
			err = errors.New("gpu: the persister has no full-scan source")
		} else {
			rows, err = src.SnapshotRows(ctx)
		}
		g.wmu.Unlock()
		var engines []gpu.Engine
		if err == nil {
			engines, err = g.buildFrom(ctx, rows)
		}
		rows = nil
		g.wmu.Lock()
		if err != nil || g.rescan {
			g.wmu.Unlock()
			gpu.CloseEngines(engines)
			if err != nil { // stay stale (SQL answers); a later write retries the rebuild
				g.wmu.Lock()
				g.rebuilding = false
				g.wmu.Unlock()
				return
			}
			continue
		}
		replayed := true
		for _, w := range g.pending {
			if gpu.ApplyEngines(engines, w[0], w[1]) != nil {
				replayed = false
				break
			}
		}
		if !replayed { // a replayed write needs a rebuild itself: scan again
			g.wmu.Unlock()
			gpu.CloseEngines(engines)
			continue
		}
		old := g.check.Swap(engines) // waits for batches running on the old versions
		g.expand.Swap(engines)
		g.mu.Lock()
		g.engines = engines
		g.stale = false
		g.mu.Unlock()
		g.pending = nil
		g.rebuilding = false
		g.wmu.Unlock()
		gpu.CloseEngines(old)
		return
	}
}

// gpuPersister wraps the SQL persister: every committed write reaches the snapshot before the call
// returns, in commit order (relationtuple.Manager, internal/relationtuple/definitions.go:28-34;
// TransactRelationTuples = inserts, then deletes, internal/persistence/sql/relationtuples.go:290-297).
type gpuPersister struct {
	persistence.Persister
	g *gpuState
}

func (p *gpuPersister) WriteRelationTuples(ctx context.Context, rs ...*relationtuple.InternalRelationTuple) error {
	return p.TransactRelationTuples(ctx, rs, nil)
}

func (p *gpuPersister) DeleteRelationTuples(ctx context.Context, rs ...*relationtuple.InternalRelationTuple) error {
	return p.TransactRelationTuples(ctx, nil, rs)
}

func (p *gpuPersister) TransactRelationTuples(ctx context.Context, ins, del []*relationtuple.InternalRelationTuple) error {
	p.g.wmu.Lock()
	defer p.g.wmu.Unlock()
	if err := p.Persister.TransactRelationTuples(ctx, ins, del); err != nil {
		return err // rolled back: the snapshot stays as it is
	}
	p.g.applyLocked(ctx, ins, del)
	return nil
}

// DeleteAllRelationTuples deletes by query (whereQuery, relationtuples.go:178-198): the rows are not
// named, so the snapshot is rebuilt from the table.
func (p *gpuPersister) DeleteAllRelationTuples(ctx context.Context, q *relationtuple.RelationQuery) error {
	p.g.wmu.Lock()
	defer p.g.wmu.Unlock()
	if err := p.Persister.DeleteAllRelationTuples(ctx, q); err != nil {
		return err
	}
	if p.g.rebuilding {
		p.g.rescan = true
		return nil
	}
	p.g.startRebuildLocked()
	return nil
}
