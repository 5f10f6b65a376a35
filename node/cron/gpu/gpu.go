// Package gpu evaluates cronsun's schedules in batch on an MI355X through
// libcronsun_gpu.so (include/cronsun_gpu.h).  It sits next to the
// reference's node/cron package and keeps that package's API: cron.Parse,
// Schedule.Next, *cron.SpecSchedule, cron.ConstantDelaySchedule and the
// cronsun.Job / JobRule / Group model.  Only those two Schedule types are
// accepted; any other Schedule stays on the CPU path (Schedule.Next).
//
// The boundary it binds is the reference's own: Schedule.Next
// (node/cron/cron.go:36-40), cron.Parse (node/cron/parser.go:181-183), the
// per-node Job.Cmds filter (job.go:591-614, driven by node/node.go:121-158),
// Cmd.lockTtl (job.go:194-233) and Cron.run's wake loop (cron.go:210-275).
//
// cgo rules kept: Go memory passed to C never holds Go pointers (structs that
// point at buffers, and those buffers, are C.malloc'ed), and every wrapper that
// passes a handle keeps its owner alive across the call (runtime.KeepAlive;
// Specs and Dispatcher hold their Engine).  C memory is viewed as Go slices
// through array-pointer conversions (int64sAt / bytesAt), not unsafe.Slice, so
// the package builds with the Go releases the reference's CI pins (1.7 / 1.8).
//
// Go is not installed in the image this package was written in, so it is not
// compiled there; tests/native/abi_c.c runs the same call sequence against the
// header in C (gcc -std=c11) and, on an MI355X, against the library.
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../cronsun_amd -lcronsun_gpu -Wl,-rpath,${SRCDIR}/../../../cronsun_amd
#include <stdlib.h>
#include "cronsun_gpu.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"sync"
	"time"
	"unsafe"

	"github.com/shunfei/cronsun"
	"github.com/shunfei/cronsun/node/cron"
)

const zeroUnix = -62135596800 // time.Time{}.Unix()

// int64sAt / bytesAt view n elements of C memory at p as a Go slice (the
// array-pointer form works on every Go release; unsafe.Slice needs 1.17)
func int64sAt(p unsafe.Pointer, n int) []int64 { return (*[1 << 28]int64)(p)[:n:n] }
func bytesAt(p unsafe.Pointer, n int) []byte   { return (*[1 << 30]byte)(p)[:n:n] }

// Exclude modes of the rule -> node resolution.
const (
	ExcludeNone       = C.CG_EXCLUDE_NONE       // Job.Cmds / IsRunOn: ExcludeNodeIDs has no effect (job.go:598-602)
	ExcludeRule       = C.CG_EXCLUDE_RULE       // N_r \ E_r
	ExcludeCumulative = C.CG_EXCLUDE_CUMULATIVE // GetJobNodes (web/job.go:222-257)
)

// ErrUnsupported is returned for a Schedule that is neither
// *cron.SpecSchedule nor cron.ConstantDelaySchedule.
var ErrUnsupported = errors.New("gpu: unsupported Schedule type (keep Schedule.Next for it)")

func lastErr(rc C.int) error {
	return fmt.Errorf("cronsun_gpu %d: %s", int(rc), C.GoString(C.cg_last_error()))
}

// Engine is one MI355X: a cg_ctx (device, stream, HBM buffers).  Calls on an
// Engine are serialised by the library and block the calling OS thread.
// Engine owns one device context.  Its methods may be called from several
// goroutines: calls that set engine state and then use it (ExpandPerNode's
// node order) hold mu across both steps.
type Engine struct {
	ctx *C.cg_ctx
	mu  sync.Mutex
}

func NewEngine(device int) (*Engine, error) {
	var ctx *C.cg_ctx
	if rc := C.cg_init(C.int(device), &ctx); rc != 0 {
		return nil, lastErr(rc)
	}
	e := &Engine{ctx: ctx}
	runtime.SetFinalizer(e, func(e *Engine) { C.cg_destroy(e.ctx) })
	return e, nil
}

// Zone is a *time.Location for the engine.  Go does not expose a Location's
// TZif bytes, so callers pass the zoneinfo file (e.g. $ZONEINFO/<name>).
type Zone struct{ z *C.cg_zone }

func newZone(z *C.cg_zone) *Zone {
	zz := &Zone{z}
	runtime.SetFinalizer(zz, func(z *Zone) { C.cg_zone_free(z.z) })
	return zz
}

func LoadZone(tzif []byte) (*Zone, error) {
	if len(tzif) == 0 {
		return nil, errors.New("gpu: empty TZif data")
	}
	var z *C.cg_zone
	if rc := C.cg_zone_from_tzif((*C.uint8_t)(unsafe.Pointer(&tzif[0])), C.size_t(len(tzif)), &z); rc != 0 {
		return nil, lastErr(rc)
	}
	return newZone(z), nil
}

func UTC() (*Zone, error) {
	var z *C.cg_zone
	if rc := C.cg_zone_utc(&z); rc != 0 {
		return nil, lastErr(rc)
	}
	return newZone(z), nil
}

func FixedZone(offsetSec int) (*Zone, error) {
	var z *C.cg_zone
	if rc := C.cg_zone_fixed(C.int32_t(offsetSec), &z); rc != 0 {
		return nil, lastErr(rc)
	}
	return newZone(z), nil
}

// Specs is a rule set resident in HBM (32 B per rule).  It keeps its Engine
// reachable: cg_specs_free reads the engine's context, so the Engine's
// finalizer (cg_destroy) must not run first.
type Specs struct {
	s *C.cg_specs
	n int
	e *Engine
}

func (s *Specs) Len() int { return s.n }

// Upload packs the schedules (SpecSchedule masks, spec.go:7-9; the
// ConstantDelaySchedule delay, constantdelay.go:7-9) into HBM.
func (e *Engine) Upload(scheds []cron.Schedule) (*Specs, error) {
	cs := make([]C.cg_schedule, len(scheds)) // Go memory, passed only for the call
	for i, s := range scheds {
		switch v := s.(type) {
		case *cron.SpecSchedule:
			cs[i].kind = 0
			cs[i].second, cs[i].minute, cs[i].hour = C.uint64_t(v.Second), C.uint64_t(v.Minute), C.uint64_t(v.Hour)
			cs[i].dom, cs[i].month, cs[i].dow = C.uint64_t(v.Dom), C.uint64_t(v.Month), C.uint64_t(v.Dow)
		case cron.ConstantDelaySchedule:
			cs[i].kind = 1
			cs[i].delay_ns = C.int64_t(v.Delay)
		default:
			return nil, ErrUnsupported
		}
	}
	var p *C.cg_schedule
	if len(cs) > 0 {
		p = &cs[0]
	}
	var out *C.cg_specs
	if rc := C.cg_specs_upload_schedules(e.ctx, p, C.size_t(len(cs)), &out); rc != 0 {
		return nil, lastErr(rc)
	}
	sp := &Specs{out, len(scheds), e}
	runtime.SetFinalizer(sp, func(s *Specs) { C.cg_specs_free(s.s) })
	runtime.KeepAlive(cs)
	runtime.KeepAlive(e)
	return sp, nil
}

func unixOf(v C.int64_t, loc *time.Location) time.Time {
	if int64(v) == zeroUnix {
		return time.Time{}
	}
	return time.Unix(int64(v), 0).In(loc)
}

// NextBatch returns Schedule.Next(t[i]) for every rule i (spec.go:55-145,
// constantdelay.go:25-27); the zero time where Next returns it.
func (e *Engine) NextBatch(sp *Specs, z *Zone, t []time.Time) ([]time.Time, error) {
	if len(t) != sp.n {
		return nil, fmt.Errorf("gpu: NextBatch: %d times for %d rules", len(t), sp.n)
	}
	if sp.n == 0 {
		return nil, nil
	}
	in := make([]C.int64_t, len(t))
	out := make([]C.int64_t, len(t))
	for i := range t {
		in[i] = C.int64_t(t[i].Unix())
	}
	rc := C.cg_next_batch(e.ctx, sp.s, z.z, &in[0], &out[0])
	runtime.KeepAlive(e)
	runtime.KeepAlive(sp)
	runtime.KeepAlive(z)
	if rc != 0 {
		return nil, lastErr(rc)
	}
	res := make([]time.Time, len(t))
	for i, v := range out {
		res[i] = unixOf(v, t[i].Location())
	}
	return res, nil
}

// Expand runs the reference loop t = Next(t) until t > t1 for every rule and
// returns a rule-major CSR: rule i fires at times[offsets[i]:offsets[i+1]]
// (unix seconds, ascending) within (t0, t1].  The first call sizes the result
// (no times buffer: offsets and n_events only); the times are then copied out
// of the engine's last result, so the horizon is expanded once.
func (e *Engine) Expand(sp *Specs, z *Zone, t0, t1 time.Time) (offsets, times []int64, err error) {
	defer runtime.KeepAlive(e)
	defer runtime.KeepAlive(sp)
	defer runtime.KeepAlive(z)
	// The cg_csr struct holds a pointer, so it and the buffer it points to live
	// in C memory: cgo forbids passing Go memory that holds a Go pointer.
	csr := (*C.cg_csr)(C.calloc(1, C.size_t(unsafe.Sizeof(C.cg_csr{}))))
	defer C.free(unsafe.Pointer(csr))
	coff := (*C.int64_t)(C.malloc(C.size_t(sp.n+1) * 8))
	defer C.free(unsafe.Pointer(coff))
	csr.offsets = coff
	if rc := C.cg_expand(e.ctx, sp.s, z.z, C.int64_t(t0.Unix()), C.int64_t(t1.Unix()), csr); rc != 0 {
		return nil, nil, lastErr(rc)
	}
	offsets = make([]int64, sp.n+1)
	copy(offsets, int64sAt(unsafe.Pointer(coff), int(sp.n+1)))
	times = make([]int64, int64(csr.n_events))
	if len(times) > 0 {
		if rc := C.cg_result_copy_times(e.ctx, 0, csr.n_events, (*C.int64_t)(unsafe.Pointer(&times[0]))); rc != 0 {
			return nil, nil, lastErr(rc)
		}
	}
	return offsets, times, nil
}

// LockTtls returns Cmd.lockTtl() (job.go:194-233) for every rule at `now`:
// kinds = Job.Kind, avgMs = Job.AvgTime, lockTtl = conf.Config.LockTtl.
func (e *Engine) LockTtls(sp *Specs, z *Zone, now time.Time, kinds []int32, avgMs []int64, lockTtl int64) ([]int64, error) {
	if len(kinds) != sp.n || len(avgMs) != sp.n {
		return nil, fmt.Errorf("gpu: LockTtls: %d kinds, %d avg times for %d rules", len(kinds), len(avgMs), sp.n)
	}
	if sp.n == 0 {
		return nil, nil
	}
	t := make([]C.int64_t, sp.n)
	for i := range t {
		t[i] = C.int64_t(now.Unix())
	}
	out := make([]int64, sp.n)
	rc := C.cg_lock_ttl_batch(e.ctx, sp.s, z.z, &t[0], (*C.int32_t)(unsafe.Pointer(&kinds[0])),
		(*C.int64_t)(unsafe.Pointer(&avgMs[0])), C.int64_t(lockTtl), (*C.int64_t)(unsafe.Pointer(&out[0])))
	runtime.KeepAlive(e)
	runtime.KeepAlive(sp)
	runtime.KeepAlive(z)
	if rc != 0 {
		return nil, lastErr(rc)
	}
	return out, nil
}

// cStrings copies Go strings into C memory (Go memory holding Go pointers
// may not cross the boundary); free with freeStrings.
func cStrings(ss []string) **C.char {
	if len(ss) == 0 {
		return nil
	}
	arr := (*[1 << 28]*C.char)(C.malloc(C.size_t(len(ss)) * C.size_t(unsafe.Sizeof(uintptr(0)))))[:len(ss):len(ss)]
	for i, s := range ss {
		arr[i] = C.CString(s)
	}
	return &arr[0]
}

func freeStrings(p **C.char, n int) {
	if p == nil {
		return
	}
	arr := (*[1 << 28]*C.char)(unsafe.Pointer(p))[:n:n]
	for _, s := range arr {
		C.free(unsafe.Pointer(s))
	}
	C.free(unsafe.Pointer(p))
}

// Fire is one event of a node's schedule: the rule (index into the rules of
// BuildJobset's order) and its unix time.
type Fire struct {
	Rule int32
	Time int64
}

// Jobset is the interned job model (string IDs -> integers) of a set of jobs
// and groups: the input of every node's filter.
type Jobset struct {
	js     *C.cg_jobset
	scheds []cron.Schedule // JobRule.Schedule in rule order
}

// BuildJobset interns jobs (job.go:38-84) and groups (group.go:17-22).  Rules
// keep the jobs' order; a job's rules are contiguous.
func BuildJobset(jobs []*cronsun.Job, groups map[string]*cronsun.Group) (*Jobset, error) {
	var js *C.cg_jobset
	if rc := C.cg_jobset_new(&js); rc != 0 {
		return nil, lastErr(rc)
	}
	j := &Jobset{js: js}
	runtime.SetFinalizer(j, func(j *Jobset) { C.cg_jobset_free(j.js) })
	for gid, g := range groups {
		id := C.CString(gid)
		nids := cStrings(g.NodeIDs)
		rc := C.cg_jobset_add_group(js, id, nids, C.size_t(len(g.NodeIDs)))
		freeStrings(nids, len(g.NodeIDs))
		C.free(unsafe.Pointer(id))
		if rc != 0 {
			return nil, lastErr(rc)
		}
	}
	for _, job := range jobs {
		id := C.CString(job.ID)
		pause := C.int(0)
		if job.Pause {
			pause = 1
		}
		rc := C.cg_jobset_add_job(js, id, pause)
		C.free(unsafe.Pointer(id))
		if rc != 0 {
			return nil, lastErr(rc)
		}
		for _, r := range job.Rules {
			rid := C.CString(r.ID)
			g, n, x := cStrings(r.GroupIDs), cStrings(r.NodeIDs), cStrings(r.ExcludeNodeIDs)
			rc := C.cg_jobset_add_rule(js, rid, g, C.size_t(len(r.GroupIDs)), n, C.size_t(len(r.NodeIDs)),
				x, C.size_t(len(r.ExcludeNodeIDs)))
			freeStrings(g, len(r.GroupIDs))
			freeStrings(n, len(r.NodeIDs))
			freeStrings(x, len(r.ExcludeNodeIDs))
			C.free(unsafe.Pointer(rid))
			if rc != 0 {
				return nil, lastErr(rc)
			}
			j.scheds = append(j.scheds, r.Schedule)
		}
	}
	return j, nil
}

// Schedules returns JobRule.Schedule for every rule, in rule order (the input
// of Engine.Upload for ExpandPerNode).
func (j *Jobset) Schedules() []cron.Schedule { return j.scheds }

// ExpandPerNode is every node's loadJobs -> Job.Cmds filter
// (node/node.go:121-158, job.go:591-614) plus its Cron entries' Next loop over
// (t0, t1], for all nodes at once: node ID -> (rule, time) events, rule-major
// inside a node (rules ascending, times ascending within a rule), or with
// byTime set in the order a node's Cron keeps its entries (sort.Sort(byTime),
// cron.go:64-79: times ascending, equal times in rule order).
func (e *Engine) ExpandPerNode(sp *Specs, z *Zone, t0, t1 time.Time, j *Jobset, mode int, byTime bool) (map[string][]Fire, error) {
	defer runtime.KeepAlive(e)
	defer runtime.KeepAlive(sp)
	defer runtime.KeepAlive(z)
	defer runtime.KeepAlive(j)
	// cg_set_node_order is engine state: keep another goroutine's
	// ExpandPerNode from changing it between the two calls below
	e.mu.Lock()
	defer e.mu.Unlock()
	// cg_rules_in holds C pointers into the jobset (C memory): it may live in Go
	// memory.  cg_node_csr would hold a pointer to the node offsets, so it and
	// that buffer live in C memory (cgo's rule on Go pointers to Go pointers).
	var rin C.cg_rules_in
	if rc := C.cg_jobset_rules(j.js, &rin); rc != 0 {
		return nil, lastErr(rc)
	}
	if int(rin.n_rules) != sp.n {
		return nil, fmt.Errorf("gpu: ExpandPerNode: %d specs for %d rules", sp.n, int(rin.n_rules))
	}
	nn := int(rin.n_nodes)
	out := (*C.cg_node_csr)(C.calloc(1, C.size_t(unsafe.Sizeof(C.cg_node_csr{})))) // no event buffers: node offsets and n_events only
	defer C.free(unsafe.Pointer(out))
	coff := (*C.int64_t)(C.malloc(C.size_t(nn+1) * 8))
	defer C.free(unsafe.Pointer(coff))
	out.node_off = coff
	// byTime: the call itself leaves every node's list in (time, rule) order
	order := C.int(C.CG_NODE_ORDER_RULE)
	if byTime {
		order = C.int(C.CG_NODE_ORDER_TIME)
	}
	if rc := C.cg_set_node_order(e.ctx, order); rc != 0 {
		return nil, lastErr(rc)
	}
	if rc := C.cg_expand_per_node(e.ctx, sp.s, z.z, C.int64_t(t0.Unix()), C.int64_t(t1.Unix()), &rin,
		C.int(mode), out); rc != 0 {
		return nil, lastErr(rc)
	}
	nodeOff := make([]int64, nn+1)
	copy(nodeOff, int64sAt(unsafe.Pointer(coff), int(nn+1)))
	tm, rl := make([]int64, int64(out.n_events)), make([]int32, int64(out.n_events))
	if len(tm) > 0 {
		if rc := C.cg_node_result_copy(e.ctx, nil, (*C.int64_t)(unsafe.Pointer(&tm[0])),
			(*C.int32_t)(unsafe.Pointer(&rl[0])), out.n_events); rc != 0 {
			return nil, lastErr(rc)
		}
	}
	res := make(map[string][]Fire, int(rin.n_nodes))
	for n := 0; n < int(rin.n_nodes); n++ {
		lo, hi := nodeOff[n], nodeOff[n+1]
		if lo == hi {
			continue
		}
		fs := make([]Fire, hi-lo)
		for k := lo; k < hi; k++ {
			fs[k-lo] = Fire{Rule: rl[k], Time: tm[k]}
		}
		res[C.GoString(C.cg_jobset_node_id(j.js, C.int32_t(n)))] = fs
	}
	return res, nil
}

// Dispatcher is Cron.run's entry table in HBM: slot = index into the caller's
// Entry slice (c.indexes).  The run loop keeps its shape:
//
//	d, _ := eng.NewDispatcher(specs, zone, time.Now())
//	for {
//		eff := d.Effective()            // entries[0].Next after byTime
//		timer.Reset(eff.Sub(now))       // zero: sleep 10 years
//		select {
//		case now = <-timer.C:
//			slots, _ := d.Fire(now)
//			for _, slot := range slots { go c.runWithRecovery(c.entries[slot].Job) }
//		case e := <-c.add:  d.Set([]int64{slot(e)}, []cron.Schedule{e.Schedule}, time.Now())
//		case id := <-c.del: d.Remove([]int64{slot(id)})
//		}
//	}
type Dispatcher struct {
	d *C.cg_dispatcher
	e *Engine // cg_dispatcher_free locks the engine's context: keep it reachable
}

func (e *Engine) NewDispatcher(sp *Specs, z *Zone, now time.Time) (*Dispatcher, error) {
	var d *C.cg_dispatcher
	if rc := C.cg_dispatcher_new(e.ctx, sp.s, z.z, C.int64_t(now.Unix()), &d); rc != 0 {
		return nil, lastErr(rc)
	}
	dd := &Dispatcher{d, e}
	runtime.SetFinalizer(dd, func(d *Dispatcher) { C.cg_dispatcher_free(d.d) })
	runtime.KeepAlive(sp)
	runtime.KeepAlive(z)
	return dd, nil
}

// Effective is entries[0].Next after sort.Sort(byTime) (cron.go:220-230); the
// zero time when nothing can fire.
func (d *Dispatcher) Effective() (time.Time, error) {
	var eff C.int64_t
	rc := C.cg_dispatcher_effective(d.d, &eff)
	runtime.KeepAlive(d)
	if rc != 0 {
		return time.Time{}, lastErr(rc)
	}
	return unixOf(eff, time.Local), nil
}

// Fire is one wake at now (cron.go:234-244): the due slots, ascending.
func (d *Dispatcher) Fire(now time.Time) ([]int32, error) {
	defer runtime.KeepAlive(d)
	var n, eff C.int64_t
	if rc := C.cg_dispatcher_fire(d.d, C.int64_t(now.Unix()), &n, &eff); rc != 0 {
		return nil, lastErr(rc)
	}
	due := make([]int32, n)
	if n > 0 {
		if rc := C.cg_dispatcher_due(d.d, 0, n, (*C.int32_t)(unsafe.Pointer(&due[0]))); rc != 0 {
			return nil, lastErr(rc)
		}
	}
	return due, nil
}

// Set adds or replaces entries (cron.go:246-252): slot idx[k] gets scheds[k],
// Next = Schedule.Next(now), Prev = zero.
func (d *Dispatcher) Set(idx []int64, scheds []cron.Schedule, now time.Time) error {
	if len(idx) != len(scheds) {
		return fmt.Errorf("gpu: Set: %d slots for %d schedules", len(idx), len(scheds))
	}
	if len(idx) == 0 {
		return nil
	}
	cs := make([]C.cg_schedule, len(scheds))
	for i, s := range scheds {
		switch v := s.(type) {
		case *cron.SpecSchedule:
			cs[i].second, cs[i].minute, cs[i].hour = C.uint64_t(v.Second), C.uint64_t(v.Minute), C.uint64_t(v.Hour)
			cs[i].dom, cs[i].month, cs[i].dow = C.uint64_t(v.Dom), C.uint64_t(v.Month), C.uint64_t(v.Dow)
		case cron.ConstantDelaySchedule:
			cs[i].kind, cs[i].delay_ns = 1, C.int64_t(v.Delay)
		default:
			return ErrUnsupported
		}
	}
	rc := C.cg_dispatcher_set(d.d, (*C.int64_t)(unsafe.Pointer(&idx[0])), &cs[0], C.size_t(len(cs)),
		C.int64_t(now.Unix()))
	runtime.KeepAlive(d)
	if rc != 0 {
		return lastErr(rc)
	}
	return nil
}

// Remove empties slots (DelJob, cron.go:149-164, 254-262).
func (d *Dispatcher) Remove(idx []int64) error {
	if len(idx) == 0 {
		return nil
	}
	rc := C.cg_dispatcher_remove(d.d, (*C.int64_t)(unsafe.Pointer(&idx[0])), C.size_t(len(idx)))
	runtime.KeepAlive(d)
	if rc != 0 {
		return lastErr(rc)
	}
	return nil
}

// Comm is the library's RCCL communicator (cg_comm_*): one rank per MI355X of
// a node, each with its own Engine.  Rules shard by job-ID range (every
// cronsun node filters every job, node/node.go:121-141; a rank here evaluates
// one range of jobs for every node), and the only exchanges are the
// all-gather of per-node counts and the gather of the per-node CSR.
//
//	id, _ := gpu.CommUniqueID()            // rank 0; hand it to every rank
//	c, _ := gpu.NewComm(eng, world, rank, id)
//	... eng.ExpandPerNode over the rank's jobs ...
//	start, base, _ := c.NodeOffsets(nNodes) // where this rank's slices land
//	n, _ := c.GatherNodeCSR(0, ruleBase, 1<<31, dOff, dTime, dRule, cap)
type Comm struct {
	c *C.cg_comm
	e *Engine // cg_comm_free locks the engine's context: keep it reachable
}

// CommUniqueID is ncclGetUniqueId: made once (rank 0) and passed to every rank.
func CommUniqueID() ([C.CG_COMM_ID_BYTES]byte, error) {
	var id [C.CG_COMM_ID_BYTES]byte
	cid := (*C.uint8_t)(C.malloc(C.CG_COMM_ID_BYTES))
	defer C.free(unsafe.Pointer(cid))
	if rc := C.cg_comm_unique_id(cid); rc != 0 {
		return id, lastErr(rc)
	}
	copy(id[:], bytesAt(unsafe.Pointer(cid), int(C.CG_COMM_ID_BYTES)))
	return id, nil
}

// NewComm is ncclCommInitRank on the engine's device (collective: every rank
// calls it with the same id).
func NewComm(e *Engine, world, rank int, id [C.CG_COMM_ID_BYTES]byte) (*Comm, error) {
	cid := (*C.uint8_t)(C.malloc(C.CG_COMM_ID_BYTES))
	defer C.free(unsafe.Pointer(cid))
	copy(bytesAt(unsafe.Pointer(cid), int(C.CG_COMM_ID_BYTES)), id[:])
	var c *C.cg_comm
	if rc := C.cg_comm_init(e.ctx, C.int(world), C.int(rank), cid, &c); rc != 0 {
		return nil, lastErr(rc)
	}
	cm := &Comm{c, e}
	runtime.SetFinalizer(cm, func(cm *Comm) { C.cg_comm_free(cm.c) })
	return cm, nil
}

// AllGather returns every rank's values (rank-major), e.g. the event totals
// that place each rank's rule-major CSR in the global one.
func (cm *Comm) AllGather(mine []int64, world int) ([]int64, error) {
	defer runtime.KeepAlive(cm)
	all := make([]int64, len(mine)*world)
	if len(mine) == 0 {
		return all, nil
	}
	rc := C.cg_comm_allgather_i64(cm.c, (*C.int64_t)(unsafe.Pointer(&mine[0])), C.size_t(len(mine)),
		(*C.int64_t)(unsafe.Pointer(&all[0])))
	if rc != 0 {
		return nil, lastErr(rc)
	}
	return all, nil
}

// NodeOffsets all-gathers the per-node counts of every rank's last per-node
// result: start[n] is where this rank's slice of node n lands in the global
// list, base[N+1] the global node offsets.
func (cm *Comm) NodeOffsets(nNodes int) (start, base []int64, err error) {
	defer runtime.KeepAlive(cm)
	start, base = make([]int64, nNodes+1), make([]int64, nNodes+1)
	rc := C.cg_comm_node_offsets(cm.c, (*C.int64_t)(unsafe.Pointer(&start[0])), (*C.int64_t)(unsafe.Pointer(&base[0])))
	if rc != 0 {
		return nil, nil, lastErr(rc)
	}
	return start[:nNodes], base, nil
}

// GatherNodeCSR gathers every rank's last per-node result on root into device
// buffers (root only; pass 0 elsewhere), in chunks whose peer bytes stay within
// budget; ruleBase is this rank's first global rule.  Rule-ordered results are
// concatenated in rank (job-ID) order; when every rank's result is in (time,
// rule) order (SetNodeOrder(NodeOrderTime)) root merges each node's slices
// into one byTime list (cron.go:64-79,220).  Returns the global node-event
// total.
func (cm *Comm) GatherNodeCSR(root int, ruleBase, budget int64, dOff, dTime, dRule uintptr, cap int64) (int64, error) {
	defer runtime.KeepAlive(cm)
	var n C.int64_t
	rc := C.cg_comm_gather_node_csr(cm.c, C.int(root), C.int64_t(ruleBase), C.int64_t(budget),
		(*C.int64_t)(unsafe.Pointer(dOff)), (*C.int64_t)(unsafe.Pointer(dTime)), (*C.int32_t)(unsafe.Pointer(dRule)),
		C.int64_t(cap), &n)
	if rc != 0 {
		return int64(n), lastErr(rc)
	}
	return int64(n), nil
}

// MergeRanks merges, in place, the time-ordered rank slices of every node of a
// per-node CSR already placed in device buffers (cg_node_csr_merge_ranks):
// runBounds holds nNodes*(world+1) ascending positions, run g of node n being
// [runBounds[n*(world+1)+g], runBounds[n*(world+1)+g+1]).  Equal times end in
// rank (= global rule) order.  budget bounds the scratch copy (bytes).
func (e *Engine) MergeRanks(nNodes, world int, runBounds []int64, dTime, dRule uintptr, budget int64) error {
	e.mu.Lock()
	defer e.mu.Unlock()
	if nNodes == 0 || world <= 1 {
		return nil
	}
	if len(runBounds) < nNodes*(world+1) {
		return fmt.Errorf("cronsun gpu: run bounds: %d positions for %d nodes x %d ranks", len(runBounds), nNodes, world)
	}
	rb := (*C.int64_t)(C.malloc(C.size_t(8 * nNodes * (world + 1))))
	defer C.free(unsafe.Pointer(rb))
	copy(int64sAt(unsafe.Pointer(rb), int(nNodes*(world+1))), runBounds)
	rc := C.cg_node_csr_merge_ranks(e.ctx, C.int32_t(nNodes), C.int32_t(world), rb,
		(*C.int64_t)(unsafe.Pointer(dTime)), (*C.int32_t)(unsafe.Pointer(dRule)), C.int64_t(budget))
	runtime.KeepAlive(e)
	if rc != 0 {
		return lastErr(rc)
	}
	return nil
}

// GatherPlan is the gather's chunk plan for per-node counts counts[g*nNodes+n]
// (host only): chunk i = {first node, end node, part, parts}; a node with more
// peer events than the budget is split into parts.
func GatherPlan(counts []int64, world, nNodes, root int, budget int64) ([][4]int64, error) {
	if len(counts) < world*nNodes {
		return nil, fmt.Errorf("cronsun gpu: gather plan: %d counts for %d ranks x %d nodes", len(counts), world, nNodes)
	}
	var n C.int64_t
	words := world * nNodes
	if words < 1 {
		words = 1
	}
	cc := (*C.int64_t)(C.malloc(C.size_t(8 * words)))
	defer C.free(unsafe.Pointer(cc))
	copy(int64sAt(unsafe.Pointer(cc), int(world*nNodes)), counts)
	// sizing call: *n_chunks is set, CG_ECAPACITY when there are any chunks
	if rc := C.cg_comm_gather_plan(cc, C.int32_t(world), C.int32_t(nNodes), C.int32_t(root), C.int64_t(budget), nil, 0, &n); rc != 0 && rc != C.CG_ECAPACITY {
		return nil, lastErr(rc)
	}
	out := make([][4]int64, int(n))
	if n == 0 {
		return out, nil
	}
	buf := (*C.int64_t)(C.malloc(C.size_t(8 * 4 * int(n))))
	defer C.free(unsafe.Pointer(buf))
	if rc := C.cg_comm_gather_plan(cc, C.int32_t(world), C.int32_t(nNodes), C.int32_t(root), C.int64_t(budget), buf, n, &n); rc != 0 {
		return nil, lastErr(rc)
	}
	flat := int64sAt(unsafe.Pointer(buf), 4*int(n))
	for i := range out {
		copy(out[i][:], flat[4*i:4*i+4])
	}
	return out, nil
}
