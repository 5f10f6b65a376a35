"""Batch engine over one MI355X: the node/cron/gpu package of the design,
seen from Python.  Wraps a cg_ctx (one HIP device + stream + HBM buffers).

  Engine.upload(schedules)                  -> Specs (SoA packed in HBM)
  Engine.next_batch(specs, loc, t)          Schedule.Next for every rule
  Engine.lock_ttl_batch(specs, loc, now, kind, avg_time_ms, lock_ttl)
                                            Cmd.lockTtl for every rule
  Engine.dispatcher(specs, loc, now)        Cron.run's entry state in HBM
  Engine.expand(specs, loc, t0, t1)         rule-major CSR of fire times
  Engine.expand_device(specs, loc, t0, t1)  same, left in HBM (bench)
  Engine.expand_per_node(specs, loc, t0, t1, rules, mode)
                                            per-node (time, rule) CSR
"""
import ctypes as C
import threading

import numpy as np

from . import _lib
from ._lib import CgError, check, lib


class Specs:
    """An uploaded rule set (device-resident, 32 B per rule)."""

    def __init__(self, engine, handle, n, parent=None):
        self.engine = engine
        self._h = handle
        self.n = n
        self._parent = parent  # keeps the parent of a slice alive

    def __len__(self):
        return self.n

    def slice(self, first, count):
        h = C.c_void_p()
        check(lib().cg_specs_slice(self._h, first, count, C.byref(h)))
        return Specs(self.engine, h, count, parent=self)

    def free(self):
        if self._h:
            lib().cg_specs_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceRules:
    """An uploaded rule set (cg_rules): the interned jobs/groups in HBM."""

    def __init__(self, engine, handle, rules):
        self.engine = engine
        self._h = handle
        self.n_rules, self.n_nodes = rules.n_rules, rules.n_nodes

    def free(self):
        if self._h:
            lib().cg_rules_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Comm:
    """The library's RCCL communicator (cg_comm_*): one rank per MI355X, bound
    to an Engine's device and stream.  unique_id() on rank 0, handed to every
    rank (e.g. torch.distributed.broadcast_object_list), then Comm(engine,
    world, rank, id) on every rank."""

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * 128)()
        check(lib().cg_comm_unique_id(buf))
        return bytes(buf)

    def __init__(self, engine, world, rank, uid):
        if len(uid) != 128:
            raise ValueError("RCCL unique id must be 128 bytes")
        self.engine, self.world, self.rank = engine, int(world), int(rank)
        h = C.c_void_p()
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        check(lib().cg_comm_init(engine._h, self.world, self.rank, buf, C.byref(h)))
        self._h = h

    def allgather_i64(self, values):
        """all[g, i] = rank g's values[i] (host int64)."""
        mine = np.ascontiguousarray(values, dtype=np.int64)
        out = np.zeros((self.world, mine.size), dtype=np.int64)
        check(lib().cg_comm_allgather_i64(self._h, mine.ctypes.data, mine.size, out.ctypes.data))
        return out

    def node_offsets(self, n_nodes):
        """(node_start [N], node_base [N+1]) of every rank's last per-node result
        (the all-gather of per-node counts)."""
        start = np.zeros(max(n_nodes, 1), dtype=np.int64)
        base = np.zeros(n_nodes + 1, dtype=np.int64)
        check(lib().cg_comm_node_offsets(self._h, start.ctypes.data, base.ctypes.data))
        return start[:n_nodes], base

    def gather_node_csr(self, root, rule_base, budget_bytes, d_node_off=0, d_time=0, d_rule=0, cap=0):
        """cg_comm_gather_node_csr into device pointers (root); returns the
        global node-event total."""
        n = C.c_int64()
        check(lib().cg_comm_gather_node_csr(self._h, int(root), int(rule_base), int(budget_bytes),
                                            d_node_off or None, d_time or None, d_rule or None, int(cap),
                                            C.byref(n)))
        return n.value

    def free(self):
        if getattr(self, "_h", None):
            lib().cg_comm_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Dispatcher:
    """Cron.run's entries (node/cron/cron.go:210-275) resident in HBM
    (cg_dispatcher_*): slots with a schedule, Next and Prev."""

    def __init__(self, engine, handle):
        self.engine = engine
        self._h = handle

    def __len__(self):
        return int(lib().cg_dispatcher_count(self._h))

    @property
    def effective(self):
        """The earliest non-zero Next (ZERO_TIME: nothing can fire)."""
        e = C.c_int64()
        check(lib().cg_dispatcher_effective(self._h, C.byref(e)))
        return e.value

    def fire(self, now):
        """One wake at `now` >= effective: the due slots (ascending) and the
        next effective time."""
        n, e = C.c_int64(), C.c_int64()
        check(lib().cg_dispatcher_fire(self._h, int(now), C.byref(n), C.byref(e)))
        due = np.empty(max(n.value, 1), dtype=np.int32)
        check(lib().cg_dispatcher_due(self._h, 0, n.value, due.ctypes.data))
        return due[:n.value], e.value

    def fire_count(self, now):
        """One wake, leaving the due list in HBM: (n_due, next effective)."""
        n, e = C.c_int64(), C.c_int64()
        check(lib().cg_dispatcher_fire(self._h, int(now), C.byref(n), C.byref(e)))
        return n.value, e.value

    def set(self, idx, schedules, now):
        """Add or replace entries: slot idx[j] <- schedules[j], Next = Next(now)."""
        ix = np.ascontiguousarray(np.atleast_1d(idx), dtype=np.int64)
        arr = _as_c_schedules(schedules)
        check(lib().cg_dispatcher_set(self._h, ix.ctypes.data, C.cast(arr, C.c_void_p), len(ix),
                                      int(now)))

    def remove(self, idx):
        ix = np.ascontiguousarray(np.atleast_1d(idx), dtype=np.int64)
        check(lib().cg_dispatcher_remove(self._h, ix.ctypes.data, len(ix)))

    def snapshot(self):
        """(next, prev, live) per slot."""
        n = len(self)
        nx = np.empty(max(n, 1), dtype=np.int64)
        pv = np.empty(max(n, 1), dtype=np.int64)
        lv = np.empty(max(n, 1), dtype=np.uint8)
        check(lib().cg_dispatcher_snapshot(self._h, nx.ctypes.data, pv.ctypes.data, lv.ctypes.data))
        return nx[:n], pv[:n], lv[:n].astype(bool)

    def free(self):
        if self._h:
            lib().cg_dispatcher_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _as_c_schedules(schedules):
    arr = (_lib.cg_schedule * max(len(schedules), 1))()
    for i, s in enumerate(schedules):
        arr[i] = s.to_c() if hasattr(s, "to_c") else s
    return arr


class RulesIn:
    """Integer-interned jobs/groups (cg_rules_in).  Arrays are numpy and kept
    alive by this object."""

    FIELDS = ("group_off", "group_nodes", "group_exists", "rule_job", "nid_off", "nids",
              "gid_off", "gids", "ex_off", "ex", "job_pause")
    DTYPES = {"group_off": np.int64, "group_nodes": np.int32, "group_exists": np.uint8,
              "rule_job": np.int32, "nid_off": np.int64, "nids": np.int32, "gid_off": np.int64,
              "gids": np.int32, "ex_off": np.int64, "ex": np.int32, "job_pause": np.uint8}

    def __init__(self, n_nodes, n_groups, n_rules, n_jobs, rule_key=None, **arrays):
        """rule_key (optional, [R]): the rules' Cmd keys (Job.ID+Rule.ID,
        job.go:130-132) interned so that two rules of one job compare equal
        exactly when their Rule.IDs are; None = every rule its own key."""
        self.n_nodes, self.n_groups, self.n_rules, self.n_jobs = n_nodes, n_groups, n_rules, n_jobs
        for f in self.FIELDS:
            a = np.ascontiguousarray(arrays[f], dtype=self.DTYPES[f])
            if a.size == 0:
                a = np.zeros(1, dtype=self.DTYPES[f])
            setattr(self, f, a)
        self.rule_key = None
        if rule_key is not None:
            k = np.ascontiguousarray(rule_key, dtype=np.int32)
            if k.shape != (n_rules,):
                raise ValueError("rule_key must hold one key per rule")
            self.rule_key = k if k.size else np.zeros(1, dtype=np.int32)

    def slice_rules(self, lo, hi):
        """The rules [lo, hi) as their own rule set (job-ID-range shard): the
        same nodes and groups, the jobs of those rules renumbered from 0.  A
        job's rules must not be split by the cut."""
        if lo < 0 or hi > self.n_rules or lo > hi:
            raise ValueError("rule range out of bounds")
        if 0 < lo < self.n_rules and self.rule_job[lo - 1] == self.rule_job[lo]:
            raise ValueError("the cut splits a job's rules")
        if 0 < hi < self.n_rules and self.rule_job[hi - 1] == self.rule_job[hi]:
            raise ValueError("the cut splits a job's rules")
        rj = self.rule_job[lo:hi]
        j0 = int(rj[0]) if hi > lo else 0
        j1 = int(rj[-1]) + 1 if hi > lo else 0

        def part(off, vals):
            o = off[lo:hi + 1] - off[lo]
            return o, vals[off[lo]:off[hi]]
        nid_off, nids = part(self.nid_off, self.nids)
        gid_off, gids = part(self.gid_off, self.gids)
        ex_off, ex = part(self.ex_off, self.ex)
        return RulesIn(self.n_nodes, self.n_groups, hi - lo, j1 - j0,
                       group_off=self.group_off, group_nodes=self.group_nodes,
                       group_exists=self.group_exists, rule_job=rj - j0, nid_off=nid_off, nids=nids,
                       gid_off=gid_off, gids=gids, ex_off=ex_off, ex=ex,
                       job_pause=self.job_pause[j0:j1],
                       rule_key=None if self.rule_key is None else self.rule_key[lo:hi])

    def to_c(self):
        s = _lib.cg_rules_in()
        s.n_nodes, s.n_groups, s.n_rules, s.n_jobs = (
            self.n_nodes, self.n_groups, self.n_rules, self.n_jobs)
        for f in self.FIELDS:
            setattr(s, f, getattr(self, f).ctypes.data)
        s.rule_key = self.rule_key.ctypes.data if self.rule_key is not None else None
        return s


class Engine:
    def __init__(self, device=0):
        self._lock = threading.Lock()
        h = C.c_void_p()
        check(lib().cg_init(device, C.byref(h)))
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().cg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ specs
    def upload(self, schedules):
        arr = _as_c_schedules(schedules)
        h = C.c_void_p()
        check(lib().cg_specs_upload_schedules(self._h, C.cast(arr, C.c_void_p), len(schedules),
                                              C.byref(h)))
        return Specs(self, h, len(schedules))

    def upload_c(self, arr, n):
        """Upload a ctypes array of cg_schedule (e.g. from cron.parse_batch)."""
        h = C.c_void_p()
        check(lib().cg_specs_upload_schedules(self._h, C.cast(arr, C.c_void_p), n, C.byref(h)))
        return Specs(self, h, n)

    def upload_soa(self, second, minute, hour, dom, month, dow, delay_ns):
        cols = [np.ascontiguousarray(x, dtype=np.uint64) for x in (second, minute, hour, dom, month, dow)]
        d = np.ascontiguousarray(delay_ns, dtype=np.int64)
        soa = _lib.cg_spec_soa(*[c.ctypes.data for c in cols], d.ctypes.data)
        h = C.c_void_p()
        check(lib().cg_specs_upload(self._h, C.byref(soa), len(d), C.byref(h)))
        return Specs(self, h, len(d))

    def _specs(self, specs):
        return specs if isinstance(specs, Specs) else self.upload(specs)

    @staticmethod
    def _loc(loc):
        if loc is None:
            from .cron import UTC
            return UTC()
        return loc

    # ------------------------------------------------------------- Next
    def next_batch(self, specs, loc, t_in):
        sp = self._specs(specs)
        t = np.ascontiguousarray(t_in, dtype=np.int64)
        if t.shape[0] != sp.n:
            raise ValueError("one input time per rule")
        out = np.empty_like(t)
        check(lib().cg_next_batch(self._h, sp._h, self._loc(loc).handle, t.ctypes.data,
                                  out.ctypes.data))
        return out

    def lock_ttl_batch(self, specs, loc, now, kind, avg_time_ms, lock_ttl=300):
        """Cmd.lockTtl (job.go:194-233) per rule at time now[i] (scalar or
        per rule): the lease TTL in seconds, 0 for a rule that never fires.
        kind = Job.Kind, avg_time_ms = Job.AvgTime, lock_ttl = conf LockTtl."""
        sp = self._specs(specs)
        n = sp.n
        t = np.ascontiguousarray(np.broadcast_to(np.asarray(now, dtype=np.int64), (n,)))
        k = np.ascontiguousarray(np.broadcast_to(np.asarray(kind, dtype=np.int32), (n,)))
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(avg_time_ms, dtype=np.int64), (n,)))
        out = np.empty(n, dtype=np.int64)
        check(lib().cg_lock_ttl_batch(self._h, sp._h, self._loc(loc).handle, t.ctypes.data,
                                      k.ctypes.data, a.ctypes.data, int(lock_ttl),
                                      out.ctypes.data))
        return out

    def dispatcher(self, specs, loc, now):
        """Cron.run start (cron.go:212-215) over `specs` at `now`."""
        sp = self._specs(specs)
        h = C.c_void_p()
        check(lib().cg_dispatcher_new(self._h, sp._h, self._loc(loc).handle, int(now), C.byref(h)))
        return Dispatcher(self, h)

    # -------------------------------------------------------- expansion
    def expand(self, specs, loc, t0, t1):
        sp = self._specs(specs)
        n = C.c_int64()
        check(lib().cg_expand_device(self._h, sp._h, self._loc(loc).handle, int(t0), int(t1),
                                     C.byref(n)))
        off = np.empty(sp.n + 1, dtype=np.int64)
        check(lib().cg_result_copy_offsets(self._h, off.ctypes.data))
        times = np.empty(max(n.value, 1), dtype=np.int64)
        check(lib().cg_result_copy_times(self._h, 0, n.value, times.ctypes.data))
        return off, times[:n.value]

    def count(self, specs, loc, t0, t1):
        """Fires per rule in (t0, t1] (count pass only, cg_count)."""
        sp = self._specs(specs)
        out = np.empty(max(sp.n, 1), dtype=np.int64)
        tot = C.c_int64()
        check(lib().cg_count(self._h, sp._h, self._loc(loc).handle, int(t0), int(t1),
                             out.ctypes.data, C.byref(tot)))
        return out[:sp.n]

    def expand_device(self, specs, loc, t0, t1):
        n = C.c_int64()
        check(lib().cg_expand_device(self._h, specs._h, self._loc(loc).handle, int(t0), int(t1),
                                     C.byref(n)))
        return n.value

    def expand_async(self, specs, loc, t0, t1):
        """Enqueue a pipelined expansion (cg_expand_device_async): returns at
        once; results and errors come with expand_wait()."""
        check(lib().cg_expand_device_async(self._h, specs._h, self._loc(loc).handle, int(t0), int(t1)))

    def expand_wait(self):
        """Wait for the async expansions since the last wait; the event total of
        the last one (its result is then the engine's current result)."""
        n = C.c_int64()
        check(lib().cg_expand_wait(self._h, C.byref(n)))
        return n.value

    def result_device(self):
        off, times, n = C.c_void_p(), C.c_void_p(), C.c_int64()
        check(lib().cg_result_device(self._h, C.byref(off), C.byref(times), C.byref(n)))
        return off.value, times.value, n.value

    def copy_times(self, first, count):
        out = np.empty(max(count, 1), dtype=np.int64)
        check(lib().cg_result_copy_times(self._h, int(first), int(count), out.ctypes.data))
        return out[:count]

    def kernel_times(self):
        """ms per phase of the last expansion: count, scan, block map,
        write(closed form), write(walk), offsets."""
        buf = (C.c_float * 12)()
        k = lib().cg_last_kernel_times(self._h, buf, 12)
        return list(buf)[:min(k, 6)]

    def set_phase_timing(self, level):
        """2: HIP events between all expansion phases (default); 1: around
        k_write_cf only (the other phases then read -1)."""
        check(lib().cg_set_phase_timing(self._h, int(level)))

    def node_kernel_times(self):
        """ms per phase of the last per-node call: rule->node join,
        transpose + per-node offsets, per-node write."""
        buf = (C.c_float * 12)()
        lib().cg_last_kernel_times(self._h, buf, 12)
        return list(buf)[6:9]

    def dispatch_kernel_times(self):
        """ms of the last dispatcher wake: scan, due compaction, advance."""
        buf = (C.c_float * 12)()
        lib().cg_last_kernel_times(self._h, buf, 12)
        return list(buf)[9:12]

    def sync(self):
        check(lib().cg_sync(self._h))

    # --------------------------------------------------------- per node
    def rule_nodes(self, rules, mode=_lib.EXCLUDE_NONE):
        rin = rules.to_c()
        nnz = C.c_int64()
        check(lib().cg_rule_nodes(self._h, C.byref(rin), mode, None, None, 0, C.byref(nnz)))
        off = np.empty(rules.n_rules + 1, dtype=np.int64)
        nodes = np.empty(max(nnz.value, 1), dtype=np.int32)
        check(lib().cg_rule_nodes(self._h, C.byref(rin), mode, off.ctypes.data, nodes.ctypes.data,
                                  nnz.value, C.byref(nnz)))
        return off, nodes[:nnz.value]

    def expand_per_node(self, specs, loc, t0, t1, rules, mode=_lib.EXCLUDE_NONE):
        sp = self._specs(specs)
        rin = rules.to_c()
        En, nnz = C.c_int64(), C.c_int64()
        check(lib().cg_expand_per_node_device(self._h, sp._h, self._loc(loc).handle, int(t0),
                                              int(t1), C.byref(rin), mode, C.byref(En),
                                              C.byref(nnz)))
        out = _lib.cg_node_csr()
        node_off = np.empty(rules.n_nodes + 1, dtype=np.int64)
        time = np.empty(max(En.value, 1), dtype=np.int64)
        rule = np.empty(max(En.value, 1), dtype=np.int32)
        out.node_off, out.time, out.rule = node_off.ctypes.data, time.ctypes.data, rule.ctypes.data
        out.cap = En.value
        check(lib().cg_expand_per_node(self._h, sp._h, self._loc(loc).handle, int(t0), int(t1),
                                       C.byref(rin), mode, C.byref(out)))
        return node_off, time[:En.value], rule[:En.value]

    def expand_per_node_device(self, specs, loc, t0, t1, rules, mode=_lib.EXCLUDE_NONE):
        rin = rules.to_c()
        En, nnz = C.c_int64(), C.c_int64()
        check(lib().cg_expand_per_node_device(self._h, specs._h, self._loc(loc).handle, int(t0),
                                              int(t1), C.byref(rin), mode, C.byref(En),
                                              C.byref(nnz)))
        return En.value, nnz.value

    def upload_rules(self, rules):
        """A rule set resident in HBM (validated once; cg_rules_upload)."""
        h = C.c_void_p()
        rin = rules.to_c()
        check(lib().cg_rules_upload(self._h, C.byref(rin), C.byref(h)))
        return DeviceRules(self, h, rules)

    def expand_per_node_rules_device(self, specs, loc, t0, t1, drules, mode=_lib.EXCLUDE_NONE):
        En, nnz = C.c_int64(), C.c_int64()
        check(lib().cg_expand_per_node_rules_device(self._h, specs._h, self._loc(loc).handle,
                                                    int(t0), int(t1), drules._h, mode,
                                                    C.byref(En), C.byref(nnz)))
        return En.value, nnz.value

    def expand_per_node_async(self, specs, loc, t0, t1, drules, mode=_lib.EXCLUDE_NONE):
        """Enqueue one per-node window (cg_expand_per_node_rules_device_async):
        the next window's expansion and records overlap this one's writer.
        Results and errors come with expand_per_node_wait()."""
        check(lib().cg_expand_per_node_rules_device_async(self._h, specs._h, self._loc(loc).handle, int(t0),
                                                          int(t1), drules._h, mode))

    def expand_per_node_wait(self, with_total=False):
        """Wait for the pipelined per-node windows; returns the last window's
        node-event total (its result is then the readable per-node result),
        and with with_total also the node events of every window waited for."""
        n, tot = C.c_int64(), C.c_int64()
        check(lib().cg_expand_per_node_wait(self._h, C.byref(n), C.byref(tot)))
        return (n.value, tot.value) if with_total else n.value

    def node_result_device(self):
        """Device pointers of the last per-node result: (node_off, time, rule, n_events)."""
        o, t, r, n = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int64()
        check(lib().cg_node_result_device(self._h, C.byref(o), C.byref(t), C.byref(r), C.byref(n)))
        return o.value, t.value, r.value, n.value

    def node_result_tensors(self, n_nodes):
        """The last per-node result as zero-copy torch views of the engine's
        device buffers (node_off int64 [N+1], time int64 [E], rule int32 [E]),
        valid until the next per-node call (__cuda_array_interface__)."""
        import torch
        o, t, r, n = self.node_result_device()

        class _View:
            def __init__(self, ptr, count, typestr):
                self.__cuda_array_interface__ = {"shape": (count,), "typestr": typestr,
                                                 "data": (ptr, False), "version": 3}
        dev = torch.device("cuda", self.device)
        return (torch.as_tensor(_View(o, n_nodes + 1, "<i8"), device=dev),
                torch.as_tensor(_View(t, n, "<i8"), device=dev),
                torch.as_tensor(_View(r, n, "<i4"), device=dev))

    def node_result(self, n_nodes, n_events):
        """Copy the last per-node result (node_off, time, rule) to host."""
        node_off = np.empty(n_nodes + 1, dtype=np.int64)
        time = np.empty(max(n_events, 1), dtype=np.int64)
        rule = np.empty(max(n_events, 1), dtype=np.int32)
        check(lib().cg_node_result_copy(self._h, node_off.ctypes.data, time.ctypes.data,
                                        rule.ctypes.data, n_events))
        return node_off, time[:n_events], rule[:n_events]

    def node_checksum_enqueue(self, d_nodes, k, d_out):
        """cg_node_checksum_enqueue: checksums of k nodes' lists of the last
        enqueued window (device pointers: int32 nodes [k], uint64 out [2k])."""
        check(lib().cg_node_checksum_enqueue(self._h, d_nodes, int(k), d_out))

    @staticmethod
    def node_list_checksum(time, rule):
        """The host form of cg_node_checksum_enqueue's checksums of one list."""
        def mix(x):
            x = x ^ (x >> np.uint64(30))
            x = x * np.uint64(0xBF58476D1CE4E5B9)
            x = x ^ (x >> np.uint64(27))
            x = x * np.uint64(0x94D049BB133111EB)
            return x ^ (x >> np.uint64(31))
        with np.errstate(over="ignore"):
            h = mix(np.arange(len(time), dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
            ct = mix(np.asarray(time, dtype=np.int64).view(np.uint64) ^ h).sum(dtype=np.uint64)
            cr = mix(np.asarray(rule, dtype=np.int64).view(np.uint64) ^ h).sum(dtype=np.uint64)
        return int(ct), int(cr)

    def node_copy_range(self, first, count):
        """Events [first, first+count) of the last per-node result (time, rule)."""
        time = np.empty(max(count, 1), dtype=np.int64)
        rule = np.empty(max(count, 1), dtype=np.int32)
        check(lib().cg_node_result_copy_range(self._h, int(first), int(count), time.ctypes.data,
                                              rule.ctypes.data))
        return time[:count], rule[:count]

    def set_node_order(self, order):
        """Order of every node's list in later per-node calls
        (cg_set_node_order): _lib.NODE_ORDER_RULE (rule-major, the default) or
        _lib.NODE_ORDER_TIME ((time, rule), the byTime order of Cron.run,
        cron.go:64-79,220: the time-order pass runs inside every per-node call,
        pipelined windows included)."""
        check(lib().cg_set_node_order(self._h, int(order)))

    def node_order_by_time(self):
        """Reorder every node's list of the last per-node result by (time,
        rule) in device memory (cg_node_result_order_by_time; the byTime order
        of Cron.run, cron.go:64-79,220).  Returns the pass's ms."""
        check(lib().cg_node_result_order_by_time(self._h))
        buf = (C.c_float * 13)()
        lib().cg_last_kernel_times(self._h, buf, 13)
        return buf[12]

    def last_order_ms(self):
        """ms of the last time-order pass (cg_last_kernel_times [12]): the pass
        inside the last synchronous per-node call in CG_NODE_ORDER_TIME, or
        the last cg_node_result_order_by_time."""
        buf = (C.c_float * 13)()
        check(lib().cg_last_kernel_times(self._h, buf, 13))
        return buf[12]

    def node_csr_place(self, n_nodes, src_node_off, src_time, src_rule, rule_add, dst_start, dst_time, dst_rule):
        """Place one rank's per-node slice into the gathered per-node CSR on
        this engine's device (cg_node_csr_place); arguments are device
        pointers (ints), e.g. torch tensors' data_ptr()."""
        check(lib().cg_node_csr_place(self._h, int(n_nodes), C.c_void_p(src_node_off), C.c_void_p(src_time),
                                      C.c_void_p(src_rule), int(rule_add), C.c_void_p(dst_start),
                                      C.c_void_p(dst_time), C.c_void_p(dst_rule)))

    def node_csr_merge_ranks(self, n_nodes, world, run_bounds, d_time, d_rule, budget_bytes=1 << 31):
        """Merge every node's rank slices of a gathered per-node CSR into
        (time, rule) order in place (cg_node_csr_merge_ranks): run_bounds
        [n_nodes, world + 1] (host int64; run g of node n is [rb[n, g],
        rb[n, g + 1])), each run already in (time, rule) order; d_time /
        d_rule device pointers on this engine's device."""
        rb = np.ascontiguousarray(run_bounds, dtype=np.int64)
        if rb.size != n_nodes * (world + 1):
            raise ValueError("run_bounds must hold n_nodes * (world + 1) positions")
        check(lib().cg_node_csr_merge_ranks(self._h, int(n_nodes), int(world), rb.ctypes.data, C.c_void_p(d_time),
                                            C.c_void_p(d_rule), int(budget_bytes)))

    def node_counts_to_device(self, d_ptr):
        check(lib().cg_node_counts_to_device(self._h, C.c_void_p(d_ptr)))

    def fill(self, d_ptr, nbytes, byte_value=0xFF):
        """Fill a device buffer with one byte value (cg_fill_device)."""
        check(lib().cg_fill_device(self._h, C.c_void_p(d_ptr), int(nbytes), int(byte_value)))

    def fill_rates(self, d_ptr, nbytes, reps=5):
        """Store ceiling of this device over nbytes of a device buffer
        (cg_fill_rate_device): mean ms of k_fill_stream with nontemporal
        stores, with plain stores, and of hipMemsetAsync."""
        ms = (C.c_float * 3)()
        check(lib().cg_fill_rate_device(self._h, C.c_void_p(d_ptr), int(nbytes), int(reps), ms))
        return {"fill_stream_nt": ms[0], "fill_stream_plain": ms[1], "hipMemsetAsync": ms[2]}

    def count_value(self, d_ptr, n, elem_bytes=8, value=-1):
        """Elements of a device array equal to value (cg_count_value_device)."""
        out = C.c_int64()
        check(lib().cg_count_value_device(self._h, C.c_void_p(d_ptr), int(n), int(elem_bytes),
                                          int(value), C.byref(out)))
        return out.value

    def checksum(self, d_ptr, n, elem_bytes=8, first_index=0, add=0):
        """Order-sensitive checksum of a device array (cg_checksum_device);
        checksums of consecutive ranges add up mod 2^64."""
        out = C.c_uint64()
        check(lib().cg_checksum_device(self._h, C.c_void_p(d_ptr), int(n), int(elem_bytes),
                                       int(first_index), int(add), C.byref(out)))
        return out.value


_default = None
_default_lock = threading.Lock()


def default_engine():
    global _default
    with _default_lock:
        if _default is None:
            _default = Engine(0)
        return _default


def comm_gather_plan(counts, root, budget_bytes):
    """The library's chunk plan of the per-node CSR gather
    (cg_comm_gather_plan; host only): counts [world, N] per-node event counts
    of every rank.  Returns [(n0, n1, j, k)], as shard.node_gather_plan."""
    cnt = np.ascontiguousarray(counts, dtype=np.int64)
    world, N = cnt.shape
    n = C.c_int64()
    cap = max(1, 2 * N + 16)
    while True:
        out = np.zeros((cap, 4), dtype=np.int64)
        rc = lib().cg_comm_gather_plan(cnt.ctypes.data, world, N, int(root), int(budget_bytes), out.ctypes.data,
                                       cap, C.byref(n))
        if rc == _lib.CG_ECAPACITY:
            cap = int(n.value)
            continue
        check(rc)
        return [tuple(int(x) for x in row) for row in out[:n.value]]


def device_count():
    return lib().cg_device_count()


__all__ = ["Engine", "Specs", "Dispatcher", "RulesIn", "Comm", "default_engine", "device_count", "CgError",
           "comm_gather_plan"]
