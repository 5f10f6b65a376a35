"""ctypes bindings for oracle/liboracle.so -- the CPU restatement used as the
checker.  Test infrastructure only (imported by tests/, __graft_entry__.smoke
and bench.py's cpu_baseline leg)."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")
ZONEINFO = os.path.join(ROOT, "tests", "golden", "zoneinfo")
ZERO_TIME = -62135596800

OPT_DEFAULT = 1 | 2 | 4 | 8 | 16 | 64 | 128
OPT_STANDARD = 2 | 4 | 8 | 16 | 32 | 128


class OrSpec(C.Structure):
    _fields_ = [("second", C.c_uint64), ("minute", C.c_uint64), ("hour", C.c_uint64),
                ("dom", C.c_uint64), ("month", C.c_uint64), ("dow", C.c_uint64)]


class OrSched(C.Structure):
    _fields_ = [("kind", C.c_int), ("spec", OrSpec), ("delay_ns", C.c_int64)]


class OrEntry(C.Structure):
    _fields_ = [("s", C.POINTER(OrSched)), ("next", C.c_int64), ("prev", C.c_int64),
                ("id", C.c_int32)]


class OrJobset(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("n_groups", C.c_int32), ("n_rules", C.c_int32),
                ("n_jobs", C.c_int32),
                ("group_off", C.c_void_p), ("group_nodes", C.c_void_p),
                ("group_exists", C.c_void_p), ("rule_job", C.c_void_p),
                ("nid_off", C.c_void_p), ("nids", C.c_void_p),
                ("gid_off", C.c_void_p), ("gids", C.c_void_p),
                ("ex_off", C.c_void_p), ("ex", C.c_void_p),
                ("job_pause", C.c_void_p), ("rule_key", C.c_void_p)]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ORACLE_DIR, "cron_oracle.c")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    L = C.CDLL(LIB_PATH)
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int32
    L.or_loc_from_tzif.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(vp)]
    L.or_loc_fixed.argtypes = [i32, C.POINTER(vp)]
    L.or_loc_utc.argtypes = [C.POINTER(vp)]
    L.or_loc_free.argtypes = [vp]
    L.or_lookup.argtypes = [vp, i64, C.POINTER(i64), C.POINTER(i64)]
    L.or_lookup.restype = i32
    L.or_date.argtypes = [i64] * 6 + [vp]
    L.or_date.restype = i64
    L.or_spec_next.argtypes = [C.POINTER(OrSpec), i64, i32, vp]
    L.or_spec_next.restype = i64
    L.or_sched_next.argtypes = [C.POINTER(OrSched), i64, i32, vp]
    L.or_sched_next.restype = i64
    L.or_every.argtypes = [i64]
    L.or_every.restype = i64
    L.or_const_next.argtypes = [i64, i64, i32]
    L.or_const_next.restype = i64
    L.or_parse.argtypes = [C.c_int, C.c_char_p, C.c_size_t, C.POINTER(OrSched), C.c_char_p, C.c_size_t]
    L.or_get_range.argtypes = [C.c_char_p, C.c_size_t, C.c_uint, C.c_uint, C.POINTER(C.c_uint64), C.c_char_p, C.c_size_t]
    L.or_get_field.argtypes = L.or_get_range.argtypes
    L.or_get_bits.argtypes = [C.c_uint, C.c_uint, C.c_uint]
    L.or_get_bits.restype = C.c_uint64
    L.or_parse_duration.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(i64), C.c_char_p, C.c_size_t]
    L.or_expand.argtypes = [C.POINTER(OrSched), i64, i64, vp, C.POINTER(i64), i64]
    L.or_expand.restype = i64
    L.or_expand_batch.argtypes = [C.POINTER(OrSched), C.c_size_t, i64, i64, vp, C.c_int, vp, vp]
    L.or_expand_batch.restype = i64
    L.or_rule_on_node.argtypes = [C.POINTER(OrJobset), C.c_int, i32, i32]
    L.or_job_is_run_on.argtypes = [C.POINTER(OrJobset), i32, i32]
    L.or_job_nodes.argtypes = [C.POINTER(OrJobset), i32, C.POINTER(i32), i32]
    L.or_job_nodes.restype = i32
    L.or_node_rules_batch.argtypes = [C.POINTER(OrJobset), C.c_int, vp, C.c_size_t, C.c_int, vp, vp]
    L.or_node_rules_batch.restype = i64
    L.or_cron_start.argtypes = [C.POINTER(OrEntry), C.c_size_t, i64, vp]
    L.or_cron_start.restype = None
    L.or_cron_effective.argtypes = [C.POINTER(OrEntry), C.c_size_t]
    L.or_cron_effective.restype = i64
    L.or_cron_fire.argtypes = [C.POINTER(OrEntry), C.c_size_t, i64, i64, vp, C.POINTER(i32)]
    L.or_cron_fire.restype = i64
    L.or_lock_ttl.argtypes = [C.POINTER(OrSched), i64, i32, vp, C.c_int, i64, i64]
    L.or_lock_ttl.restype = i64
    _lib = L
    return L


class Loc:
    """An oracle Location (Go *time.Location restatement)."""

    def __init__(self, name):
        L = lib()
        self.name = name
        h = C.c_void_p()
        if name == "UTC" or name == "Go:UTC":
            rc = L.or_loc_utc(C.byref(h))
        elif name.startswith("fixed:"):
            rc = L.or_loc_fixed(int(name.split(":", 1)[1]), C.byref(h))
        else:
            data = read_tzif(name)
            rc = L.or_loc_from_tzif(data, len(data), C.byref(h))
        if rc != 0:
            raise ValueError(f"oracle: cannot load zone {name}")
        self.h = h

    def __del__(self):
        try:
            lib().or_loc_free(self.h)
        except Exception:
            pass

    def lookup(self, sec):
        s, e = C.c_int64(), C.c_int64()
        off = lib().or_lookup(self.h, sec, C.byref(s), C.byref(e))
        return off, s.value, e.value


def read_tzif(name):
    with open(os.path.join(ZONEINFO, name), "rb") as f:
        return f.read()


def parse(spec, options=OPT_DEFAULT):
    """-> (OrSched or None, error string or None)"""
    s = OrSched()
    err = C.create_string_buffer(1024)
    b = spec.encode()
    rc = lib().or_parse(options, b, len(b), C.byref(s), err, 1024)
    if rc != 0:
        return None, err.value.decode(errors="replace")
    return s, None


def sched_next(s, t, loc, nsec=0):
    return lib().or_sched_next(C.byref(s), t, nsec, loc.h)


class OracleCron:
    """Cron.run's entries driven one wake at a time (or_cron_*, cron.go:210-275).
    Entry ids are the caller's slot numbers."""

    def __init__(self, scheds, loc):
        self.loc = loc
        self.keep = {}
        self.rows = []  # [sched, next, prev, id]
        for i, sc in enumerate(scheds):
            self.keep[i] = sc
            self.rows.append([sc, ZERO_TIME, ZERO_TIME, i])

    def _arr(self):
        a = (OrEntry * max(len(self.rows), 1))()
        for k, (sc, nx, pv, i) in enumerate(self.rows):
            a[k].s = C.pointer(sc)
            a[k].next, a[k].prev, a[k].id = nx, pv, i
        return a

    def _back(self, a):
        self.rows = [[self.keep[a[k].id], a[k].next, a[k].prev, a[k].id]
                     for k in range(len(self.rows))]

    def start(self, now):
        a = self._arr()
        lib().or_cron_start(a, len(self.rows), now, self.loc.h)
        self._back(a)

    def effective(self):
        a = self._arr()
        e = lib().or_cron_effective(a, len(self.rows))
        self._back(a)
        return e

    def fire(self, effective, now):
        a = self._arr()
        ids = (C.c_int32 * max(len(self.rows), 1))()
        k = lib().or_cron_fire(a, len(self.rows), effective, now, self.loc.h, ids)
        self._back(a)
        return sorted(ids[i] for i in range(k))

    def set(self, i, sc, now):
        """add/replace (cron.go:246-252): Next = Next(now), Prev = zero"""
        self.keep[i] = sc
        nx = lib().or_sched_next(C.byref(sc), now, 0, self.loc.h)
        self.rows = [r for r in self.rows if r[3] != i] + [[sc, nx, ZERO_TIME, i]]

    def remove(self, i):
        self.rows = [r for r in self.rows if r[3] != i]

    def snapshot(self):
        return {r[3]: (r[1], r[2]) for r in self.rows}


def lock_ttl(s, now, loc, kind, avg_time, lock_ttl_conf, nsec=0):
    """Cmd.lockTtl (job.go:194-233)."""
    return lib().or_lock_ttl(C.byref(s), now, nsec, loc.h, kind, avg_time, lock_ttl_conf)


def expand(s, t0, t1, loc):
    L = lib()
    n = L.or_expand(C.byref(s), t0, t1, loc.h, None, 0)
    out = (C.c_int64 * max(n, 1))()
    L.or_expand(C.byref(s), t0, t1, loc.h, out, n)
    return list(out[:n])


def sched_array(scheds):
    arr = (OrSched * len(scheds))()
    for i, s in enumerate(scheds):
        arr[i] = s
    return arr


def expand_batch(arr, t0, t1, loc, threads=8, with_times=True):
    """-> (offsets int64[R+1], times int64[E]).  Raises NonTerminating if the
    reference loop never ends for some rule (see stuck_rules)."""
    R = len(arr)
    off = np.zeros(R + 1, dtype=np.int64)
    L = lib()
    total = L.or_expand_batch(arr, R, t0, t1, loc.h, threads, off.ctypes.data, None)
    if total < 0:
        raise NonTerminating(stuck_rules(arr, t0, t1, loc))
    if not with_times:
        return off, None
    times = np.zeros(max(total, 1), dtype=np.int64)
    L.or_expand_batch(arr, R, t0, t1, loc.h, threads, off.ctypes.data, times.ctypes.data)
    return off, times[:total]


def jobset(rin):
    """OrJobset view of an integer-interned rule set (cronsun_amd RulesIn);
    the arrays stay owned by rin."""
    js = OrJobset()
    js.n_nodes, js.n_groups, js.n_rules, js.n_jobs = rin.n_nodes, rin.n_groups, rin.n_rules, rin.n_jobs
    for f in rin.FIELDS:
        setattr(js, f, getattr(rin, f).ctypes.data)
    js.rule_key = rin.rule_key.ctypes.data if rin.rule_key is not None else None
    return js


def node_rules(rin, mode, nodes, threads=8):
    """Rules scheduled on each of `nodes` (each node's own filter over every
    rule, node.go:121-158 -> Job.Cmds): (off[k+1], rules[]) ascending."""
    js = jobset(rin)
    nd = np.ascontiguousarray(nodes, dtype=np.int32)
    off = np.zeros(len(nd) + 1, dtype=np.int64)
    L = lib()
    total = L.or_node_rules_batch(C.byref(js), mode, nd.ctypes.data, len(nd), threads,
                                  off.ctypes.data, None)
    out = np.zeros(max(total, 1), dtype=np.int32)
    L.or_node_rules_batch(C.byref(js), mode, nd.ctypes.data, len(nd), threads, off.ctypes.data,
                          out.ctypes.data)
    return off, out[:total]


def node_list(eo, et, rules):
    """A node's (time, rule) list: the fire lists of `rules` (ascending) in
    rule-major order, from the oracle's rule-major CSR (eo, et)."""
    rules = np.asarray(rules, dtype=np.int64)
    lens = eo[rules + 1] - eo[rules]
    total = int(lens.sum())
    if total == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int32)
    excl = np.concatenate([[0], np.cumsum(lens)[:-1]])
    idx = np.repeat(eo[rules] - excl, lens) + np.arange(total)
    return et[idx], np.repeat(rules, lens).astype(np.int32)


class NonTerminating(Exception):
    """The reference Next loop never terminates for these rule indices."""

    def __init__(self, rules):
        super().__init__(f"non-terminating reference loop for rules {rules[:10]}")
        self.rules = rules


def stuck_rules(arr, t0, t1, loc):
    L = lib()
    return [i for i in range(len(arr)) if L.or_expand(C.byref(arr[i]), t0, t1, loc.h, None, 0) < 0]
