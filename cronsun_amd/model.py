"""cronsun's Job / JobRule / Group model (job.go:38-84, group.go:17-22) and
its rule -> node resolution, on top of the C++ host interning in
libcronsun_gpu.so (cg_jobset_*).

  JobRule.Valid()                  job.go:291-308
  Job.Cmds(nid, groups)            job.go:591-614  (ExcludeNodeIDs is a no-op there)
  Job.IsRunOn(nid, groups)         job.go:616-630
  Job.GetJobNodes(groups)          web/job.go:222-257 (cumulative excludes)
  JobSet.lock_ttls(now, loc)       Cmd.lockTtl (job.go:194-233) for every rule
  JobSet(jobs, groups)             all jobs interned at once -> RulesIn for the
                                   GPU per-node expansion (node/node.go:121-158
                                   for every node at once)
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import _lib
from ._lib import check, lib
from .cron import Parse, ParseError, Schedule
from .engine import RulesIn

KindCommon, KindAlone, KindInterval = 0, 1, 2


class ErrNilRule(ValueError):
    """errors.go:19 -- a JobRule with an empty timer."""


@dataclass
class Group:
    ID: str
    Name: str = ""
    NodeIDs: List[str] = field(default_factory=list)

    def Included(self, nid):  # group.go:111-119
        return nid in self.NodeIDs


@dataclass
class JobRule:
    ID: str
    Timer: str = ""
    GroupIDs: List[str] = field(default_factory=list)
    NodeIDs: List[str] = field(default_factory=list)
    ExcludeNodeIDs: List[str] = field(default_factory=list)
    Schedule: Optional[Schedule] = None

    def Valid(self):
        """job.go:291-308: parse Timer into Schedule once."""
        if self.Schedule is not None:
            return None
        if len(self.Timer) == 0:
            raise ErrNilRule("invalid job rule, empty timer.")
        try:
            self.Schedule = Parse(self.Timer)
        except ParseError as e:
            raise ParseError(f"invalid JobRule[{self.Timer}], parse err: {e}") from None
        return None


GroupMap = Dict[str, Group]  # Job has a field named Group


@dataclass
class Job:
    ID: str
    Name: str = ""
    Group: str = ""
    Command: str = ""
    User: str = ""
    Rules: List[JobRule] = field(default_factory=list)
    Pause: bool = False
    Timeout: int = 0
    Parallels: int = 0
    Retry: int = 0
    Interval: int = 0
    Kind: int = KindCommon
    AvgTime: int = 0  # ms, job.go:62 (updated by Job.avgTime, job.go:579-589)

    def ValidRules(self):  # job.go:683-690
        for r in self.Rules:
            r.Valid()

    def Cmds(self, nid, gs: GroupMap):
        """job.go:591-614 -> {Job.ID + Rule.ID: (job, rule)}"""
        js = JobSet([self], gs)
        idx = js.cmds(0, nid)
        return {self.ID + js.rules[i].ID: (self, js.rules[i]) for i in idx}

    def IsRunOn(self, nid, gs: GroupMap):
        return JobSet([self], gs).is_run_on(0, nid)

    def GetJobNodes(self, gs: GroupMap):
        return JobSet([self], gs).job_nodes(0)


def _cstr_array(strs):
    enc = [s.encode() for s in strs]
    arr = (C.c_char_p * max(len(enc), 1))(*enc)
    return arr, len(enc), enc


class _Interned:
    """Host-side queries over an interned cg_jobset handle (self._h)."""

    def rules_in(self) -> RulesIn:
        """Copy the interned arrays into a RulesIn (numpy-owned)."""
        return rules_in_of(self._h)

    def node_index(self, nid):
        return lib().cg_jobset_node_index(self._h, nid.encode())

    def node_id(self, idx):
        v = lib().cg_jobset_node_id(self._h, idx)
        return None if v is None else v.decode()

    def cmds(self, job, nid):
        out = np.zeros(max(self.n_rules, 1), dtype=np.int32)
        k = check(lib().cg_jobset_cmds(self._h, job, nid.encode(), out.ctypes.data, len(out)))
        return [int(x) for x in out[:k]]

    def is_run_on(self, job, nid):
        return bool(check(lib().cg_jobset_is_run_on(self._h, job, nid.encode())))

    def job_nodes(self, job):
        cap = 1 << 16
        out = np.zeros(cap, dtype=np.int32)
        k = check(lib().cg_jobset_job_nodes(self._h, job, out.ctypes.data, cap))
        return [self.node_id(int(x)) for x in out[:min(k, cap)]]

    def __del__(self):
        try:
            lib().cg_jobset_free(self._h)
        except Exception:
            pass


class JobSet(_Interned):
    """All jobs + groups interned by the C++ host layer (cg_jobset)."""

    def __init__(self, jobs, groups: GroupMap):
        L = lib()
        h = C.c_void_p()
        check(L.cg_jobset_new(C.byref(h)))
        self._h = h
        self.jobs = list(jobs)
        self.rules: List[JobRule] = []
        self.rule_job: List[int] = []
        for gid, g in groups.items():
            arr, n, keep = _cstr_array(g.NodeIDs)
            check(L.cg_jobset_add_group(h, gid.encode(), C.cast(arr, C.c_void_p), n))
        for ji, j in enumerate(self.jobs):
            check(L.cg_jobset_add_job(h, j.ID.encode(), 1 if j.Pause else 0))
            for r in j.Rules:
                g, ng, k1 = _cstr_array(r.GroupIDs)
                nn_, nnn, k2 = _cstr_array(r.NodeIDs)
                ex, ne, k3 = _cstr_array(r.ExcludeNodeIDs)
                check(L.cg_jobset_add_rule(h, r.ID.encode(), C.cast(g, C.c_void_p), ng,
                                           C.cast(nn_, C.c_void_p), nnn, C.cast(ex, C.c_void_p), ne))
                self.rules.append(r)
                self.rule_job.append(ji)

    @property
    def n_rules(self):
        return len(self.rules)

    def lock_ttls(self, now, loc=None, lock_ttl=300, engine=None):
        """Cmd.lockTtl for every (job, rule) Cmd at time `now` (unix seconds):
        the etcd lease TTL newLock would take (job.go:235-241), 0 for a rule
        that never fires.  lock_ttl = conf.Config.LockTtl."""
        from .engine import default_engine
        eng = engine or default_engine()
        kind = np.array([self.jobs[j].Kind for j in self.rule_job], dtype=np.int32)
        avg = np.array([self.jobs[j].AvgTime for j in self.rule_job], dtype=np.int64)
        return eng.lock_ttl_batch(self.schedules(), loc, now, kind, avg, lock_ttl)

    def schedules(self):
        """Parsed schedules in rule order (JobRule.Valid on each)."""
        for r in self.rules:
            r.Valid()
        return [r.Schedule for r in self.rules]


def rules_in_of(h) -> RulesIn:
    """cg_jobset_rules of a handle, copied into a numpy-owned RulesIn."""
    c = _lib.cg_rules_in()
    check(lib().cg_jobset_rules(h, C.byref(c)))

    def arr(ptr, n, dt):
        if n == 0:
            return np.zeros(0, dtype=dt)
        ct = {np.int64: C.c_int64, np.int32: C.c_int32, np.uint8: C.c_uint8}[dt]
        return np.ctypeslib.as_array((ct * n).from_address(ptr)).copy()

    R, G, J = c.n_rules, c.n_groups, c.n_jobs
    nid_off = arr(c.nid_off, R + 1, np.int64)
    gid_off = arr(c.gid_off, R + 1, np.int64)
    ex_off = arr(c.ex_off, R + 1, np.int64)
    group_off = arr(c.group_off, G + 1, np.int64)
    return RulesIn(
        c.n_nodes, G, R, J,
        group_off=group_off, group_nodes=arr(c.group_nodes, int(group_off[-1]), np.int32),
        group_exists=arr(c.group_exists, G, np.uint8), rule_job=arr(c.rule_job, R, np.int32),
        nid_off=nid_off, nids=arr(c.nids, int(nid_off[-1]), np.int32),
        gid_off=gid_off, gids=arr(c.gids, int(gid_off[-1]), np.int32),
        ex_off=ex_off, ex=arr(c.ex, int(ex_off[-1]), np.int32),
        job_pause=arr(c.job_pause, J, np.uint8),
        rule_key=arr(c.rule_key, R, np.int32) if c.rule_key else None)
