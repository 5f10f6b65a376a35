"""Bulk ingestion of cronsun's etcd values: the JSON of
every key under /cronsun/group/ and /cronsun/cmd/ decoded, validated and
interned in C++ (cg_jobset_ingest_*, cronsun_amd/csrc/cg_ingest.cpp), the
batch form of GetGroups("") + GetJobs() (group.go:39-63, job.go:339-365).

  js = EtcdJobSet(job_docs, group_docs, threads=16)
  js.job_status, js.group_status     per value: INGEST_OK / UNMARSHAL / ...
  js.schedules_c()                   JobRule.Schedule per rule (cg_schedule[])
                                     -> Engine.upload_c for the GPU paths
  js.rules_in()                      the interned CSR for the per-node paths
  js.job_meta()                      Kind, AvgTime, Parallels per job
  js.lock_ttls(now, ...)             Cmd.lockTtl per rule on the GPU
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib
from .model import _Interned


def _docs_array(docs):
    docs = [d if isinstance(d, (bytes, bytearray)) else d.encode() for d in docs]
    ptrs = (C.c_char_p * max(len(docs), 1))(*docs)
    lens = np.array([len(d) for d in docs] or [0], dtype=np.uint64)
    return docs, ptrs, lens


class EtcdJobSet(_Interned):
    def __init__(self, job_docs, group_docs=(), threads=16):
        L = lib()
        h = C.c_void_p()
        check(L.cg_jobset_new(C.byref(h)))
        self._h = h
        keep_g, gp, gl = _docs_array(group_docs)
        self.group_status = np.zeros(max(len(keep_g), 1), dtype=np.int32)
        check(L.cg_jobset_ingest_groups(h, C.cast(gp, C.c_void_p), gl.ctypes.data, len(keep_g),
                                        threads, self.group_status.ctypes.data))
        self.group_status = self.group_status[:len(keep_g)]
        keep_j, jp, jl = _docs_array(job_docs)
        self.job_status = np.zeros(max(len(keep_j), 1), dtype=np.int32)
        check(L.cg_jobset_ingest_jobs(h, C.cast(jp, C.c_void_p), jl.ctypes.data, len(keep_j),
                                      threads, self.job_status.ctypes.data))
        self.job_status = self.job_status[:len(keep_j)]
        c = _lib.cg_rules_in()
        check(L.cg_jobset_rules(h, C.byref(c)))
        self.n_rules, self.n_jobs, self.n_nodes, self.n_groups = (c.n_rules, c.n_jobs, c.n_nodes,
                                                                  c.n_groups)

    def schedules_c(self):
        """ctypes array of cg_schedule, rule order (for Engine.upload_c)."""
        arr = (_lib.cg_schedule * max(self.n_rules, 1))()
        check(lib().cg_jobset_schedules(self._h, C.cast(arr, C.c_void_p), self.n_rules))
        return arr

    def job_meta(self):
        kind = np.zeros(max(self.n_jobs, 1), dtype=np.int32)
        avg = np.zeros(max(self.n_jobs, 1), dtype=np.int64)
        par = np.zeros(max(self.n_jobs, 1), dtype=np.int64)
        check(lib().cg_jobset_job_meta(self._h, kind.ctypes.data, avg.ctypes.data, par.ctypes.data,
                                       self.n_jobs))
        n = self.n_jobs
        return kind[:n], avg[:n], par[:n]

    def job_id(self, j):
        v = lib().cg_jobset_job_id(self._h, j)
        return None if v is None else v

    def group_id(self, g):
        return lib().cg_jobset_group_id(self._h, g)

    def rule_id(self, r):
        v = lib().cg_jobset_rule_id(self._h, r)
        return None if v is None else v

    def lock_ttls(self, now, loc=None, lock_ttl=300, engine=None):
        """Cmd.lockTtl (job.go:194-233) for every rule at `now`, on the GPU."""
        from .engine import default_engine
        eng = engine or default_engine()
        kind, avg, _ = self.job_meta()
        rj = self.rules_in().rule_job[:self.n_rules]
        sp = eng.upload_c(self.schedules_c(), self.n_rules)
        return eng.lock_ttl_batch(sp, loc, now, kind[rj], avg[rj], lock_ttl)


__all__ = ["EtcdJobSet"]
