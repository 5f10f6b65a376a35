"""ctypes binding of libcronsun_gpu.so (the C-ABI in include/cronsun_gpu.h).

There is no CPU fallback: if the library is missing this module raises, and
compute calls fail with CG_ENODEV on a host without an MI355X.
"""
import ctypes as C
import importlib.util
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# CRONSUN_GPU_LIB: an alternative in-tree build of the same library (A/B experiments)
_DEFAULT_LIB = os.path.join(HERE, "libcronsun_gpu.so")
LIB_PATH = os.environ.get("CRONSUN_GPU_LIB") or _DEFAULT_LIB

CG_OK = 0
CG_EINVAL = -1
CG_ENOMEM = -2
CG_EHIP = -3
CG_ECAPACITY = -4
CG_EPARSE = -5
CG_ERANGE = -6
CG_ENODEV = -7
CG_EPANIC = -8
ZERO_TIME = -62135596800
NO_PROGRESS_TIME = -(1 << 63) + 1
MAX_HORIZON = 14610 * 86400  # 40 years (include/cronsun_gpu.h)

PARSE_SECOND, PARSE_MINUTE, PARSE_HOUR, PARSE_DOM = 1, 2, 4, 8
PARSE_MONTH, PARSE_DOW, PARSE_DOW_OPTIONAL, PARSE_DESCRIPTOR = 16, 32, 64, 128
PARSE_DEFAULT = 1 | 2 | 4 | 8 | 16 | 64 | 128
PARSE_STANDARD = 2 | 4 | 8 | 16 | 32 | 128

EXCLUDE_NONE, EXCLUDE_RULE, EXCLUDE_CUMULATIVE = 0, 1, 2
NODE_ORDER_RULE, NODE_ORDER_TIME = 0, 1  # cg_set_node_order
INGEST_OK, INGEST_UNMARSHAL, INGEST_INVALID, INGEST_PANIC, INGEST_REPLACED, INGEST_UNSUPPORTED = range(6)


class CgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code
        self.msg = msg


class cg_schedule(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32),
                ("second", C.c_uint64), ("minute", C.c_uint64), ("hour", C.c_uint64),
                ("dom", C.c_uint64), ("month", C.c_uint64), ("dow", C.c_uint64),
                ("delay_ns", C.c_int64)]


class cg_spec_soa(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("second", "minute", "hour", "dom", "month", "dow", "delay_ns")]


class cg_csr(C.Structure):
    _fields_ = [("offsets", C.c_void_p), ("times", C.c_void_p),
                ("times_cap", C.c_int64), ("n_events", C.c_int64)]


ABI_VERSION = 3  # CG_ABI_VERSION of include/cronsun_gpu.h


class cg_rules_in(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("n_groups", C.c_int32), ("n_rules", C.c_int32),
                ("n_jobs", C.c_int32)] + [(n, C.c_void_p) for n in (
                    "group_off", "group_nodes", "group_exists", "rule_job", "nid_off", "nids",
                    "gid_off", "gids", "ex_off", "ex", "job_pause", "rule_key")]


class cg_node_csr(C.Structure):
    _fields_ = [("node_off", C.c_void_p), ("time", C.c_void_p), ("rule", C.c_void_p),
                ("cap", C.c_int64), ("n_events", C.c_int64), ("nnz", C.c_int64)]


def _preload_torch_hip():
    """Make the process's HIP runtime the one PyTorch-ROCm ships (same SONAME
    libamdhip64.so.7), so torch and this library never load two runtimes."""
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    p = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(p):
        C.CDLL(p, mode=C.RTLD_GLOBAL)


def preload_torch_rccl():
    """Convenience only: import torch (when installed) before the first
    cg_comm call.  The library itself keeps one RCCL per process whatever the
    order: it uses an RCCL already mapped, else loads the librccl.so beside the
    HIP runtime it runs on (torch's copy under PyTorch-ROCm, which a later
    torch import then maps as the same file) by full path with local symbol
    scope, and refuses (CG_EINVAL) when a different RCCL appears later.  Round
    4 loaded "librccl.so" by name with global scope, which resolved to
    /opt/rocm's copy through LD_LIBRARY_PATH and was then bound by torch's
    libraries in place of their own: a heap abort at exit
    (tools/probe_comm_exit.py comm_torch)."""
    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def _declare(L):
    vp, i32, i64, u64, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_size_t
    P = C.POINTER
    sigs = {
        "cg_abi_version": ([], C.c_int),
        "cg_last_error": ([], C.c_char_p),
        "cg_device_count": ([], C.c_int),
        "cg_build_info": ([], C.c_int),
        "cg_parse": ([C.c_int, C.c_char_p, sz, P(cg_schedule), C.c_char_p, sz], C.c_int),
        "cg_parse_batch": ([C.c_int, vp, vp, sz, vp, vp, C.c_int], C.c_int),
        "cg_get_range": ([C.c_char_p, sz, C.c_uint, C.c_uint, C.c_int, P(u64), C.c_char_p, sz], C.c_int),
        "cg_get_field": ([C.c_char_p, sz, C.c_uint, C.c_uint, C.c_int, P(u64), C.c_char_p, sz], C.c_int),
        "cg_get_bits": ([C.c_uint, C.c_uint, C.c_uint], u64),
        "cg_every": ([i64], i64),
        "cg_parse_duration": ([C.c_char_p, sz, P(i64)], C.c_int),
        "cg_zone_from_tzif": ([C.c_char_p, sz, P(vp)], C.c_int),
        "cg_zone_fixed": ([i32, P(vp)], C.c_int),
        "cg_zone_utc": ([P(vp)], C.c_int),
        "cg_zone_free": ([vp], None),
        "cg_zone_offset": ([vp, i64, P(i32)], C.c_int),
        "cg_zone_table": ([vp, i64, i64, vp, vp, C.c_int], C.c_int),
        "cg_init": ([C.c_int, P(vp)], C.c_int),
        "cg_destroy": ([vp], None),
        "cg_sync": ([vp], C.c_int),
        "cg_specs_upload": ([vp, P(cg_spec_soa), sz, P(vp)], C.c_int),
        "cg_specs_upload_schedules": ([vp, vp, sz, P(vp)], C.c_int),
        "cg_specs_slice": ([vp, sz, sz, P(vp)], C.c_int),
        "cg_specs_count": ([vp], sz),
        "cg_specs_free": ([vp], None),
        "cg_next_batch": ([vp, vp, vp, vp, vp], C.c_int),
        "cg_lock_ttl_batch": ([vp, vp, vp, vp, vp, vp, i64, vp], C.c_int),
        "cg_dispatcher_new": ([vp, vp, vp, i64, P(vp)], C.c_int),
        "cg_dispatcher_free": ([vp], None),
        "cg_dispatcher_count": ([vp], i64),
        "cg_dispatcher_effective": ([vp, P(i64)], C.c_int),
        "cg_dispatcher_fire": ([vp, i64, P(i64), P(i64)], C.c_int),
        "cg_dispatcher_due": ([vp, i64, i64, vp], C.c_int),
        "cg_dispatcher_due_device": ([vp, P(vp), P(i64)], C.c_int),
        "cg_dispatcher_set": ([vp, vp, vp, sz, i64], C.c_int),
        "cg_dispatcher_remove": ([vp, vp, sz], C.c_int),
        "cg_dispatcher_snapshot": ([vp, vp, vp, vp], C.c_int),
        "cg_expand": ([vp, vp, vp, i64, i64, P(cg_csr)], C.c_int),
        "cg_count": ([vp, vp, vp, i64, i64, vp, P(i64)], C.c_int),
        "cg_expand_device": ([vp, vp, vp, i64, i64, P(i64)], C.c_int),
        "cg_expand_device_async": ([vp, vp, vp, i64, i64], C.c_int),
        "cg_expand_wait": ([vp, P(i64)], C.c_int),
        "cg_result_device": ([vp, P(vp), P(vp), P(i64)], C.c_int),
        "cg_result_copy_times": ([vp, i64, i64, vp], C.c_int),
        "cg_result_copy_offsets": ([vp, vp], C.c_int),
        "cg_last_kernel_times": ([vp, P(C.c_float), C.c_int], C.c_int),
        "cg_set_phase_timing": ([vp, C.c_int], C.c_int),
        "cg_expand_per_node": ([vp, vp, vp, i64, i64, P(cg_rules_in), C.c_int, P(cg_node_csr)], C.c_int),
        "cg_expand_per_node_device": ([vp, vp, vp, i64, i64, P(cg_rules_in), C.c_int, P(i64), P(i64)], C.c_int),
        "cg_node_result_device": ([vp, P(vp), P(vp), P(vp), P(i64)], C.c_int),
        "cg_node_result_copy": ([vp, vp, vp, vp, i64], C.c_int),
        "cg_node_counts_to_device": ([vp, vp], C.c_int),
        "cg_node_checksum_enqueue": ([vp, vp, C.c_int32, vp], C.c_int),
        "cg_node_csr_place": ([vp, C.c_int32, vp, vp, vp, C.c_int32, vp, vp, vp], C.c_int),
        "cg_node_csr_merge_ranks": ([vp, C.c_int32, C.c_int32, vp, vp, vp, i64], C.c_int),
        "cg_expand_per_node_rules_device_async": ([vp, vp, vp, i64, i64, vp, C.c_int], C.c_int),
        "cg_expand_per_node_wait": ([vp, P(i64), P(i64)], C.c_int),
        "cg_node_result_copy_range": ([vp, i64, i64, vp, vp], C.c_int),
        "cg_node_result_order_by_time": ([vp], C.c_int),
        "cg_set_node_order": ([vp, C.c_int], C.c_int),
        "cg_checksum_device": ([vp, vp, i64, C.c_int, i64, i64, P(u64)], C.c_int),
        "cg_fill_device": ([vp, vp, i64, C.c_int], C.c_int),
        "cg_fill_rate_device": ([vp, vp, i64, C.c_int, P(C.c_float)], C.c_int),
        "cg_count_value_device": ([vp, vp, i64, C.c_int, i64, P(i64)], C.c_int),
        "cg_rules_upload": ([vp, P(cg_rules_in), P(vp)], C.c_int),
        "cg_rules_free": ([vp], None),
        "cg_expand_per_node_rules_device": ([vp, vp, vp, i64, i64, vp, C.c_int, P(i64), P(i64)],
                                            C.c_int),
        "cg_rule_nodes": ([vp, P(cg_rules_in), C.c_int, vp, vp, i64, P(i64)], C.c_int),
        "cg_comm_unique_id": ([vp], C.c_int),
        "cg_comm_init": ([vp, C.c_int, C.c_int, vp, P(vp)], C.c_int),
        "cg_comm_free": ([vp], None),
        "cg_comm_allgather_i64": ([vp, vp, sz, vp], C.c_int),
        "cg_comm_node_offsets": ([vp, vp, vp], C.c_int),
        "cg_comm_gather_node_csr": ([vp, C.c_int, i64, i64, vp, vp, vp, i64, P(i64)], C.c_int),
        "cg_comm_gather_plan": ([vp, C.c_int32, C.c_int32, C.c_int32, i64, vp, i64, P(i64)], C.c_int),
        "cg_jobset_new": ([P(vp)], C.c_int),
        "cg_jobset_free": ([vp], None),
        "cg_jobset_add_group": ([vp, C.c_char_p, vp, sz], C.c_int),
        "cg_jobset_add_job": ([vp, C.c_char_p, C.c_int], C.c_int),
        "cg_jobset_add_rule": ([vp, C.c_char_p, vp, sz, vp, sz, vp, sz], C.c_int),
        "cg_jobset_rules": ([vp, P(cg_rules_in)], C.c_int),
        "cg_jobset_node_index": ([vp, C.c_char_p], i32),
        "cg_jobset_node_id": ([vp, i32], C.c_char_p),
        "cg_jobset_cmds": ([vp, i32, C.c_char_p, vp, i32], i32),
        "cg_jobset_is_run_on": ([vp, i32, C.c_char_p], C.c_int),
        "cg_jobset_job_nodes": ([vp, i32, vp, i32], i32),
        "cg_jobset_ingest_groups": ([vp, vp, vp, sz, C.c_int, vp], C.c_int),
        "cg_jobset_ingest_jobs": ([vp, vp, vp, sz, C.c_int, vp], C.c_int),
        "cg_jobset_schedules": ([vp, vp, sz], C.c_int),
        "cg_jobset_job_meta": ([vp, vp, vp, vp, sz], C.c_int),
        "cg_jobset_job_id": ([vp, i32], C.c_char_p),
        "cg_jobset_group_id": ([vp, i32], C.c_char_p),
        "cg_jobset_rule_id": ([vp, i32], C.c_char_p),
    }
    strict = os.path.abspath(LIB_PATH) == os.path.abspath(_DEFAULT_LIB)
    for name, (args, res) in sigs.items():
        # an older library picked by CRONSUN_GPU_LIB for an A/B may lack newer
        # entry points (tests/test_exports.py checks the production library)
        fn = getattr(L, name) if strict else getattr(L, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = res
    return list(sigs)


_L = None
SYMBOLS = []


def lib():
    """The loaded library.  Raises if it has not been built."""
    global _L, SYMBOLS
    if _L is not None:
        return _L
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C cronsun_amd/csrc` (there is no CPU fallback)")
    _preload_torch_hip()
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    SYMBOLS = _declare(L)
    if L.cg_abi_version() != ABI_VERSION:
        raise ImportError("libcronsun_gpu ABI mismatch")
    _L = L
    return L


def check(rc):
    if rc < 0:
        raise CgError(rc, (lib().cg_last_error() or b"").decode(errors="replace"))
    return rc


def last_error():
    return (lib().cg_last_error() or b"").decode(errors="replace")
