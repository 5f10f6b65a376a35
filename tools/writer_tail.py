"""Ramp and tail of the headline writer k_write_cf on config 2 (1M rules x
24 h, UTC): per-wave wall-clock stamps from the diagnostic library
(`make -C cronsun_amd/csrc diag`, CG_WRITE_STAMPS=1: {start, end, slices,
the time its ticket group ran dry} per wave, 100 MHz), over synchronous
expansions.  Per launch: the wave start spread (ramp), when the first and the
p50/p90/p99 waves finish relative to the last (tail), the idle share of the
wave-time (sum over waves of last end - own end), and a 10-us histogram of
wave end times.

  CRONSUN_GPU_LIB=cronsun_amd/libcronsun_gpu_diag.so CG_WRITE_STAMPS=1 \\
      python3 tools/writer_tail.py <out.json> [launches]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_path = sys.argv[1]
    n_launch = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    from cronsun_amd import _lib, cron, synth
    from cronsun_amd.engine import Engine
    L = _lib.lib()
    L.cg_diag_write_stamps.restype = C.c_int
    L.cg_diag_write_stamps.argtypes = [C.c_void_p, C.c_int64]
    specs = synth.spec_mix(1_000_000, seed=0x5EED, mix=synth.MIX_CONFIG2)
    arr, st = cron.parse_batch(specs, threads=16)
    assert (st == 0).all()
    eng = Engine(0)
    sp = eng.upload_c(arr, len(specs))
    t0 = synth.T0_2026
    eng.set_phase_timing(1)
    buf = np.zeros((1 << 16, 4), dtype=np.int64)
    rec = []
    for k in range(n_launch + 2):
        E = eng.expand_device(sp, None, t0, t0 + 86400)
        w_ms = eng.kernel_times()[3]
        n = L.cg_diag_write_stamps(buf.ctypes.data, buf.shape[0])
        if k < 2 or n == 0:
            continue
        s = buf[:n]
        live = s[:, 1] > 0
        s = s[live]
        T0 = s[:, 0].min()
        T1 = s[:, 1].max()
        dur = (T1 - T0) * 10e-3  # us
        start = (s[:, 0] - T0) * 10e-3
        end = (s[:, 1] - T0) * 10e-3
        dry = (s[s[:, 3] > 0, 3] - T0) * 10e-3
        idle = float(((T1 - s[:, 1]) * 10e-3).sum() / (len(s) * dur))
        hist, edges = np.histogram(end, bins=np.arange(0, dur + 10, 10))
        rec.append({
            "events": int(E), "waves": int(len(s)), "hip_event_ms": float(w_ms), "stamp_span_us": float(dur),
            "start_us": {q: float(np.percentile(start, p)) for q, p in (("p50", 50), ("p99", 99), ("max", 100))},
            "end_us": {q: float(np.percentile(end, p)) for q, p in (("min", 0), ("p10", 10), ("p50", 50), ("p90", 90),
                                                                     ("p99", 99), ("max", 100))},
            "dry_us": {q: float(np.percentile(dry, p)) for q, p in (("min", 0), ("p50", 50), ("max", 100))} if len(dry) else None,
            "slices": {"min": int(s[:, 2].min()), "mean": float(s[:, 2].mean()), "max": int(s[:, 2].max())},
            "idle_share_after_own_end": idle,
            "end_hist_10us": hist.tolist(),
        })
        print(json.dumps({k2: v for k2, v in rec[-1].items() if k2 != "end_hist_10us"}), flush=True)
    with open(out_path, "w") as f:
        json.dump({"workload": "config 2: 1M rules x 24 h UTC, synchronous cg_expand_device, diagnostic build "
                               "with per-wave stamps (CG_WRITE_STAMPS)", "launches": rec}, f, indent=1)


if __name__ == "__main__":
    main()
