"""Probe: does the process exit cleanly after the library's RCCL calls, and
does it hold one RCCL copy?  python3 tools/probe_comm_exit.py <mode>:
  uid          the library's unique id only (no torch)
  comm         a world-1 communicator and one all-gather (no torch)
  torch_comm   torch imported first, then the communicator
  comm_torch   the communicator first, torch imported and used afterwards
Prints "rccl copies K" (distinct librccl files mapped) and "done <mode>"."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1]
if mode == "torch_comm":
    import torch  # noqa: F401
from cronsun_amd.engine import Comm, Engine  # noqa: E402


def rccl_copies():
    paths = set()
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()[-1]
            if os.path.basename(p).startswith("librccl.so"):
                paths.add(os.path.realpath(p))
    return sorted(paths)


uid = Comm.unique_id()
if mode != "uid":
    eng = Engine(0)
    c = Comm(eng, 1, 0, uid)
    print(c.allgather_i64([7]))
    if mode == "comm_torch":
        import torch  # noqa: F401,F811
        torch.zeros(1, device="cuda")
        print(c.allgather_i64([8]))  # still usable: the same RCCL file
    c.free()
    eng.close()
cp = rccl_copies()
print("rccl copies", len(cp), cp)
print("done", mode, flush=True)
