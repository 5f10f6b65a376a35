"""Probe: does the process exit cleanly after the library's RCCL calls?
python3 tools/probe_comm_exit.py <mode>: uid | comm | torch_comm | comm_torch"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1]
if mode == "torch_comm":
    import torch  # noqa: F401
from cronsun_amd.engine import Comm, Engine  # noqa: E402

uid = Comm.unique_id()
if mode != "uid":
    eng = Engine(0)
    c = Comm(eng, 1, 0, uid)
    print(c.allgather_i64([7]))
    c.free()
    eng.close()
if mode == "comm_torch":
    import torch  # noqa: F401,F811
    torch.zeros(1, device="cuda")
print("done", mode, flush=True)
