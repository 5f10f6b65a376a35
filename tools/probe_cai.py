"""Does torch-ROCm accept __cuda_array_interface__ (zero-copy views of the
engine's device buffers)?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cronsun_amd import cron
from cronsun_amd.engine import Engine
eng = Engine(0)
off, times = eng.expand([cron.Parse("0 * * * * *")], None, 1767571200, 1767571200 + 600)
_, d_times, n = eng.result_device()


class View:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False), "version": 3}


t = torch.as_tensor(View(d_times, n), device="cuda")
print("zero-copy view:", t.device, t.dtype, t.shape, t.data_ptr() == d_times, t.cpu().tolist() == times.tolist())
