"""Which HIP / HSA / RCCL copies a process maps, in either import order, and whether the
library's RCCL communicator and torch's device work side by side (GPU diagnostic)."""
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def libs():
    out = set()
    for line in open("/proc/self/maps"):
        m = re.search(r"(/\S*(amdhip64|hsa-runtime|rccl)\S*)", line)
        if m:
            out.add(m.group(1))
    return sorted(out)


order = sys.argv[1]
if order == "torch_first":
    import torch
    torch.zeros(1, device="cuda")
elif order == "torch_lazy":  # imported, CUDA not initialised (pytest collection)
    import torch  # noqa: F401
from mythril_amd import native  # noqa: E402

ctx = native.Context(0)
print("after ctx", libs(), flush=True)
ctx.comm_init(native.comm_unique_id(), 0, 1)
print("after comm_init", libs(), flush=True)
import torch  # noqa: E402

fh = torch.zeros(4, dtype=torch.int64, device="cuda")
hc = torch.ones(4, dtype=torch.int64, device="cuda")
ctx.comm_allreduce(fh.data_ptr(), hc.data_ptr(), 4)
ctx.synchronize()
print("allreduce", fh.cpu().numpy(), hc.cpu().numpy(), flush=True)
ctx.comm_destroy()
ctx.close()
print("ok", flush=True)
