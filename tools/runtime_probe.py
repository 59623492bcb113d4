"""Which HIP runtime(s) end up in a process, by load order (diagnostic)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1]


def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l})


def create():
    from replication_erasurecoding_object_store_amd import _lib
    h = ctypes.c_void_p()
    rc = _lib.lib().rs_create(4, 2, 0, 0, ctypes.byref(h))
    return rc


if mode == "ours_first":
    from replication_erasurecoding_object_store_amd import _lib
    _lib.lib()
    import torch
    print("torch avail", torch.cuda.is_available())
    print("rc", create())
elif mode == "ours_create_first":
    print("rc", create())
    import torch
    print("torch avail", torch.cuda.is_available())
    x = torch.zeros(10, device="cuda")
    print("torch ok", float(x.sum()))
elif mode == "torch_first":
    import torch
    print("torch avail", torch.cuda.is_available())
    print("rc", create())
print(mode, maps())
