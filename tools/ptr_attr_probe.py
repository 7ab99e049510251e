"""Probe (no kernel launch): what hipPointerGetAttributes reports for pageable host memory, pinned host
memory and device memory on this ROCm build (tree.cpp need_device_ptr relies on it)."""
import ctypes as C

import numpy as np
import torch

hip = C.CDLL("libamdhip64.so")


class Attr(C.Structure):
    _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p), ("hostPointer", C.c_void_p),
                ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]


def probe(name, ptr):
    a = Attr()
    e = hip.hipPointerGetAttributes(C.byref(a), C.c_void_p(ptr))
    hip.hipGetLastError()
    print(f"{name}: err={e} type={a.type}", flush=True)


torch.cuda.init()
x = np.zeros(1 << 20, np.uint8)
probe("numpy pageable", x.ctypes.data)
probe("torch cpu pageable", torch.zeros(1 << 20, dtype=torch.uint8).data_ptr())
probe("torch pinned", torch.zeros(1 << 20, dtype=torch.uint8).pin_memory().data_ptr())
probe("torch cuda", torch.zeros(1 << 20, dtype=torch.uint8, device="cuda").data_ptr())
