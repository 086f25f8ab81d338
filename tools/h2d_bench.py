"""Host-to-device copy rates on one MI355X (dev tool): ecg_dev_upload of a
numpy (pageable) array, the same bytes from HIP pinned host memory, for a few
sizes.  Usage: python tools/h2d_bench.py"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
import ecgpu  # noqa: E402

prog = ecgpu.program(ecgpu.Device(0))
hip = ctypes.CDLL(ecgpu.lib().ecg_runtime_info().decode().split("(")[1].split(")")[0])
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.argtypes = [ctypes.c_void_p]
for mb in (128, 512, 2048):
    nbytes = mb << 20
    host = np.ones(nbytes // 8, dtype=np.uint64)
    d = ecgpu.DeviceBuffer(prog, nbytes)
    d.write(host)
    t = time.perf_counter()
    for _ in range(3):
        d.write(host)
    pageable = 3 * nbytes / (time.perf_counter() - t) / 1e9
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), nbytes, 0) == 0
    ctypes.memmove(p, host.ctypes.data, nbytes)
    L = ecgpu.lib()
    L.ecg_dev_upload(prog.handle, d.ptr, p, nbytes)
    t = time.perf_counter()
    for _ in range(3):
        L.ecg_dev_upload(prog.handle, d.ptr, p, nbytes)
    pinned = 3 * nbytes / (time.perf_counter() - t) / 1e9
    hip.hipHostFree(p)
    d.free()
    print(json.dumps({"MiB": mb, "pageable_GBps": pageable, "pinned_GBps": pinned}), flush=True)
