"""Host->device / device->host copy bandwidth on the GPU box: pageable, torch-pinned and
hipHostRegister'ed (dmx_host_register) numpy buffers, the three ways dmx_run's uploads can be
sourced.  python tools/microbench/h2d_bw.py"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))
from dmx import lib  # noqa: E402

GB = 1 << 30
dev = torch.empty(GB, dtype=torch.uint8, device="cuda")
hip = ctypes.CDLL("libamdhip64.so")


def bw(src_ptr, n, kind):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        if kind == "h2d":
            rc = hip.hipMemcpy(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(src_ptr),
                               ctypes.c_size_t(n), 1)
        else:
            rc = hip.hipMemcpy(ctypes.c_void_p(src_ptr), ctypes.c_void_p(dev.data_ptr()),
                               ctypes.c_size_t(n), 2)
        assert rc == 0, rc
    torch.cuda.synchronize()
    return 3 * n / (time.perf_counter() - t) / 1e9


page = np.ones(GB, dtype=np.uint8)
pin = torch.ones(GB, dtype=torch.uint8).pin_memory()
reg = np.ones(GB, dtype=np.uint8)
ok = lib.host_register([reg])
for kind in ("h2d", "d2h"):
    print(f"{kind}: pageable {bw(page.ctypes.data, GB, kind):.1f} GB/s  "
          f"hipHostMalloc(torch pin) {bw(pin.data_ptr(), GB, kind):.1f} GB/s  "
          f"hipHostRegister {bw(reg.ctypes.data, GB, kind):.1f} GB/s (registered: {len(ok)})")
