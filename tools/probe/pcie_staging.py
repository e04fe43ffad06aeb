"""PCIe staging options for host-buffer calls (the N-API path): 256 MiB device -> host and
host -> device through pageable memory (what hipMemcpy does with a JS ArrayBuffer), into a
pinned bounce buffer, the pinned -> pageable memcpy alone (1 and 8 threads), and the cost
of registering (pinning) the caller's pageable buffer for the call."""
import ctypes
import json
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

N = 256 << 20
dev = torch.empty(N, dtype=torch.uint8, device="cuda").fill_(7)
page = np.zeros(N, dtype=np.uint8)
page_t = torch.from_numpy(page)
pin = torch.empty(N, dtype=torch.uint8, pin_memory=True)
hip = ctypes.CDLL("libamdhip64.so")
res = {}


def t(name, fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    s = sorted(ts)[len(ts) // 2]
    res[name] = {"ms": round(s * 1e3, 2), "GBps": round(N / s / 1e9, 2)}
    print(name, res[name], flush=True)


t("d2h_pageable", lambda: page_t.copy_(dev))
t("d2h_pinned", lambda: pin.copy_(dev))
t("h2d_pageable", lambda: dev.copy_(page_t))
t("h2d_pinned", lambda: dev.copy_(pin))
pin_np = pin.numpy()
t("memcpy_pinned_to_pageable_1t", lambda: np.copyto(page, pin_np))
pool = ThreadPoolExecutor(8)


def par_copy(k=8):
    step = N // k
    list(pool.map(lambda i: np.copyto(page[i * step:(i + 1) * step], pin_np[i * step:(i + 1) * step]), range(k)))


t("memcpy_pinned_to_pageable_8t", par_copy)


def reg_cycle():
    p = page.ctypes.data
    assert hip.hipHostRegister(ctypes.c_void_p(p), ctypes.c_size_t(N), 0) == 0
    assert hip.hipHostUnregister(ctypes.c_void_p(p)) == 0


t("host_register_unregister", reg_cycle)


def reg_d2h():
    p = page.ctypes.data
    assert hip.hipHostRegister(ctypes.c_void_p(p), ctypes.c_size_t(N), 0) == 0
    page_t.copy_(dev)
    torch.cuda.synchronize()
    assert hip.hipHostUnregister(ctypes.c_void_p(p)) == 0


t("register_d2h_unregister", reg_d2h)
print(json.dumps(res))
