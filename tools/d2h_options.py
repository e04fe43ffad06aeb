"""D2H options for the host-pointer entry points (tool): pageable hipMemcpy (today), the
destination registered with hipHostRegister for the copy, and a pinned staging buffer plus a
host memcpy (1 and 8 threads); destinations pre-faulted (warm) or fresh (cold)."""
import ctypes, json, mmap, sys, time
from concurrent.futures import ThreadPoolExecutor
import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
D2H = 2
torch.cuda.init()
pool = ThreadPoolExecutor(8)
res = {}
for mib in (4, 16, 28, 64):
    n = mib << 20
    dev = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    pin = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(pin), n, 0) == 0
    pin_np = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(pin.value))
    row = {}
    for temp in ("warm", "cold"):
        small_pages = "--small-pages" in sys.argv   # 4 KiB pages, as V8's buffers (numpy: huge pages)
        def dst():
            if small_pages:
                m = mmap.mmap(-1, n)
                m.madvise(mmap.MADV_NOHUGEPAGE)
                a = np.frombuffer(m, dtype=np.uint8)
                if temp == "warm":
                    a[::4096] = 1
                return a
            return np.zeros(n, dtype=np.uint8) if temp == "warm" else np.empty(n, dtype=np.uint8)
        def timeit(fn, reps=5):
            ts = []
            for r in range(reps + 1):
                d = dst()
                t0 = time.perf_counter(); fn(d); t1 = time.perf_counter()
                if r: ts.append((t1 - t0) * 1e3)
            return round(float(np.median(ts)), 3)
        def pageable(d):
            assert hip.hipMemcpy(d.ctypes.data, dev.data_ptr(), n, D2H) == 0
        def registered(d):
            assert hip.hipHostRegister(d.ctypes.data, n, 0) == 0
            assert hip.hipMemcpy(d.ctypes.data, dev.data_ptr(), n, D2H) == 0
            assert hip.hipHostUnregister(d.ctypes.data) == 0
        def staged1(d):
            assert hip.hipMemcpy(pin.value, dev.data_ptr(), n, D2H) == 0
            np.copyto(d, pin_np)
        def staged8(d):
            assert hip.hipMemcpy(pin.value, dev.data_ptr(), n, D2H) == 0
            k = n // 8
            list(pool.map(lambda i: np.copyto(d[i * k:(i + 1) * k], pin_np[i * k:(i + 1) * k]), range(8)))
        libc = ctypes.CDLL(None, use_errno=True)
        libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        def pageable_thp(d):   # the 2 MiB-aligned interior advised for huge pages, then the copy
            a0 = (d.ctypes.data + (2 << 20) - 1) & ~((2 << 20) - 1)
            a1 = (d.ctypes.data + n) & ~((2 << 20) - 1)
            if a1 > a0:
                libc.madvise(a0, a1 - a0, 14)   # MADV_HUGEPAGE
            assert hip.hipMemcpy(d.ctypes.data, dev.data_ptr(), n, D2H) == 0
        for name, fn in (("pageable", pageable), ("pageable_thp", pageable_thp), ("registered", registered),
                         ("staged_1t", staged1), ("staged_8t", staged8)):
            row[f"{name}_{temp}_ms"] = timeit(fn)
    d = np.empty(n, dtype=np.uint8); registered(d)   # (the check: numpy memory)
    assert np.array_equal(d, dev.cpu().numpy())
    row["pinned_only_ms"] = None
    ts = []
    for r in range(6):
        t0 = time.perf_counter(); hip.hipMemcpy(pin.value, dev.data_ptr(), n, D2H); t1 = time.perf_counter()
        if r: ts.append((t1 - t0) * 1e3)
    row["pinned_only_ms"] = round(float(np.median(ts)), 3)
    res[mib] = row
    print(mib, "MiB", row, flush=True)
print(json.dumps(res))
