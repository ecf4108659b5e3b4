"""PROBE: kernel-driven host<->device copies vs. SDMA.

The library's host path overlaps the frame's H2D with the map's D2H on two
streams; on some runs the two SDMA copies serialise (38 ms instead of 22.4 at
16384^2, tools/host_numa.py).  This times, for the 16384^2 frame / map bytes:
SDMA H2D and D2H alone and together, a copy KERNEL writing the map into
page-locked host memory (and reading the frame from it) alone, and the kernel
D2H beside an SDMA H2D.  One JSON line per case.

    python tools/zc_probe.py
"""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tools", "bin", "zc_probe.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(ROOT, "tools", "zc_probe.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared",
                        "-o", SO, src], check=True)


def main():
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return
    import numpy as np
    import torch
    L = ctypes.CDLL(SO)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.zc_copy.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    L.zc_register.argtypes = [vp, sz, ctypes.POINTER(vp)]
    L.zc_unregister.argtypes = [vp]
    S = 16384
    px = np.full((S, S, 3), 7, np.uint8)
    out = np.zeros((S, S), np.float32)
    d_px = torch.empty((S, S, 3), dtype=torch.uint8, device="cuda")
    d_out = torch.full((S, S), 1.5, dtype=torch.float32, device="cuda")
    hp, ho = vp(), vp()
    assert L.zc_register(px.ctypes.data, px.nbytes, ctypes.byref(hp)) == 0
    assert L.zc_register(out.ctypes.data, out.nbytes, ctypes.byref(ho)) == 0
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]

    def sdma_h2d():
        hip.hipMemcpyAsync(d_px.data_ptr(), px.ctypes.data, px.nbytes, 1, s1.cuda_stream)

    def sdma_d2h():
        hip.hipMemcpyAsync(out.ctypes.data, d_out.data_ptr(), out.nbytes, 2, s2.cuda_stream)

    def timed(name, fns, iters=3, **kw):
        ts = []
        for _ in range(iters + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for f in fns:
                f()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        r = {"case": name, "ms": round(min(ts[1:]), 2)}
        r.update(kw)
        print(json.dumps(r), flush=True)

    timed("sdma h2d", [sdma_h2d])
    timed("sdma d2h", [sdma_d2h])
    timed("sdma h2d + sdma d2h (two streams)", [sdma_h2d, sdma_d2h])
    for blocks in (32, 64, 128, 256, 512, 1024):
        kd2h = lambda: L.zc_copy(d_out.data_ptr(), ho, out.nbytes, blocks, s2.cuda_stream)
        timed("kernel d2h", [kd2h], blocks=blocks)
        timed("sdma h2d + kernel d2h", [sdma_h2d, kd2h], blocks=blocks)
    ok = bool((out == 1.5).all())
    for blocks in (64, 256, 1024):
        kh2d = lambda: L.zc_copy(hp, d_px.data_ptr(), px.nbytes, blocks, s1.cuda_stream)
        timed("kernel h2d", [kh2d], blocks=blocks)
        timed("kernel h2d + sdma d2h", [kh2d, sdma_d2h], blocks=blocks)
    ok = ok and bool((d_px == 7).all())
    print(json.dumps({"copies_correct": ok}), flush=True)
    L.zc_unregister(px.ctypes.data)
    L.zc_unregister(out.ctypes.data)


if __name__ == "__main__":
    main()
