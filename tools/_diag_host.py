# diagnostic (r05): copies from hipHostRegister'ed pageable memory before and
# after a large torch device allocation is freed (the host path page-locks the
# caller's buffers per call this way); torch's own hipHostMalloc copies alongside
import sys, time, ctypes
sys.path.insert(0, "dct-carver_amd")
import numpy as np, torch
from dctenergy import synth
S = 16384
px = np.ones((S, S, 3), np.uint8)
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipDeviceSynchronize.argtypes = []
d = torch.empty((S, S, 3), dtype=torch.uint8, device="cuda")
pin = torch.empty((S, S, 3), dtype=torch.uint8, pin_memory=True)
def reg_copy():
    t0 = time.perf_counter()
    assert hip.hipHostRegister(px.ctypes.data, px.nbytes, 0) == 0
    t1 = time.perf_counter()
    assert hip.hipMemcpyAsync(d.data_ptr(), px.ctypes.data, px.nbytes, 1, None) == 0
    hip.hipDeviceSynchronize()
    t2 = time.perf_counter()
    hip.hipHostUnregister(px.ctypes.data)
    return round((t1 - t0) * 1e3, 2), round((t2 - t1) * 1e3, 2)
def torch_copy():
    t0 = time.perf_counter(); d.copy_(pin); torch.cuda.synchronize(); return round((time.perf_counter() - t0) * 1e3, 2)
reg_copy(); torch_copy()
print("before: register ms, H2D ms", reg_copy(), reg_copy(), "torch pinned", torch_copy(), flush=True)
fr = synth.natural_rows(0, 8192, 8192, 3, seed=0, device="cuda"); del fr
torch.cuda.empty_cache()
print("after synth 8192^2: register ms, H2D ms", reg_copy(), reg_copy(), "torch pinned", torch_copy(), flush=True)
