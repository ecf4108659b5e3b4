# diagnostic (r05): copies between hipHostRegister'ed pageable memory and the
# device -- 1-D and 2-D, each direction, and both directions at once -- before
# and after a large torch device allocation is freed (the host path page-locks
# the caller's buffers per call this way and overlaps chunked 2-D uploads with
# 1-D downloads on two streams)
import sys, time, ctypes
sys.path.insert(0, "dct-carver_amd")
import numpy as np, torch
from dctenergy import synth
S = 16384
px = np.ones((S, S, 3), np.uint8)
out = np.ones((S, S), np.float32)
hip = ctypes.CDLL("libamdhip64.so.7")
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipHostRegister.argtypes = [vp, sz, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [vp]
hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
hip.hipMemcpy2DAsync.argtypes = [vp, sz, vp, sz, sz, sz, ctypes.c_int, vp]
hip.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
hip.hipStreamSynchronize.argtypes = [vp]
d = torch.empty((S, S, 3), dtype=torch.uint8, device="cuda")
do = torch.empty((S, S), dtype=torch.float32, device="cuda")
s1, s2 = vp(), vp()
hip.hipStreamCreate(ctypes.byref(s1)); hip.hipStreamCreate(ctypes.byref(s2))
def run():
    assert hip.hipHostRegister(px.ctypes.data, px.nbytes, 0) == 0
    assert hip.hipHostRegister(out.ctypes.data, out.nbytes, 0) == 0
    r = {}
    def t(name, f):
        t0 = time.perf_counter(); f(); hip.hipStreamSynchronize(s1); hip.hipStreamSynchronize(s2)
        r[name] = round((time.perf_counter() - t0) * 1e3, 2)
    t("h2d_1d", lambda: hip.hipMemcpyAsync(d.data_ptr(), px.ctypes.data, px.nbytes, 1, s1))
    t("d2h_1d", lambda: hip.hipMemcpyAsync(out.ctypes.data, do.data_ptr(), out.nbytes, 2, s2))
    t("h2d_2d", lambda: hip.hipMemcpy2DAsync(d.data_ptr(), S * 3, px.ctypes.data, S * 3, S * 3, S, 1, s1))
    def both():
        for c in range(16):
            r0 = c * S // 16
            hip.hipMemcpy2DAsync(d.data_ptr() + r0 * S * 3, S * 3, px.ctypes.data + r0 * S * 3, S * 3, S * 3, S // 16, 1, s1)
            hip.hipMemcpyAsync(out.ctypes.data + r0 * S * 4, do.data_ptr() + r0 * S * 4, S * S // 16 * 4, 2, s2)
    t("both_chunked", both)
    hip.hipHostUnregister(px.ctypes.data); hip.hipHostUnregister(out.ctypes.data)
    return r
run()
print("before", run(), flush=True)
fr = synth.natural_rows(0, 8192, 8192, 3, seed=0, device="cuda"); del fr
torch.cuda.empty_cache()
print("after ", run(), flush=True)
