"""dctenergy -- Python binding of libdctenergy_hip.so (the MI355X energy-map backend).

The product is the C ABI in include/dctenergy.h; this module is a thin ctypes
view of it for tests, the bench and Python callers.  There is no CPU fallback:
if the HIP library is missing or no device is present, every entry point
raises (the reference's CPU path lives only in oracle/, as the checker).

Reference interface mirrored (avivrosenberg/dct-carver):
  * Context.energy_map     <- W*H calls of dct_pixel_energy (src/render.c:134-157)
  * carver.EnergyParameters / init_carver_from_vals / dct_pixel_energy
                           <- src/render.h:9-18, src/render.c:286-325
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "DCTE_LIB", os.path.join(os.path.dirname(_HERE), "build", "libdctenergy_hip.so"))

DCTE_OK = 0
DCTE_EINVAL = -1
DCTE_ENODEV = -2
DCTE_ENOMEM = -3
DCTE_EHIP = -4
DCTE_ERANGE = -5
DCTE_ENOTSUP = -6

DCTE_LQR = 0
DCTE_PREVIEW = 1
DCTE_OPT_TIE_TAU = 1
DCTE_OPT_PROFILE = 2
DCTE_OPT_PIN_HOST = 3
DCTE_OPT_TILE_H = 4
DCTE_OPT_DP_BANDWISE = 5
DCTE_OPT_DP_SPIN_LIMIT = 6
DCTE_OPT_TSTAMP_BUF = 7
DCTE_OPT_LEGACY_8 = 8
DCTE_OPT_FAIL_INJECT = 9
DCTE_OPT_EXACT = 10
DCTE_OPT_D2H_KERNEL = 11
DCTE_NORM_LQR = 0
DCTE_NORM_PREVIEW = 1
DCTE_CREATE_SAME_DEVICE = 1

# every symbol include/dctenergy.h declares
EXPORTS = ("dcte_abi_version", "dcte_device_count", "dcte_create", "dcte_destroy",
           "dcte_ctx_devices", "dcte_set_option", "dcte_energy_map",
           "dcte_energy_map_device", "dcte_energy_map_device2", "dcte_last_refined", "dcte_profile_read", "dcte_strerror",
           "dcte_last_error", "dcte_normalize_u8", "dcte_energy_image_u8", "dcte_minmax_device",
           "dcte_normalize_u8_device", "dcte_seam_carve_device", "dcte_energy_points",
           "dcte_energy_points_device", "dcte_seam_find_device", "dcte_seam_find",
           "dcte_carve", "dcte_energy_windows", "dcte_energy_windows_device",
           "dcte_energy_window", "dcte_normalize_u8_host", "dcte_carver_create",
           "dcte_carver_step", "dcte_carver_width", "dcte_carver_height",
           "dcte_carver_band_width", "dcte_carver_destroy", "dcte_energy_map2",
           "dcte_carver_create2")

_lib = None


def _rowstride(px):
    """Bytes between rows; numpy leaves the stride of a 1-row array arbitrary."""
    return px.strides[0] if px.shape[0] > 1 else px.shape[1] * (px.shape[2] if px.ndim == 3 else 1)


class DcteError(RuntimeError):
    def __init__(self, code, detail=""):
        self.code = code
        msg = f"dctenergy error {code}: {_strerror(code)}"
        if detail:
            msg += f" ({detail})"
        super().__init__(msg)


def _strerror(code):
    try:
        return lib().dcte_strerror(code).decode()
    except OSError:
        return "library not loaded"


def lib():
    """Load libdctenergy_hip.so (raises OSError when it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"libdctenergy_hip.so not found at {LIB_PATH}; run __graft_entry__.build()")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64
    # (soname libamdhip64.so.7, loaded by the unversioned name).  Loaded after
    # ours, it would come in as a second runtime and find no device; loaded
    # first, our NEEDED libamdhip64.so.7 binds to it.  So torch goes first
    # whenever it is installed.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    L.dcte_abi_version.restype = ctypes.c_int
    L.dcte_device_count.restype = ctypes.c_int
    L.dcte_create.restype = ctypes.c_int
    L.dcte_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_uint]
    L.dcte_destroy.restype = None
    L.dcte_destroy.argtypes = [vp]
    L.dcte_ctx_devices.restype = ctypes.c_int
    L.dcte_ctx_devices.argtypes = [vp]
    L.dcte_set_option.restype = ctypes.c_int
    L.dcte_set_option.argtypes = [vp, ctypes.c_int, ctypes.c_double]
    L.dcte_energy_map.restype = ctypes.c_int
    L.dcte_energy_map.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_size_t, ctypes.c_int, ctypes.c_float,
                                  ctypes.c_float, ctypes.c_int, ctypes.c_int, vp]
    L.dcte_energy_map2.restype = ctypes.c_int
    L.dcte_energy_map2.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_size_t, ctypes.c_int, ctypes.c_float,
                                   ctypes.c_float, ctypes.c_int, vp, vp]
    L.dcte_energy_map_device.restype = ctypes.c_int
    L.dcte_energy_map_device.argtypes = [vp, ctypes.c_int, vp, ctypes.c_longlong, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                         ctypes.c_float, ctypes.c_int, vp, ctypes.c_longlong, vp]
    L.dcte_energy_map_device2.restype = ctypes.c_int
    L.dcte_energy_map_device2.argtypes = [vp, ctypes.c_int, vp, ctypes.c_longlong, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                          vp, ctypes.c_longlong, vp]
    L.dcte_last_refined.restype = ctypes.c_longlong
    L.dcte_last_refined.argtypes = [vp]
    L.dcte_profile_read.restype = ctypes.c_int
    L.dcte_profile_read.argtypes = [vp, ctypes.POINTER(ctypes.c_longlong),
                                    ctypes.POINTER(ctypes.c_double)]
    L.dcte_normalize_u8.restype = ctypes.c_int
    L.dcte_normalize_u8.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp]
    L.dcte_energy_image_u8.restype = ctypes.c_int
    L.dcte_energy_image_u8.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_size_t, ctypes.c_int, ctypes.c_float,
                                       ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       vp]
    L.dcte_minmax_device.restype = ctypes.c_int
    L.dcte_minmax_device.argtypes = [vp, ctypes.c_int, vp, ctypes.c_longlong, vp, vp]
    L.dcte_normalize_u8_device.restype = ctypes.c_int
    L.dcte_normalize_u8_device.argtypes = [vp, ctypes.c_int, vp, ctypes.c_longlong, vp,
                                           ctypes.c_int, ctypes.c_int, vp, vp]
    i, f, ll = ctypes.c_int, ctypes.c_float, ctypes.c_longlong
    L.dcte_seam_carve_device.restype = i
    L.dcte_seam_carve_device.argtypes = [vp, i, vp, ll, i, i, i, vp, vp, ll, vp, ll, vp, ll, i, f, f,
                                         i, vp]
    L.dcte_energy_points.restype = i
    L.dcte_energy_points.argtypes = [vp, vp, i, i, i, ctypes.c_size_t, vp, i, i, f, f, i, vp]
    L.dcte_energy_points_device.restype = i
    L.dcte_energy_points_device.argtypes = [vp, i, vp, ll, i, i, i, vp, i, i, f, f, i, vp, vp]
    L.dcte_energy_windows.restype = i
    L.dcte_energy_windows.argtypes = [vp, vp, i, i, f, f, vp]
    L.dcte_energy_windows_device.restype = i
    L.dcte_energy_windows_device.argtypes = [vp, i, vp, i, i, f, f, vp, vp]
    L.dcte_seam_find_device.restype = i
    L.dcte_seam_find_device.argtypes = [vp, i, vp, ll, i, i, vp, vp]
    L.dcte_seam_find.restype = i
    L.dcte_seam_find.argtypes = [vp, vp, i, i, vp]
    L.dcte_carve.restype = i
    L.dcte_carve.argtypes = [vp, vp, i, i, i, ctypes.c_size_t, i, f, f, i, i, i, vp, vp]
    L.dcte_energy_window.restype = i
    L.dcte_energy_window.argtypes = [i, vp, f, f, vp]
    L.dcte_normalize_u8_host.restype = i
    L.dcte_normalize_u8_host.argtypes = [vp, ctypes.c_size_t, i, i, vp]
    L.dcte_carver_create.restype = i
    L.dcte_carver_create.argtypes = [vp, vp, i, i, i, ctypes.c_size_t, i, f, f, i, vp,
                                     ctypes.POINTER(vp)]
    L.dcte_carver_create2.restype = i
    L.dcte_carver_create2.argtypes = [vp, vp, i, i, i, ctypes.c_size_t, i, f, f, i, vp, vp,
                                      ctypes.POINTER(vp)]
    L.dcte_carver_step.restype = i
    L.dcte_carver_step.argtypes = [vp, vp, vp, vp, vp]
    for fn in ("dcte_carver_width", "dcte_carver_height", "dcte_carver_band_width"):
        getattr(L, fn).restype = i
        getattr(L, fn).argtypes = [vp]
    L.dcte_carver_destroy.restype = None
    L.dcte_carver_destroy.argtypes = [vp]
    L.dcte_strerror.restype = ctypes.c_char_p
    L.dcte_strerror.argtypes = [ctypes.c_int]
    L.dcte_last_error.restype = ctypes.c_char_p
    L.dcte_last_error.argtypes = [vp]
    _lib = L
    return L


def device_count():
    return lib().dcte_device_count()


# -- context-free CPU entries: no device, no context
def energy_window(win, edges=0.5, textures=0.5):
    """One N x N float64 window in the reference's data[i][j] layout (i = x
    offset) -> weighted_max_dct_correlation(dctNxN(window)) as float32
    (src/dct.c:77-110), computed on the CPU in the reference's fp64 order."""
    win = np.ascontiguousarray(win, dtype=np.float64)
    if win.ndim != 2 or win.shape[0] != win.shape[1]:
        raise ValueError("win must be N x N")
    out = ctypes.c_float()
    rc = lib().dcte_energy_window(win.shape[0], win.ctypes.data, edges, textures,
                                  ctypes.byref(out))
    if rc != DCTE_OK:
        raise DcteError(rc)
    return np.float32(out.value)


def normalize_u8_host(E, mode=DCTE_NORM_PREVIEW, channels=1):
    """Energy map -> u8 layer on the CPU (the bytes dcte_normalize_u8 gives)."""
    E = np.ascontiguousarray(E, dtype=np.float32)
    out = np.empty(E.shape + ((channels,) if channels > 1 else ()), np.uint8)
    rc = lib().dcte_normalize_u8_host(E.ctypes.data, E.size, mode, channels, out.ctypes.data)
    if rc != DCTE_OK:
        raise DcteError(rc)
    return out


class Context:
    """One dcte_ctx (a set of devices).  Not thread-safe, like the reference
    callback (src/render.c:140 shares params->data)."""

    def __init__(self, ngpus=0, tie_tau=None, same_device=False, exact=False):
        """same_device: `ngpus` logical devices that are all device 0
        (DCTE_CREATE_SAME_DEVICE) -- the multi-device host path on one GPU.
        exact: DCTE_OPT_EXACT (every pixel bit-identical to the reference)."""
        L = lib()
        h = ctypes.c_void_p()
        rc = L.dcte_create(ctypes.byref(h), ngpus,
                           DCTE_CREATE_SAME_DEVICE if same_device else 0)
        if rc != DCTE_OK:
            raise DcteError(rc)
        self._h = h
        if tie_tau is not None:
            self.set_option(DCTE_OPT_TIE_TAU, tie_tau)
        if exact:
            self.set_option(DCTE_OPT_EXACT, 1)

    # -- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            lib().dcte_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc):
        if rc != DCTE_OK:
            raise DcteError(rc, lib().dcte_last_error(self._h).decode())

    @property
    def ndevices(self):
        return lib().dcte_ctx_devices(self._h)

    @property
    def last_refined(self):
        return lib().dcte_last_refined(self._h)

    def set_option(self, opt, value):
        self._check(lib().dcte_set_option(self._h, opt, float(value)))

    def profile_read(self):
        """-> (map-kernel launches, summed device ms) since the last read."""
        n = ctypes.c_longlong()
        ms = ctypes.c_double()
        self._check(lib().dcte_profile_read(self._h, ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    # -- host entry point
    @staticmethod
    def _frame(px):
        """-> (px as a uint8 array with packed pixels, h, w, bpp, rowstride)"""
        px = np.asarray(px)
        if px.dtype != np.uint8:
            raise TypeError("px must be uint8")
        if px.ndim == 2:
            h, w = px.shape
            bpp = 1
        elif px.ndim == 3:
            h, w, bpp = px.shape
        else:
            raise ValueError("px must be HxW or HxWxC")
        if px.strides[-1] != 1 or (px.ndim == 3 and px.strides[1] != bpp):
            px = np.ascontiguousarray(px)
        return px, h, w, bpp, _rowstride(px)

    @staticmethod
    def _out(out, shape):
        if out is None:
            return np.empty(shape, np.float32)
        if out.shape != shape or out.dtype != np.float32 or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous {shape} float32 array")
        return out

    def energy_map(self, px, n=8, edges=0.5, textures=0.5, semantics=DCTE_LQR,
                   transposed=False, out=None):
        """Energy map of an HxW (grey) or HxWxC uint8 frame -> HxW float32."""
        px, h, w, bpp, rowstride = self._frame(px)
        out = self._out(out, (w, h) if transposed else (h, w))
        self._check(lib().dcte_energy_map(self._h, px.ctypes.data, w, h, bpp, rowstride, n,
                                          edges, textures, semantics, int(bool(transposed)),
                                          out.ctypes.data))
        return out

    def energy_map2(self, px, n=8, edges=0.5, textures=0.5, semantics=DCTE_LQR, out=None,
                    out_t=None, want=(True, True)):
        """Both orientations from one upload (dcte_energy_map2): -> (HxW map,
        WxH map of the transposed frame); want = which of the two to compute
        (None in its place when not)."""
        px, h, w, bpp, rowstride = self._frame(px)
        o = self._out(out, (h, w)) if want[0] else None
        ot = self._out(out_t, (w, h)) if want[1] else None
        self._check(lib().dcte_energy_map2(self._h, px.ctypes.data, w, h, bpp, rowstride, n,
                                           edges, textures, semantics,
                                           o.ctypes.data if o is not None else None,
                                           ot.ctypes.data if ot is not None else None))
        return o, ot

    # -- energy image as 8-bit grey
    def normalize_u8(self, E, mode=DCTE_NORM_PREVIEW, channels=1):
        E = np.ascontiguousarray(E, dtype=np.float32)
        out = np.empty(E.shape + ((channels,) if channels > 1 else ()), np.uint8)
        self._check(lib().dcte_normalize_u8(self._h, E.ctypes.data, E.size, mode, channels,
                                            out.ctypes.data))
        return out

    def energy_image_u8(self, px, n=8, edges=0.5, textures=0.5, mode=DCTE_NORM_LQR, channels=1,
                        semantics=DCTE_LQR, out=None):
        px = np.ascontiguousarray(px, dtype=np.uint8)
        h, w = px.shape[:2]
        bpp = 1 if px.ndim == 2 else px.shape[2]
        shape = (h, w) + ((channels,) if channels > 1 else ())
        if out is None:
            out = np.empty(shape, np.uint8)
        elif out.shape != shape or out.dtype != np.uint8 or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous uint8 array of shape {shape}")
        self._check(lib().dcte_energy_image_u8(self._h, px.ctypes.data, w, h, bpp, _rowstride(px),
                                               n, edges, textures, semantics, mode, channels,
                                               out.ctypes.data))
        return out

    def minmax_device(self, d_E, n, d_minmax, stream=0, device=0):
        self._check(lib().dcte_minmax_device(self._h, device, ctypes.c_void_p(d_E), n,
                                             ctypes.c_void_p(d_minmax), ctypes.c_void_p(stream)))

    def normalize_u8_device(self, d_E, n, d_minmax, d_out, mode=DCTE_NORM_PREVIEW, channels=1,
                            stream=0, device=0):
        self._check(lib().dcte_normalize_u8_device(self._h, device, ctypes.c_void_p(d_E), n,
                                                   ctypes.c_void_p(d_minmax), mode, channels,
                                                   ctypes.c_void_p(d_out), ctypes.c_void_p(stream)))

    # -- device entry point (HBM-resident frames; addresses as ints)
    def energy_map_device(self, d_px, rowstride, w, h, bpp, in_row0, in_rows, y0, y1, n,
                          edges, textures, d_out, out_stride, stream=0, device=0,
                          semantics=DCTE_LQR):
        self._check(lib().dcte_energy_map_device(
            self._h, device, ctypes.c_void_p(d_px), rowstride, w, h, bpp, in_row0, in_rows,
            y0, y1, n, edges, textures, semantics, ctypes.c_void_p(d_out), out_stride,
            ctypes.c_void_p(stream)))

    def energy_map_device2(self, d_px, rowstride, w, h, bpp, in_row0, in_rows, y0, y1, yb0, yb1,
                           n, edges, textures, d_out, out_stride, stream=0, device=0,
                           semantics=DCTE_LQR):
        """Rows [y0, y1) and [yb0, yb1) in one map launch (a band's two edge
        ranges); row y of either at d_out + (y - y0) * out_stride."""
        self._check(lib().dcte_energy_map_device2(
            self._h, device, ctypes.c_void_p(d_px), rowstride, w, h, bpp, in_row0, in_rows,
            y0, y1, yb0, yb1, n, edges, textures, semantics, ctypes.c_void_p(d_out), out_stride,
            ctypes.c_void_p(stream)))

    def energy_map_tensor(self, px, out, n=8, edges=0.5, textures=0.5, h=None, in_row0=0,
                          y0=None, y1=None, stream=None, device=0, semantics=DCTE_LQR):
        """torch.uint8 CUDA frame rows (HxW or HxWxC; row 0 = global row
        `in_row0` of an image of height `h`) -> rows [y0, y1) into `out`."""
        import torch  # plumbing only: device memory and the current stream
        if px.device.type != "cuda" or out.device.type != "cuda":
            raise ValueError("tensors must live on a HIP device")
        if px.dtype != torch.uint8 or out.dtype != torch.float32:
            raise TypeError("px uint8, out float32")
        rows, w = px.shape[0], px.shape[1]
        bpp = 1 if px.dim() == 2 else px.shape[2]
        if px.stride(-1) != 1 or (px.dim() == 3 and px.stride(1) != bpp):
            raise ValueError("px rows must be dense")
        if out.stride(-1) != 1:
            raise ValueError("out rows must be dense")
        h = rows if h is None else h
        y0 = in_row0 if y0 is None else y0
        y1 = in_row0 + rows if y1 is None else y1
        if stream is None:
            stream = torch.cuda.current_stream(px.device).cuda_stream
        self.energy_map_device(px.data_ptr(), px.stride(0), w, h, bpp, in_row0, rows, y0, y1,
                               n, edges, textures, out.data_ptr(), out.stride(0), stream, device,
                               semantics)
        return out

    # -- seam carving support
    def energy_points(self, px, xy, n=8, edges=0.5, textures=0.5, semantics=DCTE_LQR):
        """Energies of the listed pixels (K x 2 int array of (x, y)) of a host frame."""
        px = np.asarray(px)
        if px.dtype != np.uint8 or px.ndim not in (2, 3):
            raise TypeError("px must be an HxW or HxWxC uint8 array")
        px = np.ascontiguousarray(px)
        h, w = px.shape[:2]
        bpp = 1 if px.ndim == 2 else px.shape[2]
        xy = np.ascontiguousarray(xy, dtype=np.int32).reshape(-1, 2)
        out = np.empty(len(xy), np.float32)
        self._check(lib().dcte_energy_points(self._h, px.ctypes.data, w, h, bpp, _rowstride(px),
                                             xy.ctypes.data, len(xy), n, edges, textures,
                                             semantics, out.ctypes.data))
        return out

    def energy_points_tensor(self, px, xy, out, n=8, edges=0.5, textures=0.5, stream=None,
                             device=0, semantics=DCTE_LQR):
        """Device version: px torch.uint8 frame, xy int32 [K, 2], out float32 [K]."""
        import torch
        if px.dtype != torch.uint8 or xy.dtype != torch.int32 or out.dtype != torch.float32:
            raise TypeError("px uint8, xy int32, out float32")
        if not (xy.is_contiguous() and out.is_contiguous()):
            raise ValueError("xy and out must be contiguous")
        h, w = px.shape[0], px.shape[1]
        bpp = 1 if px.dim() == 2 else px.shape[2]
        if stream is None:
            stream = torch.cuda.current_stream(px.device).cuda_stream
        self._check(lib().dcte_energy_points_device(
            self._h, device, ctypes.c_void_p(px.data_ptr()), px.stride(0), w, h, bpp,
            ctypes.c_void_p(xy.data_ptr()), xy.shape[0], n, edges, textures, semantics,
            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream)))
        return out

    def seam_carve_tensor(self, px, seam, emap, px_out, emap_out, n=8, edges=0.5, textures=0.5,
                          stream=None, device=0, semantics=DCTE_LQR):
        """Remove seam[y] from every row of the device frame px (H x W[xC]) ->
        px_out (H x (W-1)[xC]); emap (map of px) -> emap_out (map of px_out)."""
        import torch
        if px.dtype != torch.uint8 or px_out.dtype != torch.uint8:
            raise TypeError("frames must be uint8")
        if seam.dtype != torch.int32 or not seam.is_contiguous():
            raise TypeError("seam must be a contiguous int32 tensor")
        if emap.dtype != torch.float32 or emap_out.dtype != torch.float32:
            raise TypeError("maps must be float32")
        h, w = px.shape[0], px.shape[1]
        bpp = 1 if px.dim() == 2 else px.shape[2]
        if seam.numel() != h or px_out.shape[0] != h or px_out.shape[1] != w - 1:
            raise ValueError("seam needs h entries, px_out h x (w-1)")
        if emap.shape[1] < w or emap_out.shape[1] < w - 1:
            raise ValueError("map shapes")
        if stream is None:
            stream = torch.cuda.current_stream(px.device).cuda_stream
        self._check(lib().dcte_seam_carve_device(
            self._h, device, ctypes.c_void_p(px.data_ptr()), px.stride(0), w, h, bpp,
            ctypes.c_void_p(seam.data_ptr()), ctypes.c_void_p(emap.data_ptr()), emap.stride(0),
            ctypes.c_void_p(px_out.data_ptr()), px_out.stride(0),
            ctypes.c_void_p(emap_out.data_ptr()), emap_out.stride(0), n, edges, textures,
            semantics, ctypes.c_void_p(stream)))
        return px_out, emap_out

    # -- per-window energies (SURVEY §8b dcte_energy_window, batched)
    def energy_windows(self, win, edges=0.5, textures=0.5):
        """win: K x N x N float64 windows in the reference's data[i][j]
        layout (i = x offset for the liblqr callback) -> K float32 energies,
        bit-identical to weighted_max_dct_correlation(dctNxN(window))."""
        win = np.ascontiguousarray(win, dtype=np.float64)
        if win.ndim != 3 or win.shape[1] != win.shape[2]:
            raise ValueError("win must be K x N x N")
        out = np.empty(win.shape[0], np.float32)
        self._check(lib().dcte_energy_windows(self._h, win.ctypes.data, win.shape[0], win.shape[1],
                                              edges, textures, out.ctypes.data))
        return out

    # -- device mirror of a liblqr carver (the update_emap hook)
    def carver(self, px, n=8, edges=0.5, textures=0.5, transposed=False, other=False):
        """-> (Carver, first map of the mirrored frame); other=True
        (dcte_carver_create2): -> (Carver, first map, map of the other
        orientation) from the same upload.  The carver keeps the context's
        arithmetic mode of this moment (DCTE_OPT_EXACT / DCTE_OPT_TIE_TAU)."""
        px = np.ascontiguousarray(px, dtype=np.uint8)
        h, w = px.shape[:2]
        bpp = 1 if px.ndim == 2 else px.shape[2]
        first = np.empty((w, h) if transposed else (h, w), np.float32)
        c = ctypes.c_void_p()
        if not other:
            self._check(lib().dcte_carver_create(self._h, px.ctypes.data, w, h, bpp, _rowstride(px),
                                                 n, edges, textures, int(bool(transposed)),
                                                 first.ctypes.data, ctypes.byref(c)))
            return Carver(self, c, bpp), first
        second = np.empty((h, w) if transposed else (w, h), np.float32)
        self._check(lib().dcte_carver_create2(self._h, px.ctypes.data, w, h, bpp, _rowstride(px), n,
                                              edges, textures, int(bool(transposed)),
                                              first.ctypes.data, second.ctypes.data,
                                              ctypes.byref(c)))
        return Carver(self, c, bpp), first, second

    # -- minimum-energy seam
    def seam_find(self, E):
        """Vertical seam (column per row) of an HxW float32 host energy map."""
        E = np.ascontiguousarray(E, dtype=np.float32)
        h, w = E.shape
        seam = np.empty(h, np.int32)
        self._check(lib().dcte_seam_find(self._h, E.ctypes.data, w, h, seam.ctypes.data))
        return seam

    def carve(self, px, seams, n=8, edges=0.5, textures=0.5, semantics=DCTE_LQR,
              transposed=False):
        """Remove `seams` minimum-energy seams from an HxW[xC] uint8 frame
        (vertical seams; horizontal with transposed=True) -- lqr_carver_resize's
        loop (src/render.c:377) on the device.  Returns (carved frame, seams),
        seams[k] = the pixel removed from each line by step k, in that step's frame."""
        px = np.asarray(px)
        if px.dtype != np.uint8 or px.ndim not in (2, 3):
            raise TypeError("px must be an HxW or HxWxC uint8 array")
        if px.strides[-1] != 1 or (px.ndim == 3 and px.strides[1] != px.shape[2]):
            px = np.ascontiguousarray(px)
        h, w = px.shape[:2]
        bpp = 1 if px.ndim == 2 else px.shape[2]
        W, H = (h, w) if transposed else (w, h)
        if not 0 <= seams < W:
            raise DcteError(DCTE_EINVAL, f"seams must lie in [0, {W})")
        out = np.empty(((h - seams, w) if transposed else (h, w - seams)) + px.shape[2:], np.uint8)
        cols = np.empty((seams, H), np.int32)
        self._check(lib().dcte_carve(self._h, px.ctypes.data, w, h, bpp, _rowstride(px), n, edges,
                                     textures, semantics, seams, int(bool(transposed)),
                                     out.ctypes.data, cols.ctypes.data if seams else None))
        return out, cols

    def seam_find_tensor(self, emap, seam, stream=None, device=0):
        """Device version: emap float32 [H, >=W] (row stride emap.stride(0)), seam int32 [H]."""
        import torch
        if emap.dtype != torch.float32 or seam.dtype != torch.int32 or not seam.is_contiguous():
            raise TypeError("emap float32, seam contiguous int32")
        h, w = emap.shape
        if seam.numel() != h or emap.stride(1) != 1:
            raise ValueError("seam needs h entries; map rows dense")
        if stream is None:
            stream = torch.cuda.current_stream(emap.device).cuda_stream
        self._check(lib().dcte_seam_find_device(
            self._h, device, ctypes.c_void_p(emap.data_ptr()), emap.stride(0), w, h,
            ctypes.c_void_p(seam.data_ptr()), ctypes.c_void_p(stream)))
        return seam


class Carver:
    """dcte_carver: the carver's frame and map in HBM; step() carves the seam
    liblqr's DP picks and returns (seam, band_x0, band energies, band pixels)."""

    def __init__(self, ctx, handle, bpp):
        self._ctx, self._h, self.bpp = ctx, handle, bpp

    @property
    def width(self):
        return lib().dcte_carver_width(self._h)

    @property
    def height(self):
        return lib().dcte_carver_height(self._h)

    @property
    def band_width(self):
        return lib().dcte_carver_band_width(self._h)

    def step(self):
        H, bw = self.height, self.band_width
        seam = np.empty(H, np.int32)
        x0 = np.empty(H, np.int32)
        e = np.empty((H, bw), np.float32)
        px = np.empty((H, bw, self.bpp), np.uint8)
        self._ctx._check(lib().dcte_carver_step(self._h, seam.ctypes.data, x0.ctypes.data,
                                                e.ctypes.data, px.ctypes.data))
        return seam, x0, e, px

    def close(self):
        if getattr(self, "_h", None):
            lib().dcte_carver_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["Context", "Carver", "DcteError", "lib", "device_count", "LIB_PATH", "EXPORTS",
           "energy_window", "normalize_u8_host",
           "DCTE_LQR", "DCTE_PREVIEW", "DCTE_OPT_TIE_TAU", "DCTE_OPT_EXACT", "DCTE_OPT_FAIL_INJECT", "DCTE_OPT_PROFILE", "DCTE_OPT_PIN_HOST", "DCTE_OPT_TILE_H", "DCTE_OPT_DP_BANDWISE", "DCTE_OPT_DP_SPIN_LIMIT",
           "DCTE_NORM_LQR", "DCTE_NORM_PREVIEW"]
