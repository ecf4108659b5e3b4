// dcte_norm.h -- launchers of the energy-map -> u8 kernels (dcte_norm.hip).
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

#include "dcte_normkey.h"

namespace dcte {

// keys: 2 device uints of scratch; minmax: 2 device floats {min, max}
hipError_t launch_minmax(const float* e, long long n, unsigned* keys, float* minmax, hipStream_t s);
hipError_t launch_to_u8(const float* e, long long n, const float* minmax, int mode, int channels,
                        uint8_t* out, hipStream_t s);

// u8 frame (rows x cols x bpp) -> its transpose (cols x rows x bpp)
hipError_t launch_transpose_u8(const uint8_t* src, long long src_pitch, int rows, int cols, int bpp,
                               uint8_t* dst, long long dst_pitch, hipStream_t s);

// bytes from device memory to page-locked host memory mapped into the device
// (host_dev = hipHostGetDevicePointer of the host buffer) by a kernel: the
// GPU's own stores over PCIe, no SDMA engine.  An SDMA upload and a
// kernel-driven download run at the same time (16384^2 frame up + map down:
// 21.3 ms), where two SDMA copies in opposite directions were serialised by
// the runtime on some runs (32.9 ms) -- tools/zc_probe.py,
// profiles/r06/zc_probe.jsonl.  src and host_dev must be 4-byte aligned.
hipError_t launch_copy_to_host(const void* src, void* host_dev, size_t bytes, hipStream_t s);

}  // namespace dcte
