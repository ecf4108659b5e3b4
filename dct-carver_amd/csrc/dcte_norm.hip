// dcte_norm.hip -- energy map -> 8-bit image.
//
// Two passes over an HBM-resident f32 map: (1) min/max, (2) normalise to u8,
// replicated over `channels` (the plug-in's output layer format).  Between
// them a multi-GPU caller all-reduces the two floats (RCCL), so every band is
// normalised with the frame's global range.
//
// Modes:
//  DCTE_NORM_PREVIEW  normalize_image, src/render.c:81-109, with
//                     DOUBLE2GUCHAR (src/render.h:6) and GIMP's ROUND:
//                     (uint8)(int)(255 * ((d - min) / (max - min)) + 0.5) in
//                     double; max == min (a division by zero in the
//                     reference, src/render.c:101) gives 0.
//  DCTE_NORM_LQR      the energy layer of display_carver_energy
//                     (src/render.c:175-202) via lqr_carver_get_energy_image:
//                     (E - min) / (max - min) in float, times 255, truncated
//                     [liblqr, unverified]; max == min gives 0.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dcte_norm.h"

namespace dcte {

__device__ __forceinline__ unsigned fkey(float f) { return norm_fkey(f); }
__device__ __forceinline__ float funkey(unsigned k) { return norm_funkey(k); }

// keys[0] = min key, keys[1] = max key; caller initialises to (~0u, 0u)
__global__ __launch_bounds__(256) void dcte_minmax(const float* __restrict__ e, long long n,
                                                   unsigned* keys)
{
    unsigned kmin = 0xffffffffu, kmax = 0u;
    const long long stride = (long long)gridDim.x * blockDim.x * 4;
    for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
        if (i + 3 < n) {
            float4 v = *reinterpret_cast<const float4*>(e + i);
            unsigned a = fkey(v.x), b = fkey(v.y), c = fkey(v.z), d = fkey(v.w);
            kmin = min(kmin, min(min(a, b), min(c, d)));
            kmax = max(kmax, max(max(a, b), max(c, d)));
        } else {
            for (long long j = i; j < n; j++) {
                unsigned a = fkey(e[j]);
                kmin = min(kmin, a);
                kmax = max(kmax, a);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        kmin = min(kmin, (unsigned)__shfl_xor((int)kmin, o));
        kmax = max(kmax, (unsigned)__shfl_xor((int)kmax, o));
    }
    __shared__ unsigned smin[4], smax[4];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        smin[wv] = kmin;
        smax[wv] = kmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 4; i++) {
            kmin = min(kmin, smin[i]);
            kmax = max(kmax, smax[i]);
        }
        atomicMin(&keys[0], kmin);
        atomicMax(&keys[1], kmax);
    }
}

__global__ void dcte_keys_to_floats(const unsigned* keys, float* minmax)
{
    minmax[0] = funkey(keys[0]);
    minmax[1] = funkey(keys[1]);
}

__global__ __launch_bounds__(256) void dcte_to_u8(const float* __restrict__ e, long long n,
                                                  const float* minmax, int mode, int channels,
                                                  uint8_t* __restrict__ out)
{
    const float mn = minmax[0], mx = minmax[1];
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint8_t v = norm_one(e[i], mn, mx, mode);
        for (int c = 0; c < channels; c++) out[i * channels + c] = v;
    }
}

static int grid_for(long long n)
{
    long long g = (n + 1023) / 1024;
    return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

hipError_t launch_minmax(const float* e, long long n, unsigned* keys, float* minmax, hipStream_t s)
{
    hipError_t err = hipMemsetAsync(keys, 0xff, sizeof(unsigned), s);
    if (err == hipSuccess) err = hipMemsetAsync(keys + 1, 0, sizeof(unsigned), s);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(dcte_minmax, dim3(grid_for(n)), dim3(256), 0, s, e, n, keys);
    hipLaunchKernelGGL(dcte_keys_to_floats, dim3(1), dim3(1), 0, s, keys, minmax);
    return hipGetLastError();
}

hipError_t launch_to_u8(const float* e, long long n, const float* minmax, int mode, int channels,
                        uint8_t* out, hipStream_t s)
{
    hipLaunchKernelGGL(dcte_to_u8, dim3(grid_for(n)), dim3(256), 0, s, e, n, minmax, mode,
                       channels, out);
    return hipGetLastError();
}

}  // namespace dcte

namespace dcte {

// ------------------------------------------------------------------ transpose
// u8 interleaved frame (rows x cols x bpp, pitch src_pitch bytes) ->
// its transpose (cols x rows x bpp, pitch dst_pitch), through 64x64 LDS tiles.
template <int BPP>
__global__ __launch_bounds__(256) void dcte_transpose_u8(const uint8_t* __restrict__ src,
                                                        long long src_pitch, int rows, int cols,
                                                        uint8_t* __restrict__ dst,
                                                        long long dst_pitch)
{
    __shared__ uint8_t tile[64][64 * BPP + 4];
    const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
    for (int i = threadIdx.x; i < 64 * 64 * BPP; i += 256) {
        const int rr = i / (64 * BPP), cb = i % (64 * BPP);
        const int r = r0 + rr, cbyte = c0 * BPP + cb;
        if (r < rows && cbyte < cols * BPP) tile[rr][cb] = src[(long long)r * src_pitch + cbyte];
    }
    __syncthreads();
    // dst row = source column c0 + cc, dst column = source row r0 + rr
    for (int i = threadIdx.x; i < 64 * 64 * BPP; i += 256) {
        const int cc = i / (64 * BPP), rb = i % (64 * BPP);
        const int rr = rb / BPP, ch = rb % BPP;
        const int c = c0 + cc, r = r0 + rr;
        if (c < cols && r < rows) dst[(long long)c * dst_pitch + (long long)r * BPP + ch] = tile[rr][cc * BPP + ch];
    }
}

// 16-byte vectors while both sides are 16-byte aligned (the common case: a
// host array and a 256-byte aligned device buffer at the same offset mod 16),
// dwords otherwise; grid-stride, a few workgroups (the copy is PCIe-bound:
// 32 .. 1024 blocks all took 19.7-20.0 ms for 1 GiB, tools/zc_probe.py)
__global__ __launch_bounds__(256) void dcte_copy_to_host(const uint8_t* __restrict__ src,
                                                          uint8_t* __restrict__ dst, size_t bytes)
{
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15u) == 0) {
        const size_t n16 = bytes / 16;
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (size_t i = t; i < n16; i += stride) d4[i] = s4[i];
        for (size_t i = n16 * 4 + t; i < bytes / 4; i += stride)
            reinterpret_cast<uint32_t*>(dst)[i] = reinterpret_cast<const uint32_t*>(src)[i];
    } else {
        for (size_t i = t; i < bytes / 4; i += stride)
            reinterpret_cast<uint32_t*>(dst)[i] = reinterpret_cast<const uint32_t*>(src)[i];
    }
    for (size_t i = bytes / 4 * 4 + t; i < bytes; i += stride) dst[i] = src[i];
}

hipError_t launch_copy_to_host(const void* src, void* host_dev, size_t bytes, hipStream_t s)
{
    if (bytes == 0) return hipSuccess;
    if ((((uintptr_t)src | (uintptr_t)host_dev) & 3u) != 0) return hipErrorInvalidValue;
    const size_t want = (bytes + 256 * 16 * 8 - 1) / (256 * 16 * 8);   // >= 8 vectors per thread
    const unsigned blocks = (unsigned)(want < 128 ? (want < 1 ? 1 : want) : 128);
    hipLaunchKernelGGL(dcte_copy_to_host, dim3(blocks), dim3(256), 0, s,
                       static_cast<const uint8_t*>(src), static_cast<uint8_t*>(host_dev), bytes);
    return hipGetLastError();
}

hipError_t launch_transpose_u8(const uint8_t* src, long long src_pitch, int rows, int cols, int bpp,
                               uint8_t* dst, long long dst_pitch, hipStream_t s)
{
    dim3 grid((cols + 63) / 64, (rows + 63) / 64);
    switch (bpp) {
    case 1: hipLaunchKernelGGL(dcte_transpose_u8<1>, grid, dim3(256), 0, s, src, src_pitch, rows, cols, dst, dst_pitch); break;
    case 3: hipLaunchKernelGGL(dcte_transpose_u8<3>, grid, dim3(256), 0, s, src, src_pitch, rows, cols, dst, dst_pitch); break;
    case 4: hipLaunchKernelGGL(dcte_transpose_u8<4>, grid, dim3(256), 0, s, src, src_pitch, rows, cols, dst, dst_pitch); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace dcte
