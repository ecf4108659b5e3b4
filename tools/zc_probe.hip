// zc_probe.hip -- PROBE (not product): copies between HBM and page-locked
// host memory done by a kernel (the GPU's own loads / stores over PCIe)
// instead of the SDMA engines, alone and beside an SDMA copy in the other
// direction.  Built by tools/zc_probe.py into tools/bin/.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) copy16(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                              size_t n16)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n16; i += stride) {
        dst[i] = src[i];
    }
}

extern "C" int zc_copy(const void* src, void* dst, size_t bytes, int blocks, void* stream)
{
    hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)src, (uint4*)dst, bytes / 16);
    return (int)hipGetLastError();
}

extern "C" int zc_register(void* p, size_t bytes, void** dev)
{
    hipError_t e = hipHostRegister(p, bytes, hipHostRegisterMapped);
    if (e != hipSuccess) return (int)e;
    return (int)hipHostGetDevicePointer(dev, p, 0);
}

extern "C" int zc_unregister(void* p) { return (int)hipHostUnregister(p); }
