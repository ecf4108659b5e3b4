// Semantics probe of the gfx950 row-swap permutes used by the N = 16 dense
// refinement: prints, per lane, what v_permlane16_swap_b32 and
// v_permlane32_swap_b32 leave in (vdst, src0) when vdst = 1000 + lane and
// src0 = 2000 + lane.
//   hipcc --offload-arch=gfx950 -O2 -o tools/bin/permlane_probe tools/permlane_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned* o)
{
    const unsigned l = threadIdx.x;
    auto a = __builtin_amdgcn_permlane16_swap(1000u + l, 2000u + l, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(1000u + l, 2000u + l, false, false);
    o[l] = a[0];
    o[64 + l] = a[1];
    o[128 + l] = b[0];
    o[192 + l] = b[1];
}

int main()
{
    unsigned* d = nullptr;
    unsigned h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[4] = {"p16 vdst", "p16 src0", "p32 vdst", "p32 src0"};
    for (int k = 0; k < 4; k++) {
        printf("%s:", names[k]);
        for (int l = 0; l < 64; l += 8) printf(" [%d]=%u", l, h[64 * k + l]);
        printf(" [17]=%u [33]=%u [49]=%u\n", h[64 * k + 17], h[64 * k + 33], h[64 * k + 49]);
    }
    (void)hipFree(d);
    return 0;
}
