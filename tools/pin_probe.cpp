// pin_probe.cpp -- how hipHostRegister treats a range that does not start or
// end on a page, and what a copy to a neighbouring (unregistered) buffer that
// shares its last page does.  Decides how HostPin (dcte_capi.cpp) registers
// caller buffers.  hipcc -O2 tools/pin_probe.cpp -o /tmp/pin_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>

static const char* e(hipError_t r) { return r == hipSuccess ? "ok" : hipGetErrorString(r); }

int main()
{
    const size_t A = 1567000, B = 600000;   // px then out, packed in one allocation
    char* big = (char*)aligned_alloc(4096, 4 << 20);
    char* d = nullptr;
    (void)hipMalloc(&d, 4 << 20);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    for (int mode = 0; mode < 3; mode++) {
        char* px = big + 100;                 // unaligned start
        char* out = px + A;                   // shares px's last page
        void* reg = nullptr;
        size_t len = 0;
        if (mode == 0) { reg = px; len = A; }                                  // exact range
        if (mode == 1) {                                                       // page-rounded
            uintptr_t a = (uintptr_t)px & ~(uintptr_t)4095, b = ((uintptr_t)px + A + 4095) & ~(uintptr_t)4095;
            reg = (void*)a; len = b - a;
        }
        if (mode == 2) {                                                       // whole pages inside
            uintptr_t a = ((uintptr_t)px + 4095) & ~(uintptr_t)4095, b = ((uintptr_t)px + A) & ~(uintptr_t)4095;
            reg = (void*)a; len = b - a;
        }
        hipError_t r = hipHostRegister(reg, len, hipHostRegisterDefault);
        printf("mode %d register(%p, %zu): %s\n", mode, reg, len, e(r));
        if (r != hipSuccess) { (void)hipGetLastError(); continue; }
        hipError_t c1 = hipMemcpyAsync(out, d, B, hipMemcpyDeviceToHost, s);
        hipError_t c1s = hipStreamSynchronize(s);
        hipError_t c2 = hipMemcpyAsync(px, d, A, hipMemcpyDeviceToHost, s);
        hipError_t c2s = hipStreamSynchronize(s);
        hipError_t c3 = hipMemcpyAsync(px + A - 5000, d, 5000, hipMemcpyDeviceToHost, s);
        hipError_t c3s = hipStreamSynchronize(s);
        hipError_t c4 = hipMemcpyAsync(big, d, 200, hipMemcpyDeviceToHost, s);   // head page neighbour
        hipError_t c4s = hipStreamSynchronize(s);
        // a second registration on the out buffer (shares a page with the first)
        hipError_t r2 = hipHostRegister(out, B, hipHostRegisterDefault);
        if (r2 != hipSuccess) (void)hipGetLastError();
        hipError_t c5 = hipMemcpyAsync(out, d, B, hipMemcpyDeviceToHost, s);
        hipError_t c5s = hipStreamSynchronize(s);
        printf("  neighbour out: %s/%s  own: %s/%s  own tail: %s/%s  head neighbour: %s/%s  "
               "second register: %s  out after: %s/%s\n",
               e(c1), e(c1s), e(c2), e(c2s), e(c3), e(c3s), e(c4), e(c4s), e(r2), e(c5), e(c5s));
        (void)hipGetLastError();
        if (r2 == hipSuccess) (void)hipHostUnregister(out);
        printf("  unregister: %s\n", e(hipHostUnregister(reg)));
        (void)hipGetLastError();
    }
    return 0;
}
