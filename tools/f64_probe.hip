// f64_probe.hip -- issue rate of the fp64 VALU ops the exact map kernel
// (dcte_exact.hip) is built from, on gfx950.
//
// The exact map recomputes the reference's fp64 arithmetic (ddct8x8s /
// ddct16x16s, src/fft2d/shrtdct.c) for every pixel: ~420 fp64 adds, multiplies
// and maxima per pixel at N = 8.  Its floor is set by how many fp64 lane-ops
// a SIMD issues per clock, and whether v_max_f64 (the last-maximum scan,
// src/dct.c:100-108) costs as much as an add.  Each kernel runs K independent
// chains per lane (enough to cover the dependent latency) for ITERS
// iterations at 1, 2, 3 and 4 waves per SIMD over every CU; JSON lines:
//   {"op": ..., "waves_per_simd": W, "ms": t, "lane_ops_per_s": ...}
// (an FMA counts as one lane-op, as the exact kernel never fuses).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/f64_probe tools/f64_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

enum Op { ADD, MUL, FMA, MAX, MAXABS, CVT, MIX_ADD_F32, F32_ADD };
static const char* kName[] = {"v_add_f64", "v_mul_f64", "v_fma_f64", "v_max_f64",
                              "v_max_f64|abs|", "v_cvt_f32_f64", "v_add_f64+v_add_f32",
                              "v_add_f32"};
static const int kLaneOps[] = {1, 1, 1, 1, 1, 1, 2, 1};

constexpr int K = 8;       // independent chains per lane
constexpr int INNER = 16;  // unrolled steps per loop iteration

template <int OP>
__global__ __launch_bounds__(256) void chains(double* out, int iters, double s)
{
    const int l = threadIdx.x;
    double x[K];
    float f[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
        x[i] = s * (l + i);
        f[i] = (float)(s * (l - i));
    }
    const double a = 0.999, b = 1e-3;
    const float bf = 1e-3f;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int j = 0; j < INNER; j++) {
            double& r = x[j % K];
            float& q = f[j % K];
            if (OP == ADD) asm volatile("v_add_f64 %0, %0, %1" : "+v"(r) : "v"(b));
            if (OP == MUL) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r) : "v"(a));
            if (OP == FMA) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(r) : "v"(a), "v"(b));
            if (OP == MAX) asm volatile("v_max_f64 %0, %0, %1" : "+v"(r) : "v"(b));
            if (OP == MAXABS) asm volatile("v_max_f64 %0, |%0|, |%1|" : "+v"(r) : "v"(b));
            if (OP == CVT) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(q) : "v"(r));
            if (OP == MIX_ADD_F32) {
                asm volatile("v_add_f64 %0, %0, %1" : "+v"(r) : "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[(j + 1) % K]) : "v"(bf));
            }
            if (OP == F32_ADD) asm volatile("v_add_f32 %0, %0, %1" : "+v"(q) : "v"(bf));
        }
    }
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < K; i++) acc += x[i] + (double)f[i];
    out[blockIdx.x * blockDim.x + l] = acc;
}

template <int OP>
static void run(double* d, int cus, int waves_per_simd, int iters)
{
    const int blocks = cus * waves_per_simd;  // 4 waves per 256-thread block, one per SIMD
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(chains<OP>, dim3(blocks), dim3(256), 0, 0, d, iters / 8, 1e-3);  // warm-up
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(chains<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 1e-3);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double lanes = double(blocks) * 256.0;
    const double steps = double(iters) * INNER;
    const double insts = (OP == MIX_ADD_F32 ? 2.0 : 1.0) * steps * lanes / 64.0;
    const double lane_ops = steps * lanes * kLaneOps[OP];
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cus\": %d, \"ms\": %.4f, "
           "\"wave_inst_per_s\": %.4e, \"lane_ops_per_s\": %.4e}\n",
           kName[OP], waves_per_simd, cus, best, insts / (best * 1e-3), lane_ops / (best * 1e-3));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main()
{
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int cus = p.multiProcessorCount;
    double* d = nullptr;
    if (hipMalloc(&d, sizeof(double) * cus * 4 * 256) != hipSuccess) return 1;
    const int iters = 4096;
    for (int w : {1, 2, 3, 4}) {
        run<ADD>(d, cus, w, iters);
        run<MUL>(d, cus, w, iters);
        run<FMA>(d, cus, w, iters);
        run<MAX>(d, cus, w, iters);
        run<MAXABS>(d, cus, w, iters);
        run<CVT>(d, cus, w, iters);
        run<MIX_ADD_F32>(d, cus, w, iters);
        run<F32_ADD>(d, cus, w, iters);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    (void)hipFree(d);
    return 0;
}
