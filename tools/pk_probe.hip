// pk_probe.hip -- does packed FP32 (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32)
// issue at a higher LANE-OP rate than the scalar forms on gfx950?
//
// The N = 8 map kernel is VALU-issue-bound: a two-columns-
// per-lane layout on packed f32 would only pay if one packed instruction does
// two lane-ops in less than twice the cycles of one scalar instruction.
// Each kernel runs K independent accumulation chains per lane (K = 8, enough
// to cover the dependent latency) for ITERS iterations, at 4 and 8 waves per
// SIMD over every CU; the result is printed as JSON lines:
//   {"op": ..., "waves_per_simd": W, "ms": t, "inst_per_s": ..., "lane_ops_per_s": ...}
// lane_ops counts 2 per lane for a packed instruction, 1 for a scalar one
// (an FMA is one lane-op here, as in DESIGN's 279 lane-ops/px).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/pk_probe tools/pk_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float v2f __attribute__((ext_vector_type(2)));

enum Op { FMA, ADD, MUL, PK_FMA, PK_ADD, PK_MUL, MIX_PK_FMA_ADD };
static const char* kName[] = {"v_fma_f32", "v_add_f32", "v_mul_f32",
                              "v_pk_fma_f32", "v_pk_add_f32", "v_pk_mul_f32",
                              "v_pk_fma_f32+v_add_f32"};
static const int kLaneOps[] = {1, 1, 1, 2, 2, 2, 3};  // per lane per inner step

constexpr int K = 8;       // independent chains per lane
constexpr int INNER = 16;  // unrolled steps per loop iteration

template <int OP>
__global__ __launch_bounds__(256) void chains(float* out, int iters, float s)
{
    const int l = threadIdx.x;
    v2f x[K];
#pragma unroll
    for (int i = 0; i < K; i++) x[i] = (v2f){s * (l + i), s * (l - i)};
    const v2f a = {0.999f, 1.001f}, b = {1e-3f, -1e-3f};
    const float as = 0.999f, bs = 1e-3f;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int j = 0; j < INNER; j++) {
            v2f& r = x[j % K];
            if (OP == FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r.x) : "v"(as), "v"(bs));
            if (OP == ADD) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r.x) : "v"(bs));
            if (OP == MUL) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r.x) : "v"(as));
            if (OP == PK_FMA) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(r) : "v"(a), "v"(b));
            if (OP == PK_ADD) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(r) : "v"(b));
            if (OP == PK_MUL) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(r) : "v"(a));
            if (OP == MIX_PK_FMA_ADD) {
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(r) : "v"(a), "v"(b));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[(j + 1) % K].y) : "v"(bs));
            }
        }
    }
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < K; i++) acc += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + l] = acc;
}

template <int OP>
static void run(float* d, int cus, int waves_per_simd, int iters)
{
    const int blocks = cus * waves_per_simd;  // 4 waves per 256-thread block, one per SIMD
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(chains<OP>, dim3(blocks), dim3(256), 0, 0, d, iters / 8, 1e-3f);  // warm-up
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(chains<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 1e-3f);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double lanes = double(blocks) * 256.0;
    const double steps = double(iters) * INNER;
    const double insts = (OP == MIX_PK_FMA_ADD ? 2.0 : 1.0) * steps * lanes / 64.0;  // wave instructions
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
    float* d = nullptr;
    if (hipMalloc(&d, sizeof(float) * cus * 8 * 256) != hipSuccess) return 1;
    const int iters = 4096;
    for (int w : {4, 8}) {
        run<FMA>(d, cus, w, iters);
        run<ADD>(d, cus, w, iters);
        run<MUL>(d, cus, w, iters);
        run<PK_FMA>(d, cus, w, iters);
        run<PK_ADD>(d, cus, w, iters);
        run<PK_MUL>(d, cus, w, iters);
        run<MIX_PK_FMA_ADD>(d, cus, w, iters);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    (void)hipFree(d);
    return 0;
}
