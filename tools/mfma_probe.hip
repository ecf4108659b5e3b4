// mfma_probe.hip -- measures what the N = 8 co-issue design of dcte_map
// relies on (tools/mfma_probe.sh builds and runs it on the GPU box):
//  1. the register/lane layout of v_mfma_f32_4x4x1_16b_f32 (D = A x B per
//     4-lane block) and that it is a plain fmaf per element;
//  2. its issue cost per SIMD (back-to-back, independent accumulators);
//  3. VALU + MFMA co-issue: a loop of V dependent-free v_fma_f32 per lane and
//     M MFMAs, timed against V alone and M alone.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void layout(float* out)
{
    const int l = threadIdx.x;
    const float a = 1.0f + l, b = 1000.0f * (1 + l);
    v4f c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) out[l * 4 + r] = c[r];
}

// fmaf chain check: acc = fma(a_t, b_t, acc) over t, rounding per step
__global__ void chain(const float* a, const float* b, float* out, int K)
{
    const int l = threadIdx.x;
    v4f c = {0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < K; t++) c = __builtin_amdgcn_mfma_f32_4x4x1f32(a[t * 64 + l], b[t * 64 + l], c, 0, 0, 0);
    for (int r = 0; r < 4; r++) out[l * 4 + r] = c[r];
}

template <int V, int M>
__global__ __launch_bounds__(256) void mix(float* out, int iters, float s)
{
    const int l = threadIdx.x;
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = s * (l + i);
    v4f acc[8];
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (v4f){0.f, 0.f, 0.f, 0.f};
    const float ca = 0.5f + l * 1e-3f, cb = 0.25f - l * 1e-3f;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int j = 0; j < (V > M ? V : M); j++) {
            if (j < M) acc[j & 7] = __builtin_amdgcn_mfma_f32_4x4x1f32(ca, x[j & 7], acc[j & 7], 0, 0, 0);
            if (j < V) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[j & 7]) : "v"(cb), "v"(ca));
        }
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) r += x[i] + acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + l] = r;
}

template <int V, int M>
static double run_mix(float* d, int blocks, int iters)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((mix<V, M>), dim3(blocks), dim3(256), 0, 0, d, iters, 1e-3f);
    hipEventRecord(a, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL((mix<V, M>), dim3(blocks), dim3(256), 0, 0, d, iters, 1e-3f);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main()
{
    float* d;
    hipMalloc(&d, 1 << 24);
    float h[256];
    hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    // decode: value = a_i * b_j with a = 1 + i, b = 1000 (1 + j)
    printf("{\"probe\":\"layout\",\"lanes\":[");
    for (int l = 0; l < 8; l++) {
        printf("%s[", l ? "," : "");
        for (int r = 0; r < 4; r++) {
            const float v = h[l * 4 + r];
            int ai = -1, bj = -1;
            for (int i = 0; i < 64 && ai < 0; i++)
                for (int j = 0; j < 64; j++)
                    if ((float)((1.0f + i) * (1000.0f * (1 + j))) == v) { ai = i; bj = j; break; }
            printf("%s\"a%d*b%d\"", r ? "," : "", ai, bj);
        }
        printf("]");
    }
    printf("]}\n");

    // fmaf chain bit-check on random data, K = 4 and 8
    const int K = 8;
    float ha[K * 64], hb[K * 64];
    srand(3);
    for (int i = 0; i < K * 64; i++) {
        ha[i] = (float)(rand() % 20001 - 10000) * 1.2345678e-1f;
        hb[i] = (float)(rand() % 20001 - 10000) * 7.654321e-2f;
    }
    float *da, *db;
    hipMalloc(&da, sizeof(ha));
    hipMalloc(&db, sizeof(hb));
    hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
    int bad_fma = 0, bad_sep = 0;
    for (int k = 4; k <= 8; k += 4) {
        hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, da, db, d, k);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        // assumes layout D[r] of lane l = A[lane 4(l/4)+r] * B[lane l]; checked above
        for (int l = 0; l < 64; l++)
            for (int r = 0; r < 4; r++) {
                const int la = 4 * (l / 4) + r, lb = l;
                float acc = 0.f, acc2 = 0.f;
                for (int t = 0; t < k; t++) {
                    acc = fmaf(ha[t * 64 + la], hb[t * 64 + lb], acc);
                    volatile float p = ha[t * 64 + la] * hb[t * 64 + lb];
                    acc2 = acc2 + p;
                }
                bad_fma += h[l * 4 + r] != acc;
                bad_sep += h[l * 4 + r] != acc2;
            }
    }
    printf("{\"probe\":\"fmaf_chain\",\"mismatch_vs_fmaf\":%d,\"mismatch_vs_mul_add\":%d,\"of\":512}\n",
           bad_fma, bad_sep);

    // issue costs: blocks = 4 waves per SIMD on 256 CUs
    const int blocks = 256 * 4, iters = 4096;
    double t_v = run_mix<16, 0>(d, blocks, iters);
    double t_m = run_mix<0, 16>(d, blocks, iters);
    double t_vm = run_mix<16, 16>(d, blocks, iters);
    double t_v32m8 = run_mix<32, 8>(d, blocks, iters);
    double t_v32 = run_mix<32, 0>(d, blocks, iters);
    double t_m8 = run_mix<0, 8>(d, blocks, iters);
    // per SIMD: waves per SIMD = blocks * 4 waves / 1024 SIMDs = 4
    const double ops = (double)iters * 4 /*waves per SIMD*/;
    auto cyc = [&](double ms, int per_iter) { return ms * 1e-3 * 2.4e9 / (ops * per_iter); };
    printf("{\"probe\":\"issue\",\"ms\":{\"V16\":%.4f,\"M16\":%.4f,\"V16M16\":%.4f,\"V32\":%.4f,\"M8\":%.4f,\"V32M8\":%.4f},"
           "\"cyc_per_valu_at_2.4GHz\":%.2f,\"cyc_per_mfma_at_2.4GHz\":%.2f}\n",
           t_v, t_m, t_vm, t_v32, t_m8, t_v32m8, cyc(t_v, 16), cyc(t_m, 16));
    return 0;
}
