// Microbenchmark: fp32 v_mul/v_add issue rate vs distance between a product
// and its consuming add (D = chains interleaved), at 2 / 3 / 4 waves per SIMD.
// Shapes the inner tap loop of the fast resampler (xm_resample_fast.hip).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int D>
__global__ __launch_bounds__(64) void k(float *out, float c, int iters)
{
    float a[8], x[8], p[8];
    for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 1e-3f + i; x[i] = a[i] * 0.5f; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int g = 0; g < 8; g += D) {
#pragma unroll
                for (int i = g; i < g + D; ++i) asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p[i]) : "s"(c), "v"(x[i]));
#pragma unroll
                for (int i = g; i < g + D; ++i) asm volatile("v_add_f32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(p[i]));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

int main()
{
    float *out;
    hipMalloc(&out, 1 << 26);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int dev; hipGetDevice(&dev); hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
    int cus = p.multiProcessorCount;
    const int iters = 4000;
    for (int wps : {1, 2, 3, 4, 8}) {          // waves per SIMD
        int blocks = cus * 4 * wps;
        for (int D : {1, 2, 4, 8}) {
            auto run = [&] {
                if (D == 1) k<1><<<blocks, 64>>>(out, 0.3f, iters);
                if (D == 2) k<2><<<blocks, 64>>>(out, 0.3f, iters);
                if (D == 4) k<4><<<blocks, 64>>>(out, 0.3f, iters);
                if (D == 8) k<8><<<blocks, 64>>>(out, 0.3f, iters);
            };
            run(); hipDeviceSynchronize();
            hipEventRecord(e0); run(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            double winstr = (double)blocks * iters * 16 * 16;          // wave-instructions
            double per_simd = winstr / (cus * 4) / (ms * 1e-3);        // instr/s per SIMD
            printf("waves/SIMD %d  D=%d  %7.3f ms  %.3f G wave-instr/s/SIMD\n", wps, D, ms, per_simd / 1e9);
        }
    }
    return 0;
}
