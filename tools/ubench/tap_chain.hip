// Microbenchmark (dev): issue rate of the headline kernel's packed tap
// pattern on gfx950 -- per tap a v_pk_mul_f32 per output pair and a dependent
// v_pk_add_f32 into that output's accumulator -- with NCH independent
// accumulation chains per wave, at 1 or 2 waves per SIMD (blocks of 256 or
// 512 threads, one block per CU).  Prints core-clock cycles (clock64 =
// s_memtime) per instruction per wave and per SIMD.  PK = 0: the same pattern
// with plain v_mul_f32 / v_add_f32 on one channel.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int NCH, int PK>
__global__ __launch_bounds__(512) void k(float *out, int iters, unsigned long long *cyc)
{
    f2 x[8], acc[NCH];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = f2{threadIdx.x * 1e-3f + i, 1.0f - i * 1e-3f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) acc[c] = f2{0.0f, 0.0f};
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            f2 p[NCH];
            if (PK) {
#pragma unroll
                for (int c = 0; c < NCH; ++c)
                    asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(p[c]) : "v"(x[(t + c) & 7]), "v"(x[(t + 3 * c + 1) & 7]));
#pragma unroll
                for (int c = 0; c < NCH; ++c) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[c]) : "v"(p[c]));
            } else {
#pragma unroll
                for (int c = 0; c < NCH; ++c)
                    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p[c].x) : "v"(x[(t + c) & 7].x), "v"(x[(t + 3 * c + 1) & 7].y));
#pragma unroll
                for (int c = 0; c < NCH; ++c) asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[c].x) : "v"(p[c].x));
            }
        }
    }
    const long long t1 = clock64();
    f2 s = f2{0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += acc[c];
    out[blockIdx.x * 512 + threadIdx.x] = s.x + s.y;
    if (threadIdx.x == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
}

template <int NCH, int PK>
void run(int threads, float *out, unsigned long long *cyc)
{
    const int iters = 4000;
    hipMemset(cyc, 0, 8);
    k<NCH, PK><<<256, threads>>>(out, 100, cyc);
    hipDeviceSynchronize();
    hipMemset(cyc, 0, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k<NCH, PK><<<256, threads>>>(out, iters, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double instr_per_wave = (double)iters * 8 * NCH * 2;
    const int wps = threads / 64 / 4;   // waves per SIMD
    const double cyc_per_wave = (double)c / 256.0;   // clock64 cycles of one wave (block leader)
    printf("%s chains %d  waves/SIMD %d  %.3f ms  %.2f clk per packed instr per wave  -> %.2f clk per instr per SIMD\n",
           PK ? "pk " : "f32", NCH, wps, ms, cyc_per_wave / instr_per_wave, cyc_per_wave / instr_per_wave / wps);
}

int main()
{
    float *out;
    unsigned long long *cyc;
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&cyc, 8);
    for (int th : {256, 512}) {
        run<1, 1>(th, out, cyc);
        run<2, 1>(th, out, cyc);
        run<4, 1>(th, out, cyc);
        run<8, 1>(th, out, cyc);
        run<2, 0>(th, out, cyc);
        run<4, 0>(th, out, cyc);
        run<8, 0>(th, out, cyc);
    }
    return 0;
}
