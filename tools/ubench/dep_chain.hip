// Microbenchmark: dependent-chain latency of fp32 VALU ops on gfx950, one
// wave per SIMD, and the sosfilt recurrence itself (packed L/R vs scalar).
// Shapes the biquad kernel (xm_fx.hip k_biquad_pipe).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(64) void k(float *out, const float *cf, int iters)
{
    const float b0 = cf[0], b1 = cf[1], b2 = cf[2], a1 = cf[3], a2 = cf[4];
    float s = threadIdx.x * 1e-3f, t = s + 1.0f;
    f2 ps = f2{s, t};
    float z0 = 0, z1 = 0, y0 = 0, y1 = 0;
    f2 pz0 = f2{0, 0}, pz1 = f2{0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 64; ++r) {
            if (MODE == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s) : "v"(t));            // dep add
            if (MODE == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(ps) : "v"(ps));       // dep pk add
            if (MODE == 2) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(ps) : "v"(ps));       // dep pk mul
            if (MODE == 3) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(s) : "v"(t));            // dep mul
            if (MODE == 4) {   // sosfilt section, packed (L, R)
                const f2 v = ps;
                const f2 o = b0 * v + pz0;
                pz0 = (b1 * v - a1 * o) + pz1;
                pz1 = b2 * v - a2 * o;
                ps = o * 0.5f;
            }
            if (MODE == 5) {   // sosfilt section, two scalar chains
                const float v0 = s, v1 = t;
                const float o0 = b0 * v0 + z0, o1 = b0 * v1 + y0;
                z0 = (b1 * v0 - a1 * o0) + z1;
                y0 = (b1 * v1 - a1 * o1) + y1;
                z1 = b2 * v0 - a2 * o0;
                y1 = b2 * v1 - a2 * o1;
                s = o0 * 0.5f;
                t = o1 * 0.5f;
            }
        }
    }
    out[blockIdx.x * 64 + threadIdx.x] = s + t + ps.x + ps.y + z0 + z1 + pz0.x + pz1.y + y0 + y1;
}

int main()
{
    float *out, *cf;
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cf, 64);
    float h[5] = {0.2f, 0.3f, 0.1f, -0.5f, 0.25f};
    hipMemcpy(cf, h, 20, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 20000;
    auto run = [&](auto kern, const char *name, int per) {
        kern<<<256, 64>>>(out, cf, 100);
        hipEventRecord(e0);
        kern<<<256, 64>>>(out, cf, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double ns = ms * 1e6 / ((double)iters * 64 * per);
        printf("%-40s %8.3f ms  %6.3f ns per step  (%.1f cyc @2.1GHz)\n", name, ms, ns, ns * 2.1);
    };
    run(k<0>, "dep v_add_f32", 1);
    run(k<3>, "dep v_mul_f32", 1);
    run(k<1>, "dep v_pk_add_f32", 1);
    run(k<2>, "dep v_pk_mul_f32", 1);
    run(k<4>, "sosfilt sample, packed L/R", 1);
    run(k<5>, "sosfilt sample, 2 scalar chains", 1);
    return 0;
}
