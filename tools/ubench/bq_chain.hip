// Microbenchmark (dev): cost per stereo frame of the hand-scheduled biquad
// granule step (xm_fx.hip bq_step2) for a lone wave per SIMD.
//   mode 0: registers only (input recycled from the previous output)
//   mode 1: + one ds_read_b128 / ds_write_b128 per granule (2 frames)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f4 step2(f4 v4, f2 &z0, f2 &z1, f2 b0, f2 b1, f2 b2, f2 a1, f2 a2)
{
    const f2 va = {v4[0], v4[1]}, vb = {v4[2], v4[3]};
    f2 oa, ob, p0, p1, p2, t, u;
    asm volatile(
        "v_pk_mul_f32 %[p0], %[b0], %[va]\n\t"
        "v_pk_mul_f32 %[p1], %[b1], %[va]\n\t"
        "v_pk_add_f32 %[oa], %[z0], %[p0]\n\t"
        "v_pk_mul_f32 %[p2], %[b2], %[va]\n\t"
        "v_pk_mul_f32 %[t], %[a1], %[oa] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[p0], %[b0], %[vb]\n\t"
        "v_pk_add_f32 %[t], %[p1], %[t]\n\t"
        "v_pk_mul_f32 %[u], %[a2], %[oa] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %[z0], %[z1], %[t]\n\t"
        "v_pk_add_f32 %[z1], %[p2], %[u]\n\t"
        "v_pk_add_f32 %[ob], %[z0], %[p0]\n\t"
        "v_pk_mul_f32 %[p1], %[b1], %[vb]\n\t"
        "v_pk_mul_f32 %[t], %[a1], %[ob] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[p2], %[b2], %[vb]\n\t"
        "v_pk_add_f32 %[t], %[p1], %[t]\n\t"
        "v_pk_mul_f32 %[u], %[a2], %[ob] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %[z0], %[z1], %[t]\n\t"
        "v_pk_add_f32 %[z1], %[p2], %[u]"
        : [oa] "=&v"(oa), [ob] "=&v"(ob), [p0] "=&v"(p0), [p1] "=&v"(p1), [p2] "=&v"(p2), [t] "=&v"(t),
          [u] "=&v"(u), [z0] "+v"(z0), [z1] "+v"(z1)
        : [va] "v"(va), [vb] "v"(vb), [b0] "v"(b0), [b1] "v"(b1), [b2] "v"(b2), [a1] "v"(a1), [a2] "v"(a2));
    return f4{oa.x, oa.y, ob.x, ob.y};
}

template <int MODE>
__global__ __launch_bounds__(64) void k(float *out, const float *cf, int steps)
{
    __shared__ f4 sec[32][64];
    const int lane = threadIdx.x;
    const f2 b0 = {cf[0], cf[0]}, b1 = {cf[1], cf[1]}, b2 = {cf[2], cf[2]}, a1 = {cf[3], cf[3]}, a2 = {cf[4], cf[4]};
    f2 z0 = {0, 0}, z1 = {0, 0};
    f4 v = {lane * 1e-3f, 1, 2, 3};
    for (int g = 0; g < 32; ++g) sec[g][lane] = v;
    __builtin_amdgcn_wave_barrier();
    const f4 *src = &sec[0][(lane + 63) & 63];
    for (int n = 0; n < steps; ++n) {
        if (MODE == 0) {
#pragma unroll
            for (int g = 0; g < 32; ++g) v = step2(v, z0, z1, b0, b1, b2, a1, a2);
        } else {
            f4 n0 = src[0], n1 = src[64];
#pragma unroll
            for (int g = 0; g < 32; ++g) {
                const f4 x = n0;
                n0 = n1;
                if (g + 2 < 32) n1 = src[(g + 2) * 64];
                sec[g][lane] = step2(x, z0, z1, b0, b1, b2, a1, a2);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    out[blockIdx.x * 64 + lane] = v.x + z0.x + z1.y + sec[lane & 31][lane].x;
}

int main()
{
    float *out, *cf;
    hipMalloc(&out, 1 << 22);
    hipMalloc(&cf, 64);
    float h[5] = {0.2f, 0.3f, 0.1f, -0.5f, 0.25f};
    hipMemcpy(cf, h, 20, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int steps = 6890;   // 441000 frames / 64 frames per step
    for (int mode = 0; mode < 2; ++mode)
        for (int waves : {86, 1024}) {
            auto kern = mode ? k<1> : k<0>;
            kern<<<waves, 64>>>(out, cf, 100);
            hipEventRecord(e0);
            kern<<<waves, 64>>>(out, cf, steps);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("mode %d, %4d waves: %.3f ms for 441000 frames, %.2f ns per frame\n", mode, waves, ms,
                   ms * 1e6 / 441000.0);
        }
    return 0;
}
