// Microbenchmark (dev): cycles per frame of one biquad chain per lane, lone
// wave per SIMD, products from registers:
//   mode 0  6 VALU per frame (bq_mf_pair's scalar order)
//   mode 1  4 instructions per frame: o = p0 + z0; (t, u) = (-a1, -a2) * o
//           (v_pk_mul_f32); (t, z1) = (p1, p2) + (t, u) (v_pk_add_f32); z0 = z1 + t
//   mode 2  mode 0 with a ds_write_b128 of the outputs every 4 frames
//   mode 3  mode 1 with a ds_write_b128 of the outputs every 4 frames
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(64) void k(float *out, const float *cf, int steps, long long *cyc)
{
    __shared__ f4 sh[64];
    const int lane = threadIdx.x;
    const float na1 = -cf[3], na2 = -cf[4];
    const f2 nA = {na1, na2};
    float p0[4], p1[4], p2[4];
    for (int i = 0; i < 4; ++i) { p0[i] = cf[i] * lane; p1[i] = cf[i + 1]; p2[i] = cf[i + 2]; }
    float z0 = 0.0f, z1 = 0.0f, acc = 0.0f;
    const long long t0 = clock64();
    for (int n = 0; n < steps; ++n) {
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                o[e] = p0[e] + z0;
                if (MODE == 0 || MODE == 2) {
                    const float t = p1[e] + na1 * o[e];
                    const float w = p2[e] + na2 * o[e];
                    z0 = z1 + t;
                    z1 = w;
                } else {
                    const f2 r = f2{p1[e], p2[e]} + nA * f2{o[e], o[e]};
                    z0 = z1 + r.x;
                    z1 = r.y;
                }
            }
            if (MODE >= 2) sh[lane] = f4{o[0], o[1], o[2], o[3]};
            else acc = acc + o[g & 3];
        }
    }
    const long long t1 = clock64();
    out[blockIdx.x * 64 + lane] = z0 + z1 + acc + (MODE >= 2 ? sh[lane ^ 1][0] : 0.0f);
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
    float *cf, *out;
    long long *cyc;
    const float hcf[8] = {0.2f, -0.3f, 0.1f, -1.1f, 0.35f, 0.1f, 0.2f, 0.3f};
    const int steps = 4000, blocks = 1024;   // one wave per SIMD
    hipMalloc(&cf, 32); hipMalloc(&out, blocks * 64 * 4); hipMalloc(&cyc, blocks * 8);
    hipMemcpy(cf, hcf, 32, hipMemcpyHostToDevice);
    auto run = [&](auto kern, const char *name) {
        kern<<<blocks, 64>>>(out, cf, 10, cyc);
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        kern<<<blocks, 64>>>(out, cf, steps, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<long long> h(blocks);
        hipMemcpy(h.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (auto v : h) s += (double)v;
        const double frames = (double)steps * 64;
        printf("%-64s %7.3f ms  %6.2f ns/frame  %6.1f clock64/frame\n", name, ms, ms * 1e6 / frames, s / blocks / frames);
    };
    run(k<0>, "mode 0 scalar, 6 VALU per frame");
    run(k<1>, "mode 1 packed (t,u) / (p1,p2): 4 instructions per frame");
    run(k<2>, "mode 2 scalar + ds_write_b128 per 4 frames");
    run(k<3>, "mode 3 packed + ds_write_b128 per 4 frames");
    return 0;
}
