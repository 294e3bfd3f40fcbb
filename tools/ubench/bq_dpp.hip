// Microbenchmark (dev): the sosfilt cascade as a lane pipeline chained by DPP
// (row_shr:1) instead of LDS.  Per 16-lane row, groups of NS+1 lanes: lane 0
// of a group feeds the input, lanes 1..NS are the sections (one channel per
// lane).  Per step every lane runs 3 DPP-sourced products (b0/b1/b2 times the
// left neighbour's output of the previous step), the 6-op recurrence and one
// select (feeder: the input).  Prints ns per step (= per frame of every clip).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NS>
__global__ __launch_bounds__(64) void k(float *out, const float *cf, int steps)
{
    const int lane = threadIdx.x;
    const int g = (lane & 15) % (NS + 1);            // 0 = feeder
    const bool feeder = g == 0;
    const float b0 = feeder ? 1.0f : cf[0], b1 = cf[1], b2 = cf[2], a1 = cf[3], a2 = cf[4];
    float z0 = 0.0f, z1 = 0.0f, w = 0.0f, in = lane * 1e-3f;
    const unsigned long long mask = __builtin_amdgcn_ballot_w64(feeder);
    for (int n = 0; n < steps; ++n) {
        float p0, p1, p2, o, t, u;
        // s_nop 1: a VALU write of w needs 2 wait states before a DPP read of it
        asm volatile(
            "s_nop 1\n\t"
            "v_mul_f32_dpp %0, %3, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_mul_f32_dpp %1, %3, %5 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_mul_f32_dpp %2, %3, %6 row_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(p0), "=&v"(p1), "=&v"(p2)
            : "v"(w), "v"(b0), "v"(b1), "v"(b2));
        o = p0 + z0;
        t = a1 * o;
        u = p1 - t;
        z0 = u + z1;
        z1 = p2 - a2 * o;
        w = ((mask >> lane) & 1) ? in : o;
        in = in + 1e-6f;
    }
    out[blockIdx.x * 64 + lane] = w + z0 + z1;
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
    const int steps = 100000;
    for (int waves : {256, 1024}) {
        k<5><<<waves, 64>>>(out, cf, 1000);
        hipEventRecord(e0);
        k<5><<<waves, 64>>>(out, cf, steps);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("dpp cascade NS=5, %4d waves: %.3f ms, %.2f ns per step -> 441000 frames: %.2f ms\n", waves, ms,
               ms * 1e6 / steps, ms * 441000.0 / steps);
    }
    return 0;
}
