// Microbenchmark: issue rate of separately-rounded fp32 mul/add on gfx950,
// scalar (v_mul_f32/v_add_f32) vs packed (v_pk_mul_f32/v_pk_add_f32), with the
// coefficient as a wave-uniform SGPR operand — the inner loop of the resampler.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k(float *out, const float *coef, int iters)
{
    float c0 = coef[0], c1 = coef[1];
    float a[8], x[8];
    f2 pa[8], px[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * 1e-3f + i; x[i] = a[i] * 0.5f;
        pa[i] = f2{a[i], a[i] + 1}; px[i] = f2{x[i], x[i] + 2};
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (MODE == 0) {          // scalar mul + add (2 instr / lane-op pair)
                    float p; asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p) : "s"(c0), "v"(x[i]));
                    asm volatile("v_add_f32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(p));
                } else if (MODE == 1) {   // packed mul + add, SGPR pair operand
                    f2 p; f2 cc = f2{c0, c1};
                    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(p) : "s"(cc), "v"(px[i]));
                    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(pa[i]) : "v"(pa[i]), "v"(p));
                } else if (MODE == 2) {   // scalar fma
                    asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "s"(c0), "v"(x[i]));
                } else if (MODE == 3) {   // packed fma
                    f2 cc = f2{c0, c1};
                    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(pa[i]) : "s"(cc), "v"(px[i]));
                } else if (MODE == 4) {   // scalar mul with literal + add
                    float p; asm volatile("v_mul_f32 %0, 0x3e9a209b, %1" : "=v"(p) : "v"(x[i]));
                    asm volatile("v_add_f32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(p));
                }
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + pa[i].x + pa[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main()
{
    float *out, *coef;
    hipMalloc(&out, 1 << 24); hipMalloc(&coef, 64);
    float h[2] = {0.3f, 0.7f}; hipMemcpy(coef, h, 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int dev; hipGetDevice(&dev); hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
    int cus = p.multiProcessorCount;
    printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
    for (int wpc : {8, 16, 32}) {   // waves per CU
        int blocks = cus * wpc / 4, iters = 2000;
        const char *names[] = {"mul+add", "pk_mul+pk_add", "fma", "pk_fma", "mul(lit)+add"};
        for (int mode = 0; mode < 5; ++mode) {
            auto run = [&] {
                switch (mode) {
                case 0: k<0><<<blocks, 256>>>(out, coef, iters); break;
                case 1: k<1><<<blocks, 256>>>(out, coef, iters); break;
                case 2: k<2><<<blocks, 256>>>(out, coef, iters); break;
                case 3: k<3><<<blocks, 256>>>(out, coef, iters); break;
                case 4: k<4><<<blocks, 256>>>(out, coef, iters); break;
                }
            };
            run(); hipDeviceSynchronize();
            hipEventRecord(e0); run(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            int ipi = (mode == 2 || mode == 3) ? 1 : 2;  // instructions per inner op
            double winstr = (double)blocks * 4 * iters * 16 * 8 * ipi;  // wave-instructions
            double lanefl = (double)blocks * 256 * iters * 16 * 8 * ((mode == 1 || mode == 3) ? 2 : 1); // mul-add pairs per lane-value
            printf("wpc %2d %-14s %8.3f ms  %.3f wave-instr/clk/CU(@2.4GHz)  %.1f T mul-add pairs/s\n", wpc, names[mode], ms,
                   winstr / (ms * 1e-3) / cus / 2.4e9, lanefl / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
