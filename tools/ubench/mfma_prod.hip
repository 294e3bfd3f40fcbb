// Microbenchmark: fp32 MFMA with K = 1 and a zero accumulator as a
// multiplier — is D = A*B + 0 bit-identical to v_mul_f32 (round(a*b)), and
// how fast is "16 products on the matrix core + the adds on the VALU"
// compared with the VALU doing both?  Shapes the tap loop of the resampler.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <random>

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f32v __attribute__((ext_vector_type(32)));

// layout probe: A = 1 + lane, B = 1000 * (1 + lane); D stored per lane/reg
__global__ void k_layout(float *d)
{
    const int l = threadIdx.x;
    f16v acc = {};
    acc = __builtin_amdgcn_mfma_f32_16x16x1f32((float)(1 + l), 1000.0f * (1 + l), acc, 0, 0, 0);
    for (int r = 0; r < 16; ++r) d[l * 16 + r] = acc[r];
}

// exactness: lane l holds x[l] (B) and c[l % 16] (A): D[r] of lane l should be
// x[l] * c[r] (per the layout probe); compare with v_mul_f32 bit for bit
__global__ void k_exact(const float *x, const float *c, unsigned *bad, float *sample, int n)
{
    const int l = threadIdx.x;
    const long base = (long)blockIdx.x * 64;
    if (base >= n) return;
    const float xv = x[base + l];
    const float cv = c[(base / 64 * 16 + (l & 15)) % n];
    f16v acc = {};
    acc = __builtin_amdgcn_mfma_f32_16x16x1f32(cv, xv, acc, 0, 0, 0);
    unsigned nb = 0;
    for (int r = 0; r < 16; ++r) {
        const float cr = c[(base / 64 * 16 + r) % n];
        float p;
        asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p) : "v"(xv), "v"(cr));
        unsigned a = __builtin_bit_cast(unsigned, acc[r]), b = __builtin_bit_cast(unsigned, p);
        // +0/-0 differences are tolerated by the kernel's final "+ 0" only
        // when the value is a zero; count them separately
        if (a != b) nb += ((a << 1) == 0 && (b << 1) == 0) ? 0x10000u : 1u;
        if (blockIdx.x == 0) sample[l * 16 + r] = acc[r];
    }
    atomicAdd(bad, nb);
}

// throughput.  MODE 0: VALU only, per "frame" 20 v_mul + 20 v_add.
// MODE 1: 1 MFMA 16x16x1_4b (16 products) + 4 v_mul, then 20 v_add.
// MODE 2: MFMA only (no consumers).  MODE 3: 32x32x1_2b + 20 v_add.
template <int MODE>
__global__ __launch_bounds__(64) void k_rate(const float *in, float *out, int iters)
{
    const int l = threadIdx.x;
    float x = in[l] + (float)blockIdx.x * 1e-6f;
    const float cv = in[64 + (l & 15)];
    float acc[20];
    for (int i = 0; i < 20; ++i) acc[i] = in[128 + i];
    float c4[4] = {in[200], in[201], in[202], in[203]};
    float cs[20];
    for (int i = 0; i < 20; ++i) cs[i] = in[210 + i];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            if (MODE == 0) {
                float p[20];
#pragma unroll
                for (int i = 0; i < 20; ++i) asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p[i]) : "v"(x), "s"(cs[i]));
#pragma unroll
                for (int i = 0; i < 20; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(p[i]));
            } else if (MODE == 1 || MODE == 2) {
                f16v d = {};
                d = __builtin_amdgcn_mfma_f32_16x16x1f32(cv, x, d, 0, 0, 0);
                if (MODE == 1) {
                    float p[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p[i]) : "v"(x), "s"(c4[i]));
#pragma unroll
                    for (int i = 0; i < 16; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(d[i]));
#pragma unroll
                    for (int i = 0; i < 4; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[16 + i]) : "v"(p[i]));
                } else {
                    asm volatile("" ::"v"(d));
                }
            } else {
                f32v d = {};
                d = __builtin_amdgcn_mfma_f32_32x32x1f32(cv, x, d, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 20; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(d[i]));
            }
            x = x * 0.999f;   // fresh operand per frame (1 extra VALU in every mode)
        }
    }
    float s = 0;
    for (int i = 0; i < 20; ++i) s += acc[i];
    out[blockIdx.x * 64 + l] = s;
}

int main()
{
    // layout
    float *d;
    hipMalloc(&d, 64 * 16 * 4);
    k_layout<<<1, 64>>>(d);
    std::vector<float> h(64 * 16);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    int ok = 1;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            // hypothesis: lane l, reg r = A_b[r] * B_b[j], b = l / 16, j = l % 16
            const float want = (float)(1 + 16 * (l / 16) + r) * 1000.0f * (1 + l);
            if (h[l * 16 + r] != want) ok = 0;
        }
    printf("layout 16x16x1_4b: lane l reg r = A[lane 16*(l/16)+r] * B[lane l]: %s (lane 5: %g %g %g)\n",
           ok ? "yes" : "NO", h[5 * 16 + 0], h[5 * 16 + 1], h[5 * 16 + 15]);

    // exactness over random + special values
    const int n = 1 << 22;
    std::vector<float> hx(n), hc(n);
    std::mt19937 rng(123);
    std::uniform_real_distribution<float> u(-1.0f, 1.0f);
    for (int i = 0; i < n; ++i) {
        hx[i] = u(rng);
        hc[i] = u(rng) * 0.05f;
        const int k = i % 97;
        if (k == 0) hx[i] = 0.0f;
        if (k == 1) hx[i] = -0.0f;
        if (k == 2) hc[i] = -0.0f;
        if (k == 3) hx[i] = 1e-38f * u(rng);             // denormal-ish inputs
        if (k == 4) hc[i] = 3e-39f;                      // denormal coefficient
        if (k == 5) hx[i] = 1e-20f, hc[i] = 1e-20f;      // product underflows to denormal/zero
        if (k == 6) hx[i] = 3e38f, hc[i] = 10.0f;        // overflow -> inf
        if (k == 7) hx[i] = 1.0f + (float)i * 1e-7f;     // exact-ish ties
        if (k == 8) hx[i] = 1.5e-19f, hc[i] = 7.3e-20f;  // product in the denormal range
    }
    float *dx, *dc, *ds;
    unsigned *db;
    hipMalloc(&dx, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&db, 4); hipMalloc(&ds, 64 * 16 * 4);
    hipMemcpy(dx, hx.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dc, hc.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(db, 0, 4);
    k_exact<<<n / 64, 64>>>(dx, dc, db, ds, n);
    unsigned bad = 0;
    hipMemcpy(&bad, db, 4, hipMemcpyDeviceToHost);
    printf("exactness 16x16x1 (C=0) vs v_mul_f32 over %d products: %u value mismatches, %u zero-sign mismatches\n",
           n * 16, bad & 0xffff, bad >> 16);
    // host cross-check of a sample (separately rounded product on the CPU)
    std::vector<float> hs(64 * 16);
    hipMemcpy(hs.data(), ds, hs.size() * 4, hipMemcpyDeviceToHost);
    int hbad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            volatile float p = hx[l] * hc[r];
            if (memcmp((const void *)&p, &hs[l * 16 + r], 4)) ++hbad;
        }
    printf("host check of block 0: %d mismatches of 1024\n", hbad);

    // rates
    float *in, *out;
    hipMalloc(&in, 4096); hipMalloc(&out, 64 * 4 * 256 * 64);
    std::vector<float> hin(1024);
    for (auto &v : hin) v = u(rng);
    hipMemcpy(in, hin.data(), 4096, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 2000;
    for (int wps = 1; wps <= 4; wps *= 2) {
        const int blocks = 256 * 4 * wps;
        auto run = [&](auto kern, const char *name, double products_per_frame) {
            for (int rep = 0; rep < 3; ++rep) kern<<<blocks, 64>>>(in, out, iters);
            hipEventRecord(e0);
            for (int rep = 0; rep < 10; ++rep) kern<<<blocks, 64>>>(in, out, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= 10;
            const double prod = (double)blocks * 64 * iters * 8 * products_per_frame;
            printf("waves/SIMD %d  %-34s %8.3f ms  %6.2f T useful products(+adds)/s\n", wps, name, ms, prod / (ms * 1e-3) / 1e12);
        };
        run(k_rate<0>, "VALU 20 mul + 20 add", 20);
        run(k_rate<1>, "MFMA16x16x1 + 4 mul + 20 add", 20);
        run(k_rate<2>, "MFMA16x16x1 only (16 products)", 16);
        run(k_rate<3>, "MFMA32x32x1_2b + 20 add", 20);
    }
    return 0;
}
