// Microbenchmark (dev): can the biquad's feed-forward products b_k * x go to
// the matrix core while the VALU runs only the feedback recurrence?
//  1. layout of v_mfma_f32_4x4x1_16b_f32: lane l, reg r = A[lane 4*(l/4)+r] * B[lane l]?
//  2. exactness: D = A*B + (-0) against v_mul_f32, bit for bit, over random,
//     zero, denormal, underflowing and overflowing operands (and C = +0 for
//     comparison: there a -0 product comes back +0)
//  3. cycles per frame for a lone wave per SIMD:
//     mode 0  packed stereo bq_step2 (9 v_pk ops per frame, 2 chains per lane)
//     mode 1  one chain per lane, products from registers (6 VALU per frame)
//     mode 2  one chain per lane, products by one 4x4x1 MFMA per frame one
//             granule (4 frames) ahead, x from LDS by ds_read2_b32, outputs
//             to LDS by ds_write2_b32 (the shape of a channel-per-lane kernel)
//     mode 3  mode 0 with its LDS traffic (one ds_read_b128 / ds_write_b128
//             per granule of 2 stereo frames)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <random>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void k_layout(float *d)
{
    const int l = threadIdx.x;
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(1 + l), 1000.0f * (1 + l), acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}

template <bool NEGZ>
__global__ void k_exact(const float *x, const float *c, unsigned *bad, int n)
{
    const int l = threadIdx.x;
    const long base = (long)blockIdx.x * 64;
    if (base >= n) return;
    const float xv = x[base + l];
    const float cv = c[base + l];   // A of lane l: coefficient c[base + l]
    const float z = NEGZ ? -0.0f : 0.0f;
    f4 acc = {z, z, z, z};
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(cv, xv, acc, 0, 0, 0);
    unsigned nb = 0;
    for (int r = 0; r < 4; ++r) {
        const float cr = c[base + 4 * (l / 4) + r];
        float p;
        asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p) : "v"(xv), "v"(cr));
        const unsigned a = __builtin_bit_cast(unsigned, acc[r]), b = __builtin_bit_cast(unsigned, p);
        if (a != b) nb += ((a << 1) == 0 && (b << 1) == 0) ? 0x10000u : 1u;
    }
    atomicAdd(bad, nb);
}

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

// one frame of one chain from precomputed products (sosfilt order):
// o = P0 + z0; z0 = (P1 - a1*o) + z1; z1 = P2 - a2*o
__device__ __forceinline__ float step1(f4 p, float &z0, float &z1, float na1, float na2)
{
    float o, t, u, w;
    asm volatile(
        "v_add_f32 %[o], %[z0], %[p0]\n\t"
        "v_mul_f32 %[t], %[na1], %[o]\n\t"
        "v_mul_f32 %[u], %[na2], %[o]\n\t"
        "v_add_f32 %[t], %[p1], %[t]\n\t"
        "v_add_f32 %[w], %[p2], %[u]\n\t"
        "v_add_f32 %[z0], %[z1], %[t]\n\t"
        "v_mov_b32 %[z1], %[w]"
        : [o] "=&v"(o), [t] "=&v"(t), [u] "=&v"(u), [w] "=&v"(w), [z0] "+v"(z0), [z1] "+v"(z1)
        : [p0] "v"(p[0]), [p1] "v"(p[1]), [p2] "v"(p[2]), [na1] "v"(na1), [na2] "v"(na2));
    return o;
}

// the same without the move: z1 ping-pongs between two registers (frames in pairs)
__device__ __forceinline__ void step1x2(f4 pa, f4 pb, float &z0, float &z1, float na1, float na2, float &oa, float &ob)
{
    float t, u, w;
    asm volatile(
        "v_add_f32 %[oa], %[z0], %[pa0]\n\t"
        "v_mul_f32 %[t], %[na1], %[oa]\n\t"
        "v_mul_f32 %[u], %[na2], %[oa]\n\t"
        "v_add_f32 %[t], %[pa1], %[t]\n\t"
        "v_add_f32 %[w], %[pa2], %[u]\n\t"
        "v_add_f32 %[z0], %[z1], %[t]\n\t"
        "v_add_f32 %[ob], %[z0], %[pb0]\n\t"
        "v_mul_f32 %[t], %[na1], %[ob]\n\t"
        "v_mul_f32 %[u], %[na2], %[ob]\n\t"
        "v_add_f32 %[t], %[pb1], %[t]\n\t"
        "v_add_f32 %[z1], %[pb2], %[u]\n\t"
        "v_add_f32 %[z0], %[w], %[t]"
        : [oa] "=&v"(oa), [ob] "=&v"(ob), [t] "=&v"(t), [u] "=&v"(u), [w] "=&v"(w), [z0] "+v"(z0), [z1] "+v"(z1)
        : [pa0] "v"(pa[0]), [pa1] "v"(pa[1]), [pa2] "v"(pa[2]), [pb0] "v"(pb[0]), [pb1] "v"(pb[1]),
          [pb2] "v"(pb[2]), [na1] "v"(na1), [na2] "v"(na2));
}

constexpr int GR = 32;   // granules per pass

template <int MODE>
__global__ __launch_bounds__(64) void k(float *out, const float *cf, int steps, long long *cyc)
{
    __shared__ f4 sec[GR + 2][64];
    const int lane = threadIdx.x;
    for (int g = 0; g < GR + 2; ++g) sec[g][lane] = f4{lane * 1e-3f, 1e-3f * g, 2, 3};
    __builtin_amdgcn_wave_barrier();
    const long long t0 = clock64();
    float res = 0.0f;
    if (MODE == 0 || MODE == 3) {
        const f2 b0 = {cf[0], cf[0]}, b1 = {cf[1], cf[1]}, b2 = {cf[2], cf[2]}, a1 = {cf[3], cf[3]}, a2 = {cf[4], cf[4]};
        f2 z0 = {0, 0}, z1 = {0, 0};
        f4 v = {lane * 1e-3f, 1, 2, 3};
        const f4 *src = &sec[0][(lane + 63) & 63];
        for (int n = 0; n < steps; ++n) {
            if (MODE == 0) {
#pragma unroll
                for (int g = 0; g < GR; ++g) v = step2(v, z0, z1, b0, b1, b2, a1, a2);
            } else {
                f4 n0 = src[0], n1 = src[64];
#pragma unroll
                for (int g = 0; g < GR; ++g) {
                    const f4 x = n0;
                    n0 = n1;
                    if (g + 2 < GR) n1 = src[(g + 2) * 64];
                    v = step2(x, z0, z1, b0, b1, b2, a1, a2);
                    sec[g][lane] = v;
                }
            }
        }
        res = v[0] + v[1] + v[2] + v[3];
    } else {
        // one chain per lane; a granule = 4 frames of it
        const float na1 = -cf[3], na2 = -cf[4];
        const float A = (lane & 3) < 3 ? cf[lane & 3] : 0.0f;   // block rows: b0, b1, b2, 0
        float z0 = 0.0f, z1 = 0.0f;
        const float *fsrc = (const float *)&sec[0][0] + ((lane + 60) & 63) * 4;   // "previous section" row
        float *fdst = (float *)&sec[0][0] + lane * 4;
        if (MODE == 1) {
            f4 p[4];
            for (int i = 0; i < 4; ++i) p[i] = f4{cf[i] * lane, cf[i + 1], cf[i + 2], 0.0f};
            for (int n = 0; n < steps; ++n) {
#pragma unroll
                for (int g = 0; g < GR; ++g) {
                    float oa, ob, oc, od;
                    step1x2(p[0], p[1], z0, z1, na1, na2, oa, ob);
                    step1x2(p[2], p[3], z0, z1, na1, na2, oc, od);
                    p[g & 3][3] = oa + od;   // keep the outputs alive (unused slot)
                    (void)ob; (void)oc;
                }
            }
            res = z0 + z1 + p[0][3] + p[1][3] + p[2][3] + p[3][3];
        } else {
            const f4 nz = {-0.0f, -0.0f, -0.0f, -0.0f};
            // granule g: frames 4g..4g+3 at floats 256*g + 4*row + {0,1,2,3}
            f2 xa = *(const f2 *)(fsrc), xb = *(const f2 *)(fsrc + 2);
            f4 P[2][4];
#pragma unroll
            for (int e = 0; e < 4; ++e) P[0][e] = __builtin_amdgcn_mfma_f32_4x4x1f32(A, e < 2 ? xa[e] : xb[e - 2], nz, 0, 0, 0);
            for (int n = 0; n < steps; ++n) {
#pragma unroll
                for (int g = 0; g < GR; ++g) {
                    const int cb = g & 1, nb = cb ^ 1;
                    if (g + 1 < GR) {
                        xa = *(const f2 *)(fsrc + 256 * (g + 1));
                        xb = *(const f2 *)(fsrc + 256 * (g + 1) + 2);
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        P[nb][e] = __builtin_amdgcn_mfma_f32_4x4x1f32(A, e < 2 ? xa[e] : xb[e - 2], nz, 0, 0, 0);
                    float oa, ob, oc, od;
                    step1x2(P[cb][0], P[cb][1], z0, z1, na1, na2, oa, ob);
                    step1x2(P[cb][2], P[cb][3], z0, z1, na1, na2, oc, od);
                    *(f2 *)(fdst + 256 * g) = f2{oa, ob};
                    *(f2 *)(fdst + 256 * g + 2) = f2{oc, od};
                }
            }
            res = z0 + z1;
        }
    }
    const long long t1 = clock64();
    out[blockIdx.x * 64 + lane] = res;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
    float *d;
    hipMalloc(&d, 64 * 4 * 4);
    k_layout<<<1, 64>>>(d);
    std::vector<float> h(64 * 4);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    int ok = 1;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r)
            if (h[l * 4 + r] != (float)(1 + 4 * (l / 4) + r) * 1000.0f * (1 + l)) ok = 0;
    printf("layout 4x4x1_16b: lane l reg r = A[lane 4*(l/4)+r] * B[lane l]: %s (lane 5: %g %g %g %g)\n",
           ok ? "yes" : "NO", h[20], h[21], h[22], h[23]);

    const int n = 1 << 22;
    std::vector<float> hx(n), hc(n);
    std::mt19937 rng(123);
    std::uniform_real_distribution<float> u(-1.0f, 1.0f);
    for (int i = 0; i < n; ++i) {
        hx[i] = u(rng);
        hc[i] = u(rng) * 2.0f;
        const int k = i % 89;
        if (k == 0) hx[i] = 0.0f;
        if (k == 1) hx[i] = -0.0f;
        if (k == 2) hc[i] = -0.0f;
        if (k == 3) hx[i] = 1e-38f * u(rng);             // denormal inputs
        if (k == 4) hc[i] = 3e-39f;                      // denormal coefficient
        if (k == 5) hx[i] = 1e-20f, hc[i] = 1e-20f;      // underflow
        if (k == 6) hx[i] = 3e38f, hc[i] = 10.0f;        // overflow -> inf
        if (k == 8) hx[i] = 1.5e-19f, hc[i] = 7.3e-20f;  // product in the denormal range
        if (k == 9) hx[i] = 2.5e-38f * u(rng);           // normal x, denormal products
    }
    float *dx, *dc;
    unsigned *db;
    hipMalloc(&dx, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&db, 4);
    hipMemcpy(dx, hx.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dc, hc.data(), n * 4, hipMemcpyHostToDevice);
    for (int negz = 1; negz >= 0; --negz) {
        hipMemset(db, 0, 4);
        if (negz) k_exact<true><<<n / 64, 64>>>(dx, dc, db, n);
        else k_exact<false><<<n / 64, 64>>>(dx, dc, db, n);
        unsigned bad = 0;
        hipMemcpy(&bad, db, 4, hipMemcpyDeviceToHost);
        printf("exactness 4x4x1 (C=%s0) vs v_mul_f32 over %d products: %u value mismatches, %u zero-sign mismatches\n",
               negz ? "-" : "+", n * 4, bad & 0xffff, bad >> 16);
    }

    float *cf, *out;
    long long *cyc;
    const float hcf[8] = {0.2f, -0.3f, 0.1f, -1.1f, 0.35f, 0.1f, 0.2f, 0.3f};
    hipMalloc(&cf, 32); hipMalloc(&out, 1024 * 64 * 4); hipMalloc(&cyc, 1024 * 8);
    hipMemcpy(cf, hcf, 32, hipMemcpyHostToDevice);
    const int steps = 2000, blocks = 1024;   // one wave per SIMD
    auto run = [&](auto kern, const char *name, double frames_per_granule) {
        kern<<<blocks, 64>>>(out, cf, 10, cyc);
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        kern<<<blocks, 64>>>(out, cf, steps, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<long long> hc2(blocks);
        hipMemcpy(hc2.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (auto v : hc2) s += (double)v;
        const double frames = (double)steps * GR * frames_per_granule;
        printf("%-58s %8.3f ms  %6.1f ns/frame  %6.1f clock64/frame\n", name, ms, ms * 1e6 / frames, s / blocks / frames);
    };
    run(k<0>, "mode 0 packed stereo, registers (2 chains/lane)", 2);
    run(k<3>, "mode 3 packed stereo + LDS b128 in/out", 2);
    run(k<1>, "mode 1 chain/lane, products in registers (6 VALU)", 4);
    run(k<2>, "mode 2 chain/lane, MFMA 4x4x1 products + LDS", 4);
    return 0;
}
