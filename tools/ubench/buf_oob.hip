// Dev probe: how does a raw buffer_load_dwordx4 treat a 16-B access that is
// partly past num_records (per dword zeroing, or the whole access)?  Also the
// LDS-DMA form (buffer_load_dwordx4 ... lds).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i4 __attribute__((ext_vector_type(4)));
__global__ void k(const float *p, float *o, unsigned nrec, unsigned soff)
{
    __shared__ float4 s[64];
    i4 rs;
    const unsigned long long b = (unsigned long long)p;
    rs.x = (int)(unsigned)b;
    rs.y = (int)((unsigned)(b >> 32) & 0xffffu);
    rs.z = (int)nrec;
    rs.w = 0x00020000;
    const unsigned off = threadIdx.x * 4;   // lane l reads bytes [4l, 4l + 16)
    float4 v;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(off), "s"(rs), "s"(soff) : "memory");
    o[threadIdx.x * 4 + 0] = v.x; o[threadIdx.x * 4 + 1] = v.y; o[threadIdx.x * 4 + 2] = v.z; o[threadIdx.x * 4 + 3] = v.w;
    const unsigned lb = (unsigned)(unsigned long long)(__attribute__((address_space(3))) void *)s;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_waitcnt vmcnt(0)"
                 :: "s"(lb), "v"(off), "s"(rs), "s"(soff) : "memory", "m0");
    __syncthreads();
    const float4 w = s[threadIdx.x];
    o[256 + threadIdx.x * 4 + 0] = w.x; o[256 + threadIdx.x * 4 + 1] = w.y; o[256 + threadIdx.x * 4 + 2] = w.z; o[256 + threadIdx.x * 4 + 3] = w.w;
}
int main()
{
    float h[64], *d, *o, r[512];
    for (int i = 0; i < 64; ++i) h[i] = (float)(i + 1);
    (void)hipMalloc(&d, 256);
    (void)hipMalloc(&o, 2048);
    (void)hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
    for (unsigned so : {0u, 8u}) {
    k<<<1, 8>>>(d, o, 20, so);   // 5 dwords in range
    (void)hipMemcpy(r, o, 2048, hipMemcpyDeviceToHost);
    printf("soffset %u\n", so);
    for (int l = 0; l < 8; ++l)
        printf("lane %d (bytes %2d..%2d): vgpr %g %g %g %g | lds %g %g %g %g\n", l, 4 * l, 4 * l + 15, r[4 * l],
               r[4 * l + 1], r[4 * l + 2], r[4 * l + 3], r[256 + 4 * l], r[257 + 4 * l], r[258 + 4 * l], r[259 + 4 * l]);
    }
    return 0;
}
