// Microbenchmark (dev): HBM read rate of the fused kernel's LDS-DMA stream
// pattern with no compute, by stream layout and piece size.  Each wave owns
// 64 streams (lanes of the fused kernel: 8 tracks x 8 SP-run slots) and reads
// 470 x 256 B per stream (94 super-periods x 5 segments) into a 16-KiB LDS
// slot, one segment step at a time (all of a step's DMA issued, then
// vmcnt(0)), 8 waves per CU as in k_rs147_mix.  Layouts of stream q of wave w:
//   0 product: mix w/4, task w%4; track q/8 at 3.84 MB strides, SP run
//     (task*8 + q%8) * 94 SPs
//   1 SP-adjacent: at SP step i the wave's 64 lanes read 64 consecutive SPs
//     (an 80 KB region), segment j%5 of SP i*64+q
//   2 coalesced: step j of the wave = 16 KiB contiguous
//   3 wave-local runs: stream q = run q of the wave's own 7.7 MB region
// PIECE: bytes per stream per DMA piece (256: 16 lanes per stream, 4 streams
// per instruction, as the product; 512: 2 streams per instruction; 1024: 1)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int i4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int NSEG = 470;               // 256-B segments per stream
constexpr uint64_t RUN = 94ull * 1280;  // bytes of one SP run
constexpr uint64_t TRK = 480000ull * 8; // bytes of one stereo f32 track

__device__ __forceinline__ uint64_t stream_addr(int layout, int w, int q, int j)   // byte address of segment j (256 B)
{
    switch (layout) {
    case 0: {
        const int mix = w >> 2, task = w & 3, t = q >> 3, s = q & 7;
        return (uint64_t)(mix * 8 + t) * TRK + (uint64_t)(task * 8 + s) * RUN + (uint64_t)j * 256;
    }
    case 1: {
        const int sp = j / 5, m = j % 5;
        return (uint64_t)w * 64 * RUN + ((uint64_t)sp * 64 + q) * 1280 + (uint64_t)m * 256;
    }
    case 2: return (uint64_t)w * 64 * RUN + (uint64_t)j * 16384 + (uint64_t)q * 256;
    default: return (uint64_t)w * 64 * RUN + (uint64_t)q * RUN + (uint64_t)j * 256;
    }
}

// SM (output store forms, MODE & 1; the product issues 19 rounds per 5 segments,
// lane (slot lane / 8, output lane % 8) of each round's 8 outputs per slot):
//   0 b64 per round, default policy (the product)   1 the same, sc1   2 the same, nt
//   3 b128 per 2 rounds (one whole 128-B piece per slot), default   4 that, sc1   5 that, nt
//   6 256 B per slot per 4 rounds (two b128 instructions), default
//   7 b64 per round, slots on interleaved super-periods (a round's 8 pieces within 9.4 KB)
template <int SM>
__device__ __forceinline__ void out_stores(int k, int w, int lane, __amdgpu_buffer_rsrc_t ro, float acc)
{
    const int mix = w >> 2, task = w & 3;
    const int r0 = (k * 19) / 5, r1 = ((k + 1) * 19) / 5;
    const uint32_t ob = 0;   // the resource is based at the wave's mix output
    const uint32_t run = 94u * 147u;
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef float f2v __attribute__((ext_vector_type(2)));
    for (int r = r0; r < r1; ++r) {
        if constexpr (SM <= 2 || SM == 7) {
            const int sl = lane >> 3, kk = lane & 7;
            uint32_t n = (uint32_t)(task * 8 + sl) * run + (uint32_t)r * 8 + kk;
            if constexpr (SM == 7) n = (uint32_t)task * 8 * run + (uint32_t)((r / 19) * 8 + sl) * 147 + (uint32_t)(r % 19) * 8 + kk;
            __builtin_amdgcn_raw_buffer_store_b64(f2v{acc, acc}, ro, ob + n * 8u, 0, SM == 1 ? 16 : SM == 2 ? 2 : 0);
        } else if constexpr (SM >= 11 && SM <= 15) {   // b64 per round, other cache-policy bits: sc0, sc0|sc1, sc0|nt, nt|sc1, all three
            const int sl = lane >> 3, kk = lane & 7;
            const uint32_t n = (uint32_t)(task * 8 + sl) * run + (uint32_t)r * 8 + kk;
            constexpr int AUX = SM == 11 ? 1 : SM == 12 ? 17 : SM == 13 ? 3 : SM == 14 ? 18 : 19;
            __builtin_amdgcn_raw_buffer_store_b64(f2v{acc, acc}, ro, ob + n * 8u, 0, AUX);
        } else if constexpr (SM <= 5) {
            if (r & 1) {
                const int sl = lane >> 3, e = lane & 7;
                const uint32_t n = (uint32_t)(task * 8 + sl) * run + (uint32_t)(r - 1) * 8 + 2 * e;
                __builtin_amdgcn_raw_buffer_store_b128(f4v{acc, acc, acc, acc}, ro, ob + n * 8u, 0, SM == 4 ? 16 : SM == 5 ? 2 : 0);
            }
        } else if constexpr (SM == 9 || SM == 10) {   // the product's pieces, every wave inside a 16-KB (9) or 1-KB (10) footprint
            const int sl = lane >> 3, kk = lane & 7;
            const uint32_t n = SM == 9 ? (uint32_t)task * 2048u + (uint32_t)sl * 256u + (uint32_t)((r * 8 + kk) & 255)
                                       : (uint32_t)task * 128u + (uint32_t)sl * 16u + (uint32_t)((r * 8 + kk) & 15);
            __builtin_amdgcn_raw_buffer_store_b64(f2v{acc, acc}, ro, ob + n * 8u, 0, 0);
        } else if constexpr (SM == 8) {   // wave-private contiguous output, 1 KiB per instruction, ~1 per 2 rounds
            if (r & 1) {
                const uint32_t n = (uint32_t)task * 8 * run + (uint32_t)(r >> 1) * 128 + 2 * lane;
                __builtin_amdgcn_raw_buffer_store_b128(f4v{acc, acc, acc, acc}, ro, ob + n * 8u, 0, 0);
            }
        } else {
            if ((r & 3) == 3) {
                for (int i = 0; i < 2; ++i) {
                    const int sl = 4 * i + (lane >> 4), e = lane & 15;
                    const uint32_t n = (uint32_t)(task * 8 + sl) * run + (uint32_t)(r - 3) * 8 + 2 * e;
                    __builtin_amdgcn_raw_buffer_store_b128(f4v{acc, acc, acc, acc}, ro, ob + n * 8u, 0, 0);
                }
            }
        }
    }
}

template <int PIECE, int POL, int MODE = 0, int SM = 0>   // POL 0: nt, 1: default, 2: sc1; MODE bits: 1 the product's output stores, 2 its slot copies, 4 its exchange
__global__ __launch_bounds__(512) void k_dma(const char *buf, int layout, int delay, unsigned *sink, char *obuf)
{
    extern __shared__ __attribute__((aligned(16))) char lds_all[];
    const int wib = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 8 + wib;
    char *slot = lds_all + wib * 16384;
    const uint32_t ldsb = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void *)slot);
    // one resource per wave from its lowest address (every layout: < 4 GB span per wave)
    uint64_t lo = ~0ull;
    for (int q = 0; q < 64; ++q) {
        const uint64_t a = stream_addr(layout, w, q, 0);
        lo = a < lo ? a : lo;
    }
    const uint64_t mb = (uint64_t)(uintptr_t)buf + lo;
    i4 rs;
    rs.x = (int)__builtin_amdgcn_readfirstlane((uint32_t)mb);
    rs.y = (int)__builtin_amdgcn_readfirstlane((uint32_t)(mb >> 32) & 0xffffu);
    rs.z = (int)0xffffffffu;
    rs.w = 0x00020000;
    constexpr int LPS = PIECE / 16;          // lanes per stream piece
    constexpr int SPI = 64 / LPS;            // streams per instruction
    constexpr int SEGP = PIECE / 256;        // segments per piece
    float acc = 0.0f;
    // every step moves 16 KiB (16 instructions): with larger pieces a step
    // covers 64 / SEGP of the streams, in turn
#pragma unroll 1
    for (int k = 0; k < NSEG; ++k) {
        const int j = k / SEGP * SEGP, gsel = k % SEGP;
#pragma unroll
        for (int d = 0; d < ((MODE & 16) ? 0 : 16); ++d) {   // MODE 16: no DMA (the stores alone)
            const int q = gsel * (64 / SEGP) + d * SPI + lane / LPS;
            const int c = lane % LPS;        // 16-B chunk within the piece
            const uint32_t off = (uint32_t)(stream_addr(layout, w, q, j + c / 16) - lo) + (uint32_t)(c % 16) * 16u;
            const uint32_t m0 = ldsb + (uint32_t)d * 1024u;
            // (POL 3, plain loads into VGPRs by inline asm, was removed: the asm
            // result carried no vmcnt dependence, so a register was reused before
            // its load landed and the kernel faulted (illegal address, round 6).
            // VGPR-load forms are measured by tools/ubench/hbm_ceiling.hip with
            // the compiler's buffer-load builtin.)
            if constexpr (POL == 0)
                asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds" ::"s"(m0), "v"(off), "s"(rs) : "memory", "m0");
            else if constexpr (POL == 1)
                asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(off), "s"(rs) : "memory", "m0");
            else
                asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen sc1 lds" ::"s"(m0), "v"(off), "s"(rs) : "memory", "m0");
        }
        if constexpr (MODE & 1)
            out_stores<SM>(k, w, lane, __builtin_amdgcn_make_buffer_rsrc(obuf + (size_t)(w >> 2) * 441000u * 8u, (short)0, (int)(441000u * 8u), 0x00020000), acc);
        if constexpr (MODE & 8)   // the step's stores younger than its DMA: wait for the DMA only (<= 4 stores after it)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (MODE & 2) {   // the slot -> register copy: 16 ds_read_b128 per segment
            float4 t = float4{0, 0, 0, 0};
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float4 v;
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"((uint32_t)(uintptr_t)(lds_void *)(slot + (lane >> 2) * 1024 + (lane & 3) * 256 + ((i + lane) & 15) * 16)), "n"(0));
                t.x += v.x; t.w += v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc += t.x + t.w;
        }
        if constexpr (MODE & 4) {   // the exchange: ~29 ds_write_b64 + 30 ds_read_b64 per segment into 4 KiB
            char *X = lds_all + 8 * 16384 + wib * 4096;
            for (int i = 0; i < 29; ++i) {
                asm volatile("ds_write_b64 %0, %1" :: "v"((uint32_t)(uintptr_t)(lds_void *)(X + (i & 7) * 512 + ((lane + 4 * (i & 7)) & 63) * 8)), "v"(float2{acc, acc}) : "memory");
            }
            float2 t = float2{0, 0};
            for (int i = 0; i < 30; ++i) {
                float2 v;
                asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)(lds_void *)(X + (i & 7) * 512 + ((lane * 8 + i) & 63) * 8)) : "memory");
                t.x += v.x;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc += t.x;
        }
        acc += *(const float *)(slot + lane * 16);
        for (int i = 0; i < delay; ++i) __builtin_amdgcn_s_sleep(8);
    }
    if (acc == 1234.5f) sink[0] = 1;
}

int main(int argc, char **argv)
{
    const size_t bytes = (size_t)2048 * 64 * RUN + (1 << 20);
    char *buf;
    unsigned *sink;
    char *obuf;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess ||
        hipMalloc(&obuf, (size_t)512 * 441000 * 8) != hipSuccess) {
        printf("alloc fail\n");
        return 1;
    }
    hipMemset(buf, 1, bytes);
    const double moved = 2048.0 * 64 * NSEG * 256;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](auto kern, const char *name, int layout, int delay) {
        hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 20480);
        kern<<<256, 512, 8 * 20480>>>(buf, layout, delay, sink, obuf);
        // every launch checked: a variant that fails prints FAILED, never the
        // previous line's time (round 5's VGPR-load line did)
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            printf("%-10s layout %d delay %3d: FAILED (%s)\n", name, layout, delay, hipGetErrorString(e));
            fflush(stdout);
            (void)hipGetLastError();
            return;
        }
        float best = 1e9;
        for (int r = 0; r < 3; ++r) {
            hipEventRecord(a);
            kern<<<256, 512, 8 * 20480>>>(buf, layout, delay, sink, obuf);
            e = hipGetLastError();
            hipEventRecord(b);
            if (e == hipSuccess) e = hipEventSynchronize(b);
            if (e != hipSuccess) {
                printf("%-10s layout %d delay %3d: FAILED (%s)\n", name, layout, delay, hipGetErrorString(e));
                fflush(stdout);
                (void)hipGetLastError();
                return;
            }
            float ms;
            hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        printf("%-10s layout %d delay %3d: %8.3f ms %8.1f GB/s\n", name, layout, delay, best, moved / (best * 1e-3) / 1e9);
        fflush(stdout);
    };
    if (argc > 1 && argv[1][0] == 'p') {   // store cache-policy bits
        run(k_dma<256, 0, 0>, "no stores", 0, 0);
        run(k_dma<256, 0, 1, 0>, "b64 def", 0, 0);
        run(k_dma<256, 0, 1, 11>, "b64 sc0", 0, 0);
        run(k_dma<256, 0, 1, 12>, "b64 sc0 sc1", 0, 0);
        run(k_dma<256, 0, 1, 13>, "b64 sc0 nt", 0, 0);
        run(k_dma<256, 0, 1, 14>, "b64 sc1 nt", 0, 0);
        run(k_dma<256, 0, 1, 15>, "b64 sc0 sc1 nt", 0, 0);
        run(k_dma<256, 2, 1, 0>, "sc1 loads + b64 def", 0, 0);
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'q') {   // the product's stores beside other read geometries
        run(k_dma<256, 0, 1, 0>, "p256 + b64", 0, 0);
        run(k_dma<512, 0, 1, 0>, "p512 + b64", 0, 0);
        run(k_dma<1024, 0, 1, 0>, "p1024 + b64", 0, 0);
        run(k_dma<1024, 0, 1, 0>, "p1024 + b64", 3, 0);
        for (int layout = 1; layout < 4; ++layout) run(k_dma<256, 0, 1, 0>, "p256 + b64", layout, 0);
        run(k_dma<256, 0, 1, 8>, "coalesced + 1K stores", 2, 0);
        return 0;
    }
    if (argc > 1 && argv[1][0] == 's') {   // output store forms beside the stream
        run(k_dma<256, 0, 0>, "no stores", 0, 0);
        run(k_dma<256, 0, 1, 0>, "b64 def", 0, 0);
        run(k_dma<256, 0, 1, 1>, "b64 sc1", 0, 0);
        run(k_dma<256, 0, 1, 2>, "b64 nt", 0, 0);
        run(k_dma<256, 0, 1, 3>, "b128 def", 0, 0);
        run(k_dma<256, 0, 1, 4>, "b128 sc1", 0, 0);
        run(k_dma<256, 0, 1, 5>, "b128 nt", 0, 0);
        run(k_dma<256, 0, 1, 6>, "256B def", 0, 0);
        run(k_dma<256, 0, 1, 7>, "b64 ilv", 0, 0);
        run(k_dma<256, 1, 1, 0>, "b64 def, def loads", 0, 0);
        run(k_dma<256, 0, 9, 0>, "b64 def, acks not waited", 0, 0);
        run(k_dma<256, 0, 9, 3>, "b128 def, acks not waited", 0, 0);
        run(k_dma<256, 0, 9, 0>, "b64 def, acks not waited", 0, 8);
        run(k_dma<256, 0, 1, 8>, "1K contiguous", 0, 0);
        run(k_dma<256, 0, 1, 9>, "b64 small footprint", 0, 0);
        run(k_dma<256, 0, 1, 10>, "b64 1K footprint", 0, 0);
        run(k_dma<256, 0, 0, 0>, "coalesced, no stores", 2, 0);
        run(k_dma<256, 0, 1, 0>, "coalesced + b64 stores", 2, 0);
        run(k_dma<256, 0, 1, 8>, "coalesced + 1K stores", 2, 0);
        run(k_dma<256, 0, 17, 0>, "b64 stores alone", 0, 0);
        run(k_dma<256, 0, 17, 8>, "1K contig stores alone", 0, 0);
        return 0;
    }
    if (argc > 1) {   // the product's other traffic beside its DMA stream
        run(k_dma<256, 0, 0>, "base", 0, 0);
        run(k_dma<256, 0, 1>, "+stores", 0, 0);
        run(k_dma<256, 0, 2>, "+copies", 0, 0);
        run(k_dma<256, 0, 4>, "+exchange", 0, 0);
        run(k_dma<256, 0, 7>, "+all", 0, 0);
        run(k_dma<256, 0, 7>, "+all", 0, 8);
        run(k_dma<256, 0, 1>, "+stores", 0, 8);
        return 0;
    }
    for (int layout = 0; layout < 4; ++layout) run(k_dma<256, 0>, "p256 nt", layout, 0);
    for (int layout : {0, 3}) run(k_dma<512, 0>, "p512 nt", layout, 0);
    for (int layout : {0, 3}) run(k_dma<1024, 0>, "p1024 nt", layout, 0);
    run(k_dma<256, 1>, "p256 def", 0, 0);
    run(k_dma<256, 2>, "p256 sc1", 0, 0);
    run(k_dma<512, 1>, "p512 def", 0, 0);
    for (int d : {4, 8, 16}) run(k_dma<256, 0>, "p256 nt", 0, d);
    for (int d : {4, 8, 16}) run(k_dma<256, 0>, "p256 nt", 1, d);
    return 0;
}
