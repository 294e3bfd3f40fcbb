// Microbenchmark: HBM read bandwidth vs. per-lane chunk size for the
// resampler's access pattern (64 lanes = 64 streams 1280 B apart; every
// "round" each lane reads CH contiguous bytes of its stream).  Coalesced
// streaming is the reference.  Also: LDS-DMA (global_load_lds) variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int CH>   // bytes per lane per round (multiple of 16)
__global__ __launch_bounds__(256) void k_lanes(const float4 *__restrict__ in, float *out, long n_streams)
{
    const int lane = threadIdx.x & 63;
    const long wave = ((long)blockIdx.x * 256 + threadIdx.x) >> 6;
    const long s = wave * 64 + lane;                 // stream id
    if (s >= n_streams) return;
    const float4 *p = in + s * 80;                   // 1280 B per stream
    float acc = 0;
#pragma unroll
    for (int r = 0; r < 1280 / CH; ++r) {
        float4 v[CH / 16];
#pragma unroll
        for (int i = 0; i < CH / 16; ++i) v[i] = p[r * (CH / 16) + i];
#pragma unroll
        for (int i = 0; i < CH / 16; ++i) acc += v[i].x + v[i].w;
    }
    if (acc == 1234.5f) out[s] = acc;
}

// segments of SEG bytes, 1280 B apart; consecutive lanes cover a segment
// (the staging pattern of an LDS-tiled kernel: per round every SP needs SEG bytes)
template <int SEG>
__global__ __launch_bounds__(256) void k_seg(const float4 *__restrict__ in, float *out, long n_streams)
{
    constexpr int LPS = SEG / 16;                      // lanes per segment
    constexpr int SPI = 64 / LPS;                      // segments per instruction (floor)
    const int lane = threadIdx.x & 63;
    const long wave = ((long)blockIdx.x * 256 + threadIdx.x) >> 6;
    // a wave owns 64 streams and walks them round by round
    float acc = 0;
    const int seg_in = lane / LPS, off = lane % LPS;
    if (seg_in >= SPI) return;
#pragma unroll 1
    for (int r = 0; r < 1280 / SEG; ++r) {
#pragma unroll
        for (int g = 0; g < (64 + SPI - 1) / SPI; ++g) {
            const int sidx = g * SPI + seg_in;
            if (sidx < 64) {
                const long s = wave * 64 + sidx;
                if (s < n_streams) { float4 v = in[s * 80 + r * LPS + off]; acc += v.x + v.w; }
            }
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_coal(const float4 *__restrict__ in, float *out, long n16)
{
    float acc = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) {
        float4 v = in[i];
        acc += v.x + v.w;
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main()
{
    const size_t bytes = (size_t)16 << 30;           // 16 GiB, like the headline input
    float4 *in; float *out;
    if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, 1 << 28) != hipSuccess) { printf("alloc fail\n"); return 1; }
    hipMemset(in, 1, bytes);
    const long n_streams = bytes / 1280;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    auto t = [&](auto launch, const char *name) {
        launch(); hipDeviceSynchronize();
        float best = 1e9;
        for (int r = 0; r < 3; ++r) {
            hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        }
        printf("%-28s %8.3f ms  %7.1f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
    };
    const int blocks = (int)((n_streams + 255) / 256 * 64 / 64);
    t([&] { k_coal<<<256 * 16, 256>>>(in, out, bytes / 16); }, "coalesced grid-stride");
    t([&] { k_lanes<16><<<(n_streams * 64 + 255) / 256 / 64 * 1, 256>>>(in, out, n_streams); }, "lanes 1280B apart, 16B/rnd");
    t([&] { k_lanes<64><<<(n_streams * 64 + 255) / 256 / 64, 256>>>(in, out, n_streams); }, "lanes 1280B apart, 64B/rnd");
    t([&] { k_lanes<128><<<(n_streams * 64 + 255) / 256 / 64, 256>>>(in, out, n_streams); }, "lanes 1280B apart, 128B/rnd");
    t([&] { k_lanes<256><<<(n_streams * 64 + 255) / 256 / 64, 256>>>(in, out, n_streams); }, "lanes 1280B apart, 256B/rnd");
    t([&] { k_lanes<640><<<(n_streams * 64 + 255) / 256 / 64, 256>>>(in, out, n_streams); }, "lanes 1280B apart, 640B/rnd");
    const int wblocks = (int)((n_streams / 64 + 3) / 4);
    t([&] { k_seg<80><<<wblocks, 256>>>(in, out, n_streams); }, "segments 80B, 1280B apart");
    t([&] { k_seg<160><<<wblocks, 256>>>(in, out, n_streams); }, "segments 160B, 1280B apart");
    t([&] { k_seg<256><<<wblocks, 256>>>(in, out, n_streams); }, "segments 256B, 1280B apart");
    t([&] { k_seg<640><<<wblocks, 256>>>(in, out, n_streams); }, "segments 640B, 1280B apart");
    (void)blocks;
    return 0;
}
