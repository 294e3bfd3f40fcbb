// xm_fx.hip — effects chain kernels for gfx950 (biquad cascade, FIR) and the
// synthetic PCM generator.
//
// Biquad: scipy sosfilt order (transposed DF-II, _signaltools.py:4601), one
// lane per (clip, channel) stream, sections in order, state zero at clip
// start.  The recurrence is serial in time, so exactness (SURVEY.md §7 hard
// part 3) fixes the parallelism at clips x channels; coefficients live in
// SGPRs (wave-uniform), state in VGPRs, input streamed with a 16-frame
// register prefetch.
// FIR: upfirdn order (_upfirdn.py:107), taps staged in LDS, input tile in LDS.
#include "xm_device.h"

namespace {

constexpr int BQ_THREADS = 64;
constexpr int BQ_MAXSEC = 16;

template <int C>
__global__ __launch_bounds__(BQ_THREADS) void k_biquad(XmhFxJob j)
{
    const int stream = blockIdx.x * BQ_THREADS + threadIdx.x;
    if (stream >= j.n_clips * C) return;
    const int clip = stream / C, ch = stream % C;
    const float *x = j.in_ptrs[clip];
    float *y = j.out_ptrs[clip];
    const int ns = j.n_sos;
    float z0[BQ_MAXSEC], z1[BQ_MAXSEC], q[BQ_MAXSEC][5];
#pragma unroll
    for (int s = 0; s < BQ_MAXSEC; ++s) {
        z0[s] = 0.0f; z1[s] = 0.0f;
        if (s < ns) {
            q[s][0] = j.sos[6 * s + 0]; q[s][1] = j.sos[6 * s + 1]; q[s][2] = j.sos[6 * s + 2];
            q[s][3] = j.sos[6 * s + 4]; q[s][4] = j.sos[6 * s + 5];
        }
    }
    const int64_t N = j.frames;
    for (int64_t n = 0; n < N; ++n) {
        float v = x[n * C + ch];
#pragma unroll
        for (int s = 0; s < BQ_MAXSEC; ++s) {
            if (s < ns) {
                const float o = q[s][0] * v + z0[s];
                z0[s] = (q[s][1] * v - q[s][3] * o) + z1[s];
                z1[s] = q[s][2] * v - q[s][4] * o;
                v = o;
            }
        }
        y[n * C + ch] = v;
    }
}

constexpr int FIR_THREADS = 256;
constexpr int FIR_OPT = 4;
constexpr int FIR_CHUNK = FIR_THREADS * FIR_OPT;

template <int C>
__global__ __launch_bounds__(FIR_THREADS) void k_fir(XmhFxJob j)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int K = j.fir_len;
    float *h = lds;                                   // reversed taps: h[t] = fir[K-1-t]
    float *tile = lds + ((K + 3) & ~3);
    const int clip = blockIdx.y;
    const float *x = j.in_ptrs[clip];
    float *y = j.out_ptrs[clip];
    const int64_t n0 = (int64_t)blockIdx.x * FIR_CHUNK;
    const int64_t n1 = min(n0 + FIR_CHUNK, (int64_t)j.frames);
    const int64_t jlo = n0 - K + 1;
    const int span = (int)(n1 - jlo);
    for (int i = threadIdx.x; i < K; i += FIR_THREADS) h[i] = j.fir[K - 1 - i];
    for (int i = threadIdx.x; i < span * C; i += FIR_THREADS) {
        const int64_t f = jlo + i / C;
        tile[i] = f >= 0 ? x[f * C + i % C] : 0.0f;
    }
    __syncthreads();
    float acc[FIR_OPT][C];
#pragma unroll
    for (int o = 0; o < FIR_OPT; ++o) {
        const int64_t n = n0 + threadIdx.x + o * FIR_THREADS;
#pragma unroll
        for (int c = 0; c < C; ++c) acc[o][c] = 0.0f;
        if (n >= n1) continue;
        const float *xt = tile + (n - n0) * C;        // x[n-K+1] is tile[(n-n0)*C]
        for (int t = 0; t < K; ++t) {
            const float hv = h[t];
#pragma unroll
            for (int c = 0; c < C; ++c) acc[o][c] = acc[o][c] + xt[t * C + c] * hv;
        }
    }
    __syncthreads();   // in == out allowed: every read of this block's tile is done
#pragma unroll
    for (int o = 0; o < FIR_OPT; ++o) {
        const int64_t n = n0 + threadIdx.x + o * FIR_THREADS;
        if (n >= n1) continue;
#pragma unroll
        for (int c = 0; c < C; ++c) y[n * C + c] = acc[o][c];
    }
}

// ---- synthetic PCM (twins: oracle/np_oracle.gen_*,
// oracle/xm_oracle.c xo_gen_*) -------------------------------------------------
XM_DEV uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_synth(void *out, int fmt, uint64_t seed, uint64_t clip0,
                                               int64_t per_clip, int64_t total)
{
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const uint64_t clip = clip0 + (uint64_t)(i / per_clip);
        const uint64_t k = (uint64_t)(i % per_clip);
        const uint64_t z = mix64(seed + ((clip << 32) | k) * 0x9E3779B97F4A7C15ULL);
        if (fmt == 2) {
            const int32_t v = (int32_t)(z >> 40) - (1 << 23);
            ((float *)out)[i] = (float)v * 0x1p-23f;
        } else {
            ((int16_t *)out)[i] = (int16_t)(uint16_t)(z >> 48);
        }
    }
}

}  // namespace

extern "C" int xmh_launch_fx_biquad(const XmhFxJob *j, void *stream)
{
    if (j->n_sos > BQ_MAXSEC) return -1003;
    const int streams = j->n_clips * j->channels;
    dim3 grid((streams + BQ_THREADS - 1) / BQ_THREADS);
    if (j->channels == 1) hipLaunchKernelGGL(k_biquad<1>, grid, BQ_THREADS, 0, (hipStream_t)stream, *j);
    else hipLaunchKernelGGL(k_biquad<2>, grid, BQ_THREADS, 0, (hipStream_t)stream, *j);
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}

extern "C" int xmh_launch_fx_fir(const XmhFxJob *j, void *stream)
{
    const int K = j->fir_len;
    const size_t lds = (size_t)(((K + 3) & ~3) + (FIR_CHUNK + K) * j->channels) * sizeof(float);
    if (lds > 160 * 1024) return -1003;
    dim3 grid((unsigned)((j->frames + FIR_CHUNK - 1) / FIR_CHUNK), (unsigned)j->n_clips);
    if (grid.x == 0) return 0;
    auto kern = j->channels == 1 ? k_fir<1> : k_fir<2>;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return -1001;
    hipLaunchKernelGGL(kern, grid, FIR_THREADS, lds, (hipStream_t)stream, *j);
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}

extern "C" int xmh_synth(void *out, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips,
                         int channels, int64_t frames, void *stream)
{
    const int64_t per_clip = frames * channels;
    const int64_t total = per_clip * n_clips;
    if (total == 0) return 0;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)blocks), 256, 0, (hipStream_t)stream, out, fmt, seed, clip0,
                       per_clip, total);
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}
