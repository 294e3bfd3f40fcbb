// xm_fx.hip — effects chain kernels for gfx950 (biquad cascade, FIR) and the
// synthetic PCM generator.
//
// Biquad: scipy sosfilt order (transposed DF-II, _signaltools.py:4601),
// sections in order, state zero at clip start.  The recurrence is serial in
// time, so exactness (SURVEY.md §7 hard part 3) limits the parallelism to
// clips x sections: k_biquad_lanes gives each (clip, section) its own lane
// and chains the sections through LDS chunks (see the comment at the kernel).
// FIR: upfirdn order (_upfirdn.py:107), taps staged in LDS, input tile in LDS.
#include <stdlib.h>
#include "xm_device.h"

namespace {

constexpr int BQ_MAXSEC = 15;   // XM_MAX_SOS (src/xm_internal.h): >= 4 clips per wave

// Section-pipelined cascade.  The recurrence of one section is serial in
// time, so the only parallelism that keeps sosfilt's rounding is across
// clips and across sections: lane = (clip k, section s), lane = k*NS + s,
// 64 / NS clips per wave (stereo (L, R) ride in one packed v_pk_* pair).
// Time advances in chunks of CH frames; at step i lane s filters chunk i - s,
// so the NS sections of a clip work on NS consecutive chunks at once and the
// per-sample recurrence (4 dependent ops) is the only serial chain.
//   section 0   reads its clip from HBM two chunks ahead into registers and
//               passes the chunk through LDS like every other section;
//   section s   reads the chunk lane - 1 (section s - 1) wrote one step earlier;
//   last        stores to global memory instead of LDS.
// One wave, so LDS needs no barrier: every read of a step precedes, in
// program order, every write of that step.
// In LDS a chunk is [CH / FPL][64 lanes][FPL frames] (16 B per lane-granule).
template <int C>
struct BqVec;
template <>
struct BqVec<1> { typedef float T; };
template <>
struct BqVec<2> { typedef float T __attribute__((ext_vector_type(2))); };
typedef float bq_f4 __attribute__((ext_vector_type(4)));

template <int C, int CH, bool ST>
__global__ __launch_bounds__(64) void k_biquad_lanes(XmhFxJob j)
{
    typedef typename BqVec<C>::T V;
    typedef const __attribute__((address_space(1))) bq_f4 gcf4;
    typedef __attribute__((address_space(1))) bq_f4 gf4;
    constexpr int FPL = 4 / C;                     // frames per 16-B granule
    constexpr int G = CH / FPL;                    // granules per chunk
    __shared__ bq_f4 in_buf[G][64];                // section 0's input
    __shared__ bq_f4 sec_buf[G][64];               // output of lane's section (s < NS - 1)
    const int ns = j.n_sos;
    const int kpw = 64 / ns;                       // clips per wave
    const int lane = threadIdx.x;
    const int s = lane % ns, kk = lane / ns;
    const int clip = blockIdx.x * kpw + kk;
    const bool valid = kk < kpw && clip < j.n_clips;
    const bool first = s == 0, last = s == ns - 1;
    const int64_t N = j.frames;
    const int64_t nchunk = (N + CH - 1) / CH;
    const float *x = valid ? j.in_ptrs[clip] : nullptr;
    float *y = valid ? j.out_ptrs[clip] : nullptr;
    const bq_f4 *src = first ? &in_buf[0][lane] : &sec_buf[0][(lane + 63) & 63];

    const float *q = j.sos + 6 * s;                 // this lane's section, state zero at clip start
    const float b0 = q[0], b1 = q[1], b2 = q[2], a1 = q[4], a2 = q[5];
    V z0 = V(0.0f), z1 = V(0.0f);
    float *st = (ST && valid) ? j.state + ((size_t)clip * ns + s) * 2 * C : nullptr;
    if (ST && st) {                                // streaming: continue from the previous block
        if constexpr (C == 2) { z0 = V{st[0], st[1]}; z1 = V{st[2], st[3]}; }
        else { z0 = st[0]; z1 = st[1]; }
    }

    bq_f4 pa[G], pb[G];                            // section 0: chunks i and i + 1 in flight
    auto load = [&](bq_f4 (&d)[G], int64_t c) {
        if (!(first && valid && c < nchunk) || (j.dev_flags & 1)) return;   // dev_flags 1: attribution, no loads
        const float *xc = x + (size_t)C * (size_t)(c * CH);
        if ((c + 1) * CH <= N && (((uintptr_t)xc) & 15) == 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) d[g] = ((gcf4 *)xc)[g];
        } else {
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    d[g][e] = (c * CH + g * FPL) * C + e < N * C ? xc[g * 4 + e] : 0.0f;
        }
    };
    auto step = [&](int64_t i, bq_f4 (&cur)[G]) {
        if (first) {
#pragma unroll
            for (int g = 0; g < G; ++g) in_buf[g][lane] = cur[g];
        }
        load(cur, i + 2);                          // refill: chunk i + 2
        const int64_t c = i - s;                   // chunk this lane filters
        bq_f4 v4[G];
#pragma unroll
        for (int g = 0; g < G; ++g) v4[g] = src[g * 64];
        if (c >= 0 && c < nchunk) {
            // the last chunk's frames past N are zero padding: with a state
            // to carry they must not advance the recurrence
            const bool tail = ST && st && (c + 1) * CH > N;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                bq_f4 r;
#pragma unroll
                for (int e = 0; e < FPL; ++e) {
                    V v;
                    if constexpr (C == 2) v = V{v4[g][2 * e], v4[g][2 * e + 1]};
                    else v = v4[g][e];
                    const V o = b0 * v + z0;              // sosfilt (_sosfilt.pyx) order
                    if (tail && c * CH + g * FPL + e >= N) {
                        // padding frame: output unused, state kept
                    } else {
                        z0 = (b1 * v - a1 * o) + z1;
                        z1 = b2 * v - a2 * o;
                    }
                    if constexpr (C == 2) { r[2 * e] = o.x; r[2 * e + 1] = o.y; }
                    else r[e] = o;
                }
                v4[g] = r;
            }
            if (!last) {
#pragma unroll
                for (int g = 0; g < G; ++g) sec_buf[g][lane] = v4[g];
            } else if (valid) {
                float *yc = y + (size_t)C * (size_t)(c * CH);
                if ((c + 1) * CH <= N && (((uintptr_t)yc) & 15) == 0) {
#pragma unroll
                    for (int g = 0; g < G; ++g) ((gf4 *)yc)[g] = v4[g];
                } else {
#pragma unroll
                    for (int g = 0; g < G; ++g)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if ((c * CH + g * FPL) * C + e < N * C) yc[g * 4 + e] = v4[g][e];
                }
            }
        }
    };
    load(pa, 0);
    load(pb, 1);
    const int64_t steps = nchunk + ns - 1;
    // Lane s reads, at step i, what lane s - 1 wrote at step i - 1: a
    // cross-lane hand-off through LDS.  The wave barrier between steps orders
    // every LDS access of step i before every one of step i + 1 for the
    // compiler as well (free in a one-wave workgroup).
    for (int64_t i = 0; i < steps; i += 2) {
        step(i, pa);
        __builtin_amdgcn_wave_barrier();
        if (i + 1 < steps) step(i + 1, pb);
        __builtin_amdgcn_wave_barrier();
    }
    if (ST && st) {
        if constexpr (C == 2) { st[0] = z0.x; st[1] = z0.y; st[2] = z1.x; st[3] = z1.y; }
        else { st[0] = z0; st[1] = z1; }
    }
}

// Stereo cascade with one channel per lane: lane = (clip k, channel ch,
// section s) = (k*2 + ch)*NS + s, 64 / (2*NS) clips per wave.  Same chunked
// section pipeline as k_biquad_lanes, but the recurrence runs on plain fp32
// ops: a wave64 v_pk_*_f32 issues in ~4.3 clk per SIMD against ~2.4 clk for
// v_mul/v_add_f32 (tools/ubench/valu_rate.hip), and a lane's per-frame
// instruction stream (9 ops around a 4-op dependent chain) was expected to
// bound the time.  Measured on config 4 it is slower (EQ 23.3 ms against 20.3
// for packed lanes), so it is kept for A/B only
// (XM_BQ_SPLIT=1); the product uses k_biquad_lanes.  Arithmetic per channel is
// sosfilt's, unchanged.  Section 0 loads whole interleaved granules (both
// channel lanes read the same 32 B) and keeps its channel; the last section
// stores its channel's samples (the two channel lanes fill each 8-B frame).
template <int CH, bool ST>
__global__ __launch_bounds__(64) void k_biquad_split(XmhFxJob j)
{
    typedef const __attribute__((address_space(1))) bq_f4 gcf4;
    constexpr int G = CH / 4;                      // mono granules (4 frames) per chunk
    __shared__ bq_f4 in_buf[G][64];
    __shared__ bq_f4 sec_buf[G][64];
    const int ns = j.n_sos;
    const int lpc = 2 * ns;                        // lanes per clip
    const int kpw = 64 / lpc;
    const int lane = threadIdx.x;
    const int s = lane % ns, ch = (lane / ns) & 1, kk = lane / lpc;
    const int clip = blockIdx.x * kpw + kk;
    const bool valid = kk < kpw && clip < j.n_clips;
    const bool first = s == 0, last = s == ns - 1;
    const int64_t N = j.frames;
    const int64_t nchunk = (N + CH - 1) / CH;
    const float *x = valid ? j.in_ptrs[clip] : nullptr;
    float *y = valid ? j.out_ptrs[clip] : nullptr;
    const bq_f4 *src = first ? &in_buf[0][lane] : &sec_buf[0][(lane + 63) & 63];

    const float *q = j.sos + 6 * s;
    const float b0 = q[0], b1 = q[1], b2 = q[2], a1 = q[4], a2 = q[5];
    float z0 = 0.0f, z1 = 0.0f;
    float *st = (ST && valid) ? j.state + ((size_t)clip * ns + s) * 4 : nullptr;   // [z0 L,R][z1 L,R]
    if (ST && st) { z0 = st[ch]; z1 = st[2 + ch]; }

    bq_f4 pa[2 * G], pb[2 * G];                    // raw interleaved granules, chunks i and i + 1
    auto load = [&](bq_f4 (&d)[2 * G], int64_t c) {
        if (!(first && valid && c < nchunk)) return;
        const float *xc = x + (size_t)2 * (size_t)(c * CH);
        if ((c + 1) * CH <= N && (((uintptr_t)xc) & 15) == 0) {
#pragma unroll
            for (int g = 0; g < 2 * G; ++g) d[g] = ((gcf4 *)xc)[g];
        } else {
#pragma unroll
            for (int g = 0; g < 2 * G; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    d[g][e] = (c * CH) * 2 + g * 4 + e < N * 2 ? xc[g * 4 + e] : 0.0f;
        }
    };
    auto step = [&](int64_t i, bq_f4 (&cur)[2 * G]) {
        if (first) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const bq_f4 u = cur[2 * g], w = cur[2 * g + 1];
                in_buf[g][lane] = ch ? bq_f4{u[1], u[3], w[1], w[3]} : bq_f4{u[0], u[2], w[0], w[2]};
            }
        }
        load(cur, i + 2);
        const int64_t c = i - s;
        bq_f4 v4[G];
#pragma unroll
        for (int g = 0; g < G; ++g) v4[g] = src[g * 64];
        if (c >= 0 && c < nchunk) {
            const bool tail = ST && st && (c + 1) * CH > N;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                bq_f4 r;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = v4[g][e];
                    const float o = b0 * v + z0;          // sosfilt (_sosfilt.pyx) order
                    if (!(tail && c * CH + g * 4 + e >= N)) {
                        z0 = (b1 * v - a1 * o) + z1;
                        z1 = b2 * v - a2 * o;
                    }
                    r[e] = o;
                }
                v4[g] = r;
            }
            if (!last) {
#pragma unroll
                for (int g = 0; g < G; ++g) sec_buf[g][lane] = v4[g];
            } else if (valid) {
                float *yc = y + (size_t)2 * (size_t)(c * CH) + ch;
                if ((c + 1) * CH <= N) {
#pragma unroll
                    for (int g = 0; g < G; ++g)
#pragma unroll
                        for (int e = 0; e < 4; ++e) yc[(g * 4 + e) * 2] = v4[g][e];
                } else {
#pragma unroll
                    for (int g = 0; g < G; ++g)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (c * CH + g * 4 + e < N) yc[(g * 4 + e) * 2] = v4[g][e];
                }
            }
        }
    };
    load(pa, 0);
    load(pb, 1);
    const int64_t steps = nchunk + ns - 1;
    for (int64_t i = 0; i < steps; i += 2) {   // cross-lane LDS hand-off: see k_biquad_lanes
        step(i, pa);
        __builtin_amdgcn_wave_barrier();
        if (i + 1 < steps) step(i + 1, pb);
        __builtin_amdgcn_wave_barrier();
    }
    if (ST && st) { st[ch] = z0; st[2 + ch] = z1; }
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
        tile[i] = f >= 0 ? x[f * C + i % C]
                         : (j.hist_in ? j.hist_in[((int64_t)clip * (K - 1) + (K - 1 + f)) * C + i % C] : 0.0f);
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

// Streaming FIR: the K-1 frames that precede the next block, from the old
// history and this block's input (run before the FIR so in == out is safe).
template <int C>
__global__ __launch_bounds__(256) void k_fir_hist(XmhFxJob j)
{
    const int K1 = j.fir_len - 1;
    const int clip = blockIdx.y;
    const float *x = j.in_ptrs[clip];
    for (int i = blockIdx.x * 256 + threadIdx.x; i < K1 * C; i += gridDim.x * 256) {
        const int64_t p = j.frames - K1 + i / C;     // block-relative frame
        j.hist_out[(int64_t)clip * K1 * C + i] =
            p >= 0 ? x[p * C + i % C] : j.hist_in[((int64_t)clip * K1 + K1 + p) * C + i % C];
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
    if (j->n_sos < 1 || j->n_sos > BQ_MAXSEC || (j->channels != 1 && j->channels != 2)) return -1003;
    if (j->n_clips == 0 || j->frames == 0) return 0;

    // 64-frame chunks: half the per-chunk LDS hand-offs of 32 and one chunk
    // more of compute to cover each prefetch (config 4: 24.06 -> 22.83 ms)
    auto kern = j->state ? (j->channels == 1 ? k_biquad_lanes<1, 64, true> : k_biquad_lanes<2, 64, true>)
                         : (j->channels == 1 ? k_biquad_lanes<1, 64, false> : k_biquad_lanes<2, 64, false>);
    int lpc = j->n_sos;                                // lanes per clip
    XmhFxJob jj = *j;
    jj.dev_flags = 0;
#ifdef XM_FX_DEVKNOBS
    // dev builds only (`make ablate`): A/B and attribution knobs.  XM_FX_DEV=1
    // skips section 0's loads (wrong results by design), so the shipped
    // library never reads these variables.
    if (const char *c = getenv("XM_BQ_CH"); c && atoi(c) == 32)   // the previous chunk length
        kern = j->state ? (j->channels == 1 ? k_biquad_lanes<1, 32, true> : k_biquad_lanes<2, 32, true>)
                        : (j->channels == 1 ? k_biquad_lanes<1, 32, false> : k_biquad_lanes<2, 32, false>);
    if (j->channels == 2 && getenv("XM_BQ_SPLIT")) {   // one channel per lane (measured slower)
        kern = j->state ? k_biquad_split<32, true> : k_biquad_split<32, false>;
        lpc = 2 * j->n_sos;
    }
    if (const char *d = getenv("XM_FX_DEV")) jj.dev_flags = atoi(d);
#endif
    const int kpw = 64 / lpc;
    dim3 grid((unsigned)((j->n_clips + kpw - 1) / kpw));
    hipLaunchKernelGGL(kern, grid, dim3(64), 0, (hipStream_t)stream, jj);
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}

extern "C" int xmh_launch_fx_fir(const XmhFxJob *j, void *stream)
{
    const int K = j->fir_len;
    const size_t lds = (size_t)(((K + 3) & ~3) + (FIR_CHUNK + K) * j->channels) * sizeof(float);
    if (lds > 160 * 1024) return -1003;
    dim3 grid((unsigned)((j->frames + FIR_CHUNK - 1) / FIR_CHUNK), (unsigned)j->n_clips);
    if (grid.x == 0) return 0;
    if (j->hist_in && K > 1) {                        // streaming: next block's history first
        if (!j->hist_out || j->hist_out == j->hist_in) return -22;
        auto hk = j->channels == 1 ? k_fir_hist<1> : k_fir_hist<2>;
        hipLaunchKernelGGL(hk, dim3((unsigned)((K - 1) * j->channels + 255) / 256, (unsigned)j->n_clips), 256, 0,
                           (hipStream_t)stream, *j);
        if (hipGetLastError() != hipSuccess) return -1001;
    }
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
