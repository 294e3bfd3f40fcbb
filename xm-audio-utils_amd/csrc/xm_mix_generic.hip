// xm_mix_generic.hip — generic gfx950 kernels for any rate pair / channel
// count / track count: LDS-staged polyphase resample + gain + ordered mix, and
// the no-resample integer (s16 Q15) and fp32 mixes.
//
// Arithmetic: include/xm_audio_common.h (pinned to scipy 1.15.3 resample_poly,
// SURVEY.md §8(a) a2/a3/a6/a7).  The headline 48k->44.1k stereo fp32 path has
// its own kernel (xm_resample_fast.hip); this file is the reference-order
// fallback every other configuration uses, and the s16 mixer (config 3).
#include <stdio.h>
#include <stdlib.h>
#include "xm_device.h"

namespace {

constexpr int GEN_THREADS = 256;
constexpr int GEN_OPT = 4;                          // outputs per thread per block
constexpr int GEN_CHUNK = GEN_THREADS * GEN_OPT;    // output frames per block
// LDS stride of a phase row of H.  The lanes of a wave read different
// phases: an even stride put them on a fraction of the banks (T = 44 at
// 147/320 with 8-B reads: SQ_LDS_BANK_CONFLICT 58 % of the LDS cycles,
// profiles/r4_v_generic_pmc.json).  T = 4 x odd keeps T and reads 16 B (4
// taps) at a time, conflict-free bank quads; other even T pad to T + 1 (odd);
// odd T stays (padding odd T to 4 x odd cost more in table staging and
// occupancy than it saved: 22.05k -> 48k stereo 9.65 -> 11.2 ms)
__host__ __device__ inline int gen_row_stride(int T) { return T % 8 == 4 ? T : (T | 1); }

// Input / output layouts and formats (XmhMixJob.io_flags, whole clips only).
// Input sample (frame f, channel c) of a track of N frames: interleaved at
// f*C + c, planar at c*N + f; in the mix format, or converted from the other
// one (XMH_IO_IN_CONV): an f32 mix reads s16 as x * 2^-15 (exact), an s16
// mix reads f32 as sat16(rint(x * 32768)).  Element size of the input:
template <bool S16>
XM_DEV int xm_in_elem(const XmhMixJob &j) { return ((j.io_flags & XMH_IO_IN_CONV) != 0) != S16 ? 2 : 4; }
XM_DEV int64_t xm_in_idx(const XmhMixJob &j, int64_t f, int c, int C)
{
    return (j.io_flags & XMH_IO_IN_PLANAR) ? (int64_t)c * j.frames_in + f : f * C + c;
}
XM_DEV int64_t xm_out_idx(const XmhMixJob &j, int64_t m, int c, int C)
{
    return (j.io_flags & XMH_IO_OUT_PLANAR) ? (int64_t)c * j.frames_out + m : m * C + c;
}
// the sample as the f32 mix sees it
XM_DEV float xm_in_f32(const XmhMixJob &j, const void *x, int64_t i)
{
    return (j.io_flags & XMH_IO_IN_CONV) ? (float)((const int16_t *)x)[i] * 0x1p-15f : ((const float *)x)[i];
}
// the sample as the s16 mix sees it
XM_DEV int32_t xm_in_s16(const XmhMixJob &j, const void *x, int64_t i)
{
    return (j.io_flags & XMH_IO_IN_CONV) ? xm_round_sat16(((const float *)x)[i] * 32768.0f)
                                         : (int32_t)((const int16_t *)x)[i];
}

// Block = (output chunk, mix).  For every track: stage the input frames the
// chunk needs into LDS (zero outside [0, N) — equivalent to scipy's skip, see
// DESIGN.md "zero padding"), then each thread forms its outputs tap by tap in
// ascending order (oldest input first) exactly as upfirdn does.
// PART (s16, config 5): write the int32 track sum instead of the saturated mix
template <int C, bool S16, bool PART = false>
__global__ __launch_bounds__(GEN_THREADS) void k_resample_mix_generic(XmhMixJob j)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int L = j.rs.L, M = j.rs.M, T = j.rs.T, rm = j.rs.rm;
    const int b = blockIdx.y;
    const int64_t ob = j.out_base, ib = j.in_base;   // streaming windows (0 for whole clips)
    const int64_t m0 = ob + (int64_t)blockIdx.x * GEN_CHUNK;   // absolute output frames
    const int64_t m1 = min(m0 + GEN_CHUNK, ob + (int64_t)j.frames_out);
    const int64_t N = j.frames_in;

    const int TH = gen_row_stride(T);
    float *H = lds;                                  // L*TH
    float *tile = lds + ((L * TH + 3) & ~3);         // span*C
    if (TH == T) {
        for (int i = threadIdx.x; i < L * T; i += GEN_THREADS) H[i] = j.rs.H[i];
    } else {   // (row, column) of element i carried from one step to the next: two divisions per thread
        const int dr = GEN_THREADS / T, dc = GEN_THREADS % T;
        int row = threadIdx.x / T, col = threadIdx.x % T;
        for (int i = threadIdx.x; i < L * T; i += GEN_THREADS) {
            H[row * TH + col] = j.rs.H[i];
            row += dr;
            col += dc;
            if (col >= T) {
                col -= T;
                ++row;
            }
        }
    }

    const int64_t jlo = ((m0 + rm) * M) / L - T + 1;
    const int64_t jhi = ((m1 - 1 + rm) * M) / L;     // inclusive
    const int span = (int)(jhi - jlo + 1);

    float accf[GEN_OPT][C];
    int32_t acci[GEN_OPT][C];
#pragma unroll
    for (int o = 0; o < GEN_OPT; ++o)
#pragma unroll
        for (int c = 0; c < C; ++c) { accf[o][c] = 0.0f; acci[o][c] = 0; }
    // phase and window start of each of the thread's outputs, once for all
    // tracks: (m + rm) * M = (m0 + rm) * M + d * M with d < GEN_CHUNK, so one
    // 64-bit division per thread and 32-bit ones per output (d * M + r0 <
    // 2^23 for M <= 4096)
    int hoff[GEN_OPT], xoff[GEN_OPT];
    {
        const int64_t Mx0 = (m0 + rm) * M;
        const int64_t q0 = Mx0 / L;
        const int r0 = (int)(Mx0 - q0 * L);
        const int qb = (int)(q0 - T + 1 - jlo);
#pragma unroll
        for (int o = 0; o < GEN_OPT; ++o) {
            const int u = r0 + (int)(threadIdx.x + o * GEN_THREADS) * M;
            const int qu = u / L;
            hoff[o] = (u - qu * L) * TH;         // phase row of H
            xoff[o] = (qb + qu) * C;             // window start in the tile
        }
    }

    for (int tr = 0; tr < j.n_tracks; ++tr) {
        __syncthreads();
        if (j.io_flags) {                            // other input format / planar (whole clips: ib = 0)
            const void *x = xm_track_ptr(j, b, tr, xm_in_elem<S16>(j));
            for (int i = threadIdx.x; i < span * C; i += GEN_THREADS) {
                const int64_t f = jlo + i / C;
                const int64_t q = xm_in_idx(j, f, i % C, C);
                tile[i] = (f >= 0 && f < N) ? (S16 ? (float)xm_in_s16(j, x, q) : xm_in_f32(j, x, q)) : 0.0f;
            }
        } else if (S16) {
            const int16_t *x = (const int16_t *)xm_track_ptr(j, b, tr, 2);
            for (int i = threadIdx.x; i < span * C; i += GEN_THREADS) {
                int64_t f = jlo + i / C;
                tile[i] = (f >= 0 && f < N) ? (float)x[(f - ib) * C + i % C] : 0.0f;
            }
        } else {
            const float *x = (const float *)xm_track_ptr(j, b, tr, 4);
            for (int i = threadIdx.x; i < span * C; i += GEN_THREADS) {
                int64_t f = jlo + i / C;
                tile[i] = (f >= 0 && f < N) ? x[(f - ib) * C + i % C] : 0.0f;
            }
        }
        __syncthreads();
        const XmhGain g = j.gains[tr];
        // a gain constant over the block's outputs: evaluated once per track
        const bool gconst = xm_gain_const(g, m0, m1 - 1);
        const float gfc = S16 ? 0.0f : xm_gain_f32(g, m0);
        const int32_t gqc = S16 ? xm_gain_q15(g, m0) : 0;
#pragma unroll
        for (int o = 0; o < GEN_OPT; ++o) {
            const int64_t m = m0 + threadIdx.x + o * GEN_THREADS;
            if (m >= m1) continue;
            const float *h = H + hoff[o];
            const float *xt = tile + xoff[o];
            float r[C];
#pragma unroll
            for (int c = 0; c < C; ++c) r[c] = 0.0f;
            // stereo taps in blocks of 8: every LDS read of the block issued
            // before the first product, so one wait covers 8 taps (the
            // compiler's own unrolling waited for each pair of taps: lgkmcnt(0)
            // every 4 VALU); same order of ops
            int t = 0;
            if constexpr (C == 2) {   // (L, R) as one packed pair: v_pk_mul_f32 + v_pk_add_f32 per tap
                typedef float f2 __attribute__((ext_vector_type(2)));
                f2 r2 = f2{0.0f, 0.0f};
                if (TH % 4 == 0) {   // 16-B rows: the block's coefficients as two ds_read_b128
                    for (; t + 8 <= T; t += 8) {
                        typedef float f4 __attribute__((ext_vector_type(4)));
                        const f4 ha = *(const f4 *)(h + t), hb = *(const f4 *)(h + t + 4);
                        const float hv[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
                        f2 xv[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) xv[u] = *(const f2 *)(xt + (t + u) * 2);
#pragma unroll
                        for (int u = 0; u < 8; ++u) r2 = r2 + xv[u] * f2{hv[u], hv[u]};
                    }
                } else {
                    for (; t + 8 <= T; t += 8) {
                        float hv[8];
                        f2 xv[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            hv[u] = h[t + u];
                            xv[u] = *(const f2 *)(xt + (t + u) * 2);
                        }
#pragma unroll
                        for (int u = 0; u < 8; ++u) r2 = r2 + xv[u] * f2{hv[u], hv[u]};
                    }
                }
                r[0] = r2.x;
                r[1] = r2.y;
            }
            for (; t < T; ++t) {
                const float hv = h[t];
#pragma unroll
                for (int c = 0; c < C; ++c) r[c] = r[c] + xt[t * C + c] * hv;
            }
            if (S16) {
                const int32_t gq = gconst ? gqc : xm_gain_q15(g, m);
#pragma unroll
                for (int c = 0; c < C; ++c) acci[o][c] += xm_q15_term(xm_round_sat16(r[c]), gq);
            } else {
                const float gf = gconst ? gfc : xm_gain_f32(g, m);
#pragma unroll
                for (int c = 0; c < C; ++c) accf[o][c] = accf[o][c] + gf * r[c];
            }
        }
    }
#pragma unroll
    for (int o = 0; o < GEN_OPT; ++o) {
        const int64_t m = m0 + threadIdx.x + o * GEN_THREADS;
        if (m >= m1) continue;
        if (S16 && PART) {
            int32_t *y = (int32_t *)xm_out_ptr(j, b, 4);
#pragma unroll
            for (int c = 0; c < C; ++c) y[(m - ob) * C + c] = acci[o][c];
        } else if (S16 && j.out_conv == 2) {
            float *y = (float *)xm_out_ptr(j, b, 4);
#pragma unroll
            for (int c = 0; c < C; ++c) y[xm_out_idx(j, m - ob, c, C)] = (float)xm_sat16(acci[o][c]) * 0x1p-15f;
        } else if (S16) {
            int16_t *y = (int16_t *)xm_out_ptr(j, b, 2);
#pragma unroll
            for (int c = 0; c < C; ++c) y[xm_out_idx(j, m - ob, c, C)] = xm_sat16(acci[o][c]);
        } else if (j.out_conv == 1) {
            int16_t *y = (int16_t *)xm_out_ptr(j, b, 2);
#pragma unroll
            for (int c = 0; c < C; ++c)
                y[xm_out_idx(j, m - ob, c, C)] = (int16_t)xm_round_sat16(accf[o][c] * 32768.0f);
        } else {
            float *y = (float *)xm_out_ptr(j, b, 4);
#pragma unroll
            for (int c = 0; c < C; ++c)
                y[xm_out_idx(j, m - ob, c, C)] = accf[o][c] + 0.0f;  // -0 -> +0 (scipy acc starts at +0)
        }
    }
}

// ---- no-resample mixes (L == M) -------------------------------------------
// s16 Q15 mix (config 3): each thread owns 8 consecutive samples (16 B) of the
// mix output and reads the same 16 B from every track: fully coalesced
// dwordx4 streams, int32 accumulate, saturate once.  Gains are evaluated per
// frame; the fast path (gain constant across the thread's frames) evaluates
// them once.
constexpr int MIX_THREADS = 256;

template <int C, bool PART = false>
__global__ __launch_bounds__(MIX_THREADS) void k_mix_s16(XmhMixJob j)
{
    constexpr int SPT = 8;                 // samples per thread (16 B)
    constexpr int FPT = SPT / C;           // frames per thread
    const int b = blockIdx.y;
    const int64_t total = j.frames_out * C;
    const int64_t s0 = ((int64_t)blockIdx.x * MIX_THREADS + threadIdx.x) * SPT;
    if (s0 >= total) return;
    const int64_t f0 = s0 / C + j.out_base;   // absolute frame (gain ramps)
    const bool full = s0 + SPT <= total;

    int32_t acc[SPT];
#pragma unroll
    for (int i = 0; i < SPT; ++i) acc[i] = 0;

    for (int tr = 0; tr < j.n_tracks; ++tr) {
        const int16_t *x = (const int16_t *)xm_track_ptr(j, b, tr, 2) + s0;
        int16_t v[SPT];
        if (full && ((((uintptr_t)x) & 15) == 0)) {
            const int4 q = *(const int4 *)x;
            __builtin_memcpy(v, &q, 16);
        } else {
#pragma unroll
            for (int i = 0; i < SPT; ++i) v[i] = (s0 + i < total) ? x[i] : 0;
        }
        const XmhGain g = j.gains[tr];
        if (xm_gain_const(g, f0, f0 + FPT - 1)) {
            const int32_t gq = xm_gain_q15(g, f0);
#pragma unroll
            for (int i = 0; i < SPT; ++i) acc[i] += xm_q15_term(v[i], gq);
        } else {
#pragma unroll
            for (int f = 0; f < FPT; ++f) {
                const int32_t gq = xm_gain_q15(g, f0 + f);
#pragma unroll
                for (int c = 0; c < C; ++c) acc[f * C + c] += xm_q15_term(v[f * C + c], gq);
            }
        }
    }
    if constexpr (PART) {   // config 5 partial: the int32 sum, saturated later by k_finish_s16
        int32_t *yp = (int32_t *)xm_out_ptr(j, b, 4) + s0;
        if (full && ((((uintptr_t)yp) & 15) == 0)) {
            int4 q0, q1;
            __builtin_memcpy(&q0, acc, 16);
            __builtin_memcpy(&q1, acc + 4, 16);
            ((int4 *)yp)[0] = q0;
            ((int4 *)yp)[1] = q1;
        } else {
            for (int i = 0; i < SPT; ++i)
                if (s0 + i < total) yp[i] = acc[i];
        }
        return;
    }
    int16_t o[SPT];
#pragma unroll
    for (int i = 0; i < SPT; ++i) o[i] = xm_sat16(acc[i]);
    if (j.out_conv == 2) {   // f32 output: exact scaling by 2^-15
        float *yf = (float *)xm_out_ptr(j, b, 4) + s0;
        for (int i = 0; i < SPT; ++i)
            if (s0 + i < total) yf[i] = (float)o[i] * 0x1p-15f;
        return;
    }
    int16_t *y = (int16_t *)xm_out_ptr(j, b, 2) + s0;
    if (full && ((((uintptr_t)y) & 15) == 0)) {
        int4 q;
        __builtin_memcpy(&q, o, 16);
        *(int4 *)y = q;
    } else {
        for (int i = 0; i < SPT; ++i)
            if (s0 + i < total) y[i] = o[i];
    }
}

// fp32 mix without resampling: acc = +0; acc = acc + g*x in track order.
template <int C>
__global__ __launch_bounds__(MIX_THREADS) void k_mix_f32(XmhMixJob j)
{
    constexpr int SPT = 4;                 // 16 B per thread
    constexpr int FPT = SPT / C;
    const int b = blockIdx.y;
    const int64_t total = j.frames_out * C;
    const int64_t s0 = ((int64_t)blockIdx.x * MIX_THREADS + threadIdx.x) * SPT;
    if (s0 >= total) return;
    const int64_t f0 = s0 / C + j.out_base;   // absolute frame (gain ramps)
    const bool full = s0 + SPT <= total;
    float acc[SPT];
#pragma unroll
    for (int i = 0; i < SPT; ++i) acc[i] = 0.0f;
    for (int tr = 0; tr < j.n_tracks; ++tr) {
        const float *x = (const float *)xm_track_ptr(j, b, tr, 4) + s0;
        float v[SPT];
        if (full && ((((uintptr_t)x) & 15) == 0)) {
            const float4 q = *(const float4 *)x;
            v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
            for (int i = 0; i < SPT; ++i) v[i] = (s0 + i < total) ? x[i] : 0.0f;
        }
        const XmhGain g = j.gains[tr];
#pragma unroll
        for (int f = 0; f < FPT; ++f) {
            const float gf = xm_gain_f32(g, f0 + f);
#pragma unroll
            for (int c = 0; c < C; ++c) acc[f * C + c] = acc[f * C + c] + gf * v[f * C + c];
        }
    }
    if (j.out_conv == 1) {   // s16 output: sat16(rint(y * 32768))
        int16_t *yq = (int16_t *)xm_out_ptr(j, b, 2) + s0;
        for (int i = 0; i < SPT; ++i)
            if (s0 + i < total) yq[i] = (int16_t)xm_round_sat16(acc[i] * 32768.0f);
        return;
    }
    float *y = (float *)xm_out_ptr(j, b, 4) + s0;
    if (full && ((((uintptr_t)y) & 15) == 0)) {
        *(float4 *)y = float4{acc[0] + 0.0f, acc[1] + 0.0f, acc[2] + 0.0f, acc[3] + 0.0f};
    } else {
        for (int i = 0; i < SPT; ++i)
            if (s0 + i < total) y[i] = acc[i] + 0.0f;
    }
}

// No-resample mix with input conversion and / or planar layouts (io_flags):
// one thread per output frame, the same per-frame arithmetic as k_mix_s16 /
// k_mix_f32 (gain at the frame, tracks in order, Q15 terms or f32 acc from
// +0), the samples read and written element by element through the layout.
// Consecutive threads take consecutive frames, so planar planes and
// interleaved rows both stay coalesced.
template <int C, bool S16>
__global__ __launch_bounds__(MIX_THREADS) void k_mix_flex(XmhMixJob j)
{
    const int b = blockIdx.y;
    const int64_t f = (int64_t)blockIdx.x * MIX_THREADS + threadIdx.x;
    if (f >= j.frames_out) return;
    float accf[C];
    int32_t acci[C];
#pragma unroll
    for (int c = 0; c < C; ++c) { accf[c] = 0.0f; acci[c] = 0; }
    for (int tr = 0; tr < j.n_tracks; ++tr) {
        const void *x = xm_track_ptr(j, b, tr, xm_in_elem<S16>(j));
        const XmhGain g = j.gains[tr];
        if (S16) {
            const int32_t gq = xm_gain_q15(g, f);
#pragma unroll
            for (int c = 0; c < C; ++c) acci[c] += xm_q15_term(xm_in_s16(j, x, xm_in_idx(j, f, c, C)), gq);
        } else {
            const float gf = xm_gain_f32(g, f);
#pragma unroll
            for (int c = 0; c < C; ++c) accf[c] = accf[c] + gf * xm_in_f32(j, x, xm_in_idx(j, f, c, C));
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int64_t i = xm_out_idx(j, f, c, C);
        if (S16 && j.out_conv == 2) ((float *)xm_out_ptr(j, b, 4))[i] = (float)xm_sat16(acci[c]) * 0x1p-15f;
        else if (S16) ((int16_t *)xm_out_ptr(j, b, 2))[i] = xm_sat16(acci[c]);
        else if (j.out_conv == 1) ((int16_t *)xm_out_ptr(j, b, 2))[i] = (int16_t)xm_round_sat16(accf[c] * 32768.0f);
        else ((float *)xm_out_ptr(j, b, 4))[i] = accf[c] + 0.0f;
    }
}

// Timeline mix: track tr of mix b is an already
// resampled signal placed at output frame place[tr].offset for place[tr].len
// frames; out[m] = ordered sum of g_tr(m) * x_tr[m - offset] with x_tr = 0
// outside [0, len).  A track that does not reach the thread's frames is
// skipped: its terms are +-0, which leaves a non-zero acc unchanged and only
// the sign of a zero acc, normalised by the final +0; Q15
// terms of 0 are exactly 0.  Gains are evaluated at the mix's frame m.
template <int C, bool S16>
__global__ __launch_bounds__(MIX_THREADS) void k_mix_placed(XmhMixJob j)
{
    constexpr int SPT = S16 ? 8 : 4;       // 16 B of output per thread
    constexpr int FPT = SPT / C;
    const int b = blockIdx.y;
    const int64_t total = j.frames_out * C;
    const int64_t s0 = ((int64_t)blockIdx.x * MIX_THREADS + threadIdx.x) * SPT;
    if (s0 >= total) return;
    const int64_t f0 = s0 / C;
    float accf[SPT];
    int32_t acci[SPT];
#pragma unroll
    for (int i = 0; i < SPT; ++i) { accf[i] = 0.0f; acci[i] = 0; }
    for (int tr = 0; tr < j.n_tracks; ++tr) {
        const int64_t off = j.place[2 * tr], len = j.place[2 * tr + 1];
        const int64_t lo = f0 - off;                 // track frame of the thread's first frame
        if (lo + FPT <= 0 || lo >= len) continue;
        const XmhGain g = j.gains[tr];
        const void *xp = j.in_ptrs[(int64_t)b * j.n_tracks + tr];
#pragma unroll
        for (int f = 0; f < FPT; ++f) {
            const int64_t tf = lo + f;
            const bool in = tf >= 0 && tf < len && s0 + f * C < total;
            if (S16) {
                const int32_t gq = xm_gain_q15(g, f0 + f);
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const int32_t v = in ? ((const int16_t *)xp)[tf * C + c] : 0;
                    acci[f * C + c] += xm_q15_term(v, gq);
                }
            } else {
                const float gf = xm_gain_f32(g, f0 + f);
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const float v = in ? ((const float *)xp)[tf * C + c] : 0.0f;
                    accf[f * C + c] = accf[f * C + c] + gf * v;
                }
            }
        }
    }
    if (S16 && j.out_conv == 2) {
        float *y = (float *)xm_out_ptr(j, b, 4) + s0;
        for (int i = 0; i < SPT; ++i)
            if (s0 + i < total) y[i] = (float)xm_sat16(acci[i]) * 0x1p-15f;
    } else if (S16) {
        int16_t *y = (int16_t *)xm_out_ptr(j, b, 2) + s0;
        for (int i = 0; i < SPT; ++i)
            if (s0 + i < total) y[i] = xm_sat16(acci[i]);
    } else if (j.out_conv == 1) {
        int16_t *y = (int16_t *)xm_out_ptr(j, b, 2) + s0;
        for (int i = 0; i < SPT; ++i)
            if (s0 + i < total) y[i] = (int16_t)xm_round_sat16(accf[i] * 32768.0f);
    } else {
        float *y = (float *)xm_out_ptr(j, b, 4) + s0;
        for (int i = 0; i < SPT; ++i)
            if (s0 + i < total) y[i] = accf[i] + 0.0f;
    }
}

// Config 5 finish: out = sat16(sum of n_parts int32 partials, in part order).
// 8 samples (32 B of each partial, 16 B out) per thread, coalesced.
__global__ __launch_bounds__(MIX_THREADS) void k_finish_s16(const int32_t *parts, int n_parts, int64_t part_stride,
                                                          int64_t part_mix_stride, int16_t *out,
                                                          int64_t out_mix_stride, int64_t samples)
{
    constexpr int SPT = 8;
    const int64_t b = blockIdx.y;
    const int64_t s0 = ((int64_t)blockIdx.x * MIX_THREADS + threadIdx.x) * SPT;
    if (s0 >= samples) return;
    const int32_t *p = parts + b * part_mix_stride + s0;
    int16_t *y = out + b * out_mix_stride + s0;
    const bool vec = s0 + SPT <= samples && ((((uintptr_t)p) | ((uintptr_t)y)) & 15) == 0 &&
                     ((part_stride * 4) & 15) == 0;
    int32_t acc[SPT];
#pragma unroll
    for (int i = 0; i < SPT; ++i) acc[i] = 0;
    for (int q = 0; q < n_parts; ++q, p += part_stride) {
        if (vec) {
            const int4 a0 = ((const int4 *)p)[0], a1 = ((const int4 *)p)[1];
            acc[0] += a0.x; acc[1] += a0.y; acc[2] += a0.z; acc[3] += a0.w;
            acc[4] += a1.x; acc[5] += a1.y; acc[6] += a1.z; acc[7] += a1.w;
        } else {
            for (int i = 0; i < SPT; ++i)
                if (s0 + i < samples) acc[i] += p[i];
        }
    }
    int16_t o[SPT];
#pragma unroll
    for (int i = 0; i < SPT; ++i) o[i] = xm_sat16(acc[i]);
    if (vec) {
        int4 qv;
        __builtin_memcpy(&qv, o, 16);
        *(int4 *)y = qv;
    } else {
        for (int i = 0; i < SPT; ++i)
            if (s0 + i < samples) y[i] = o[i];
    }
}

template <typename K>
int launch(K kern, dim3 grid, dim3 block, size_t lds, hipStream_t s, const XmhMixJob &j)
{
    if (grid.x == 0 || grid.y == 0) return 0;
    if (lds > 64 * 1024 && xmg_func_lds((const void *)kern, (int)lds)) return -1001;   // once per (kernel, device)
    hipLaunchKernelGGL(kern, grid, block, lds, s, j);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess && getenv("XM_DEBUG")) fprintf(stderr, "generic launch: %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : -1001;
}

}  // namespace

// Generic launcher (called by xmg_launch_mix in xm_shim.hip when the fast
// kernel does not apply).
extern "C" int xmg_launch_mix_generic(const XmhMixJob *j, void *stream, int *n_launches)
{
    hipStream_t s = (hipStream_t)stream;
    const int C = j->channels;
    const bool s16 = j->fmt == 1;
    if (j->frames_out == 0 || j->n_mix == 0) return 0;
    if (j->partial && !s16) return -22;   // XM_EINVAL: partials are the s16 (Q15) mix
    if (j->partial && j->out_conv) return -22;
    if ((j->in_base || j->out_base) && j->io_flags) return -22;   // layouts / conversion: whole clips only
    if (j->rs.L == j->rs.M && j->io_flags) {
        dim3 grid((unsigned)((j->frames_out + MIX_THREADS - 1) / MIX_THREADS), (unsigned)j->n_mix);
        int rc = s16 ? (C == 1 ? launch(k_mix_flex<1, true>, grid, MIX_THREADS, 0, s, *j)
                               : launch(k_mix_flex<2, true>, grid, MIX_THREADS, 0, s, *j))
                     : (C == 1 ? launch(k_mix_flex<1, false>, grid, MIX_THREADS, 0, s, *j)
                               : launch(k_mix_flex<2, false>, grid, MIX_THREADS, 0, s, *j));
        if (n_launches) *n_launches += 1;
        return rc;
    }
    if (j->rs.L == j->rs.M) {
        const int spt = s16 ? 8 : 4;
        const int64_t samples = j->frames_out * C;
        dim3 grid((unsigned)((samples + (int64_t)MIX_THREADS * spt - 1) / ((int64_t)MIX_THREADS * spt)),
                  (unsigned)j->n_mix);
        int rc;
        if (s16 && j->partial) rc = C == 1 ? launch(k_mix_s16<1, true>, grid, MIX_THREADS, 0, s, *j)
                                           : launch(k_mix_s16<2, true>, grid, MIX_THREADS, 0, s, *j);
        else if (s16) rc = C == 1 ? launch(k_mix_s16<1>, grid, MIX_THREADS, 0, s, *j)
                                  : launch(k_mix_s16<2>, grid, MIX_THREADS, 0, s, *j);
        else     rc = C == 1 ? launch(k_mix_f32<1>, grid, MIX_THREADS, 0, s, *j)
                             : launch(k_mix_f32<2>, grid, MIX_THREADS, 0, s, *j);
        if (n_launches) *n_launches += 1;
        return rc;
    }
    // every ratio and layout the fused kernel does not bake.  (Round 4 tried a
    // phase-major block kernel with per-lane LDS windows here: slower than
    // this LDS-tile kernel on every ratio measured, 1.4-1.8x; removed.)
    const int64_t L = j->rs.L, M = j->rs.M, T = j->rs.T;
    const int64_t span = (GEN_CHUNK * M) / L + 2 + T;
    const size_t lds = (size_t)(((L * gen_row_stride((int)T) + 3) & ~3) + span * C) * sizeof(float);
    if (lds > 160 * 1024) return -1003;  // XM_ENOSYS: ratio too extreme for the LDS-staged path
    dim3 grid((unsigned)((j->frames_out + GEN_CHUNK - 1) / GEN_CHUNK), (unsigned)j->n_mix);
    int rc;
    if (s16 && j->partial) rc = C == 1 ? launch(k_resample_mix_generic<1, true, true>, grid, GEN_THREADS, lds, s, *j)
                                       : launch(k_resample_mix_generic<2, true, true>, grid, GEN_THREADS, lds, s, *j);
    else if (s16) rc = C == 1 ? launch(k_resample_mix_generic<1, true>, grid, GEN_THREADS, lds, s, *j)
                              : launch(k_resample_mix_generic<2, true>, grid, GEN_THREADS, lds, s, *j);
    else     rc = C == 1 ? launch(k_resample_mix_generic<1, false>, grid, GEN_THREADS, lds, s, *j)
                         : launch(k_resample_mix_generic<2, false>, grid, GEN_THREADS, lds, s, *j);
    if (n_launches) *n_launches += 1;
    return rc;
}

extern "C" int xmg_launch_mix_placed(const XmhMixJob *j, void *stream, int *n_launches)
{
    if (j->frames_out == 0 || j->n_mix == 0) return 0;
    if (!j->place || !j->in_ptrs || (j->channels != 1 && j->channels != 2)) return -22;
    const bool s16 = j->fmt == 1;
    const int64_t spt = s16 ? 8 : 4, samples = j->frames_out * j->channels;
    dim3 grid((unsigned)((samples + MIX_THREADS * spt - 1) / (MIX_THREADS * spt)), (unsigned)j->n_mix);
    hipStream_t s = (hipStream_t)stream;
    int rc = s16 ? (j->channels == 1 ? launch(k_mix_placed<1, true>, grid, MIX_THREADS, 0, s, *j)
                                     : launch(k_mix_placed<2, true>, grid, MIX_THREADS, 0, s, *j))
                 : (j->channels == 1 ? launch(k_mix_placed<1, false>, grid, MIX_THREADS, 0, s, *j)
                                     : launch(k_mix_placed<2, false>, grid, MIX_THREADS, 0, s, *j));
    if (n_launches) *n_launches += 1;
    return rc;
}

extern "C" int xmg_launch_finish_s16(const int32_t *parts, int n_parts, int64_t part_stride, int64_t part_mix_stride,
                                     int16_t *out, int64_t out_mix_stride, int64_t batch, int64_t samples, void *stream)
{
    if (batch <= 0 || samples <= 0) return 0;
    const unsigned gx = (unsigned)((samples + (int64_t)MIX_THREADS * 8 - 1) / ((int64_t)MIX_THREADS * 8));
    for (int64_t b0 = 0; b0 < batch; b0 += 65535) {   // grid.y limit
        const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
        hipLaunchKernelGGL(k_finish_s16, dim3(gx, (unsigned)nb), dim3(MIX_THREADS), 0, (hipStream_t)stream,
                           parts + b0 * part_mix_stride, n_parts, part_stride, part_mix_stride,
                           out + b0 * out_mix_stride, out_mix_stride, samples);
        if (hipGetLastError() != hipSuccess) return -1001;
    }
    return 0;
}
