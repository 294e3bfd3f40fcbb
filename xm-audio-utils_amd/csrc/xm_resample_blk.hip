// xm_resample_blk.hip — polyphase resample + gain + ordered track sum for
// every rate pair the fused kernel (xm_resample_fast.hip) does not bake:
// any L/M, mono or stereo, f32 or s16 (Q15) mixes, s16 <-> f32 input
// conversion, interleaved or planar output, config 5 int32 partials and
// streaming windows.  Arithmetic: include/xm_audio_common.h, scipy
// resample_poly's order (acc = +0, then acc + x[j0 + t] * H[ph][t] for t
// ascending), so the results equal the oracle and the fused kernel bit for bit.
//
// Work decomposition (phase-major).  Outputs m = ob + v*LB + k (k < LB,
// LB = q*L outputs of a "lane block" whose input advances MB = q*M frames):
// output k of every lane block has the same filter phase and the same window
// offset, so a wave whose 64 lanes are 64 consecutive lane blocks walks k
// wave-uniformly -- the phase row of H is read by scalar loads (SGPRs), the
// window offset is a scalar, and each lane reads its own input window from
// LDS at an immediate offset per tap.  q is chosen so a lane block holds at
// least 64 outputs (small-L ratios such as 3/2 or 1/2).
//  * Sub-chunks of KS outputs per lane (KS <= 16): per track, each lane
//    stages the FS frames its KS outputs read (global 16-B buffer loads of
//    its own stream, converted to f32 on the way) into its LDS row, then
//    forms the KS outputs; the KS x C sums stay in registers across the
//    tracks (the ordered track sum, no exchange).
//  * LDS row stride: odd (mono) / twice an odd number (stereo) dwords, so the
//    64 lanes' reads of one tap (b32 or b64) are bank-conflict free.
//  * Frames outside [0, N) read as zero (buffer range checks; the s16 dword
//    straddling the end is loaded and its extra sample zeroed explicitly).
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <type_traits>
#include "xm_device.h"

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
// the coefficient table through the constant address space: wave-uniform
// rows are read by scalar loads into SGPRs (tap operands of the VALU ops)
typedef const __attribute__((address_space(4))) float cfloat;

constexpr int BK_KS = 16;   // outputs per lane per sub-chunk at most

struct BlkArgs {
    XmhMixJob j;
    int32_t LB, MB;          // outputs / input frames per lane block
    int32_t KS;              // outputs per lane per sub-chunk
    int32_t SE;              // LDS row stride per lane (floats)
    int32_t NLD;             // 16-B loads per lane per staging
    int32_t waves_per_mix;
    int32_t dq, dr;          // M / L, M % L (per output step)
    int32_t kq, kr;          // (KS*M) / L, (KS*M) % L (per sub-chunk step)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}

// one output: r = sum over t ascending (from +0) of x[t*C + c] * h[t]; 8
// taps per step (one scalar load of 8 coefficients, 8 LDS reads at
// immediate offsets); stereo (L, R) in one packed pair
template <int C>
__device__ __forceinline__ void dot1(const float *x, cfloat *h, int T, float (&res)[2])
{
    int t = 0;
    if (C == 2) {
        const f2 *xv = (const f2 *)x;
        f2 acc = f2{0.0f, 0.0f};
        for (; t + 8 <= T; t += 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float ht = h[t + e];
                acc = acc + xv[t + e] * f2{ht, ht};
            }
        }
        for (; t < T; ++t) {
            const float ht = h[t];
            acc = acc + xv[t] * f2{ht, ht};
        }
        res[0] = acc.x;
        res[1] = acc.y;
    } else {
        float acc = 0.0f;
        for (; t + 8 <= T; t += 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) acc = acc + x[t + e] * h[t + e];
        }
        for (; t < T; ++t) acc = acc + x[t] * h[t];
        res[0] = acc;
    }
}

// two outputs whose windows start d = 0 or 1 frame apart, from one read of
// each frame: output 0 takes x[t] * h0[t], output 1 x[t] * h1[t - d]; each
// sum still runs over its taps in ascending order from +0
template <int C>
__device__ __forceinline__ void dot2(const float *x, cfloat *h0, cfloat *h1, int T, int d, float (&r0)[2],
                                     float (&r1)[2])
{
    typedef typename std::conditional<C == 2, f2, float>::type V;
    const V *xv = (const V *)x;
    auto mul = [](V v, float hv) __attribute__((always_inline)) {
        if constexpr (C == 2) return v * f2{hv, hv};
        else return v * hv;
    };
    V a = V{}, b = V{};   // +0
    if (d == 0) {
        int t = 0;
        for (; t + 8 <= T; t += 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const V v = xv[t + e];
                a = a + mul(v, h0[t + e]);
                b = b + mul(v, h1[t + e]);
            }
        }
        for (; t < T; ++t) {
            const V v = xv[t];
            a = a + mul(v, h0[t]);
            b = b + mul(v, h1[t]);
        }
    } else {
        a = a + mul(xv[0], h0[0]);
        int t = 1;
        for (; t + 8 <= T; t += 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const V v = xv[t + e];
                a = a + mul(v, h0[t + e]);
                b = b + mul(v, h1[t + e - 1]);
            }
        }
        for (; t < T; ++t) {
            const V v = xv[t];
            a = a + mul(v, h0[t]);
            b = b + mul(v, h1[t - 1]);
        }
        b = b + mul(xv[T], h1[T - 1]);
    }
    if constexpr (C == 2) {
        r0[0] = a.x;
        r0[1] = a.y;
        r1[0] = b.x;
        r1[1] = b.y;
    } else {
        r0[0] = a;
        r1[0] = b;
    }
}

// IN16: s16 samples in memory (an s16 mix, or s16 tracks converted into an f32 one)
template <int C, bool S16, bool IN16, bool PART, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_rs_blk(BlkArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float lds_blk[];
    const XmhMixJob &j = a.j;
    const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int gw = (int)blockIdx.x * WPB + wave;               // wave of this mix
    if (gw >= a.waves_per_mix) return;                          // whole waves only
    const int b = blockIdx.y;
    float *row = lds_blk + ((size_t)wave * 64 + lane) * a.SE;   // this lane's window
    const int L = j.rs.L, M = j.rs.M, T = j.rs.T;
    const int64_t N = j.frames_in, ib = j.in_base, ob = j.out_base;
    const int64_t blk = (int64_t)gw * 64 + lane;                // lane block
    const int64_t i_lane = blk * a.LB;                          // its first output (relative)
    const int64_t i_wave = (int64_t)gw * 64 * a.LB;
    // input element format: the mix's own, or the other one (XMH_IO_IN_CONV)
    constexpr bool conv = IN16 != S16;                          // XMH_IO_IN_CONV
    constexpr int es = IN16 ? 2 : 4;                            // bytes per input sample
    constexpr int epg = 16 / es;                                // samples per 16-B load
    const int64_t nvalid = (N - ib) * C;                        // samples from the window base on
    // sub-chunk anchor: num = (ob + k0 + rm) * M = qn * L + rn
    const int64_t num0 = (ob + j.rs.rm) * (int64_t)M;
    int64_t qn = num0 / L;
    int rn = (int)(num0 % L);
    for (int k0 = 0; k0 < a.LB; k0 += a.KS) {
        if (i_wave + k0 >= j.frames_out) break;                 // the wave's outputs are all past the end
        const int ks = min(a.KS, a.LB - k0);
        // frames [w0, w0 + FS) of the lane's window, w0 = floor((ob+k0+rm)M/L) - T + 1 + blk*MB
        const int64_t w0 = qn - T + 1 + blk * a.MB;
        const int64_t e_first = (w0 - ib) * C;                 // sample index from the window base
        const int64_t e_al = (e_first >= 0 ? e_first / epg : -((-e_first + epg - 1) / epg)) * epg;
        const int sh = (int)(e_first - e_al);                  // lane shift into its row
        float accf[BK_KS][C];
        int32_t acci[BK_KS][C];
#pragma unroll
        for (int u = 0; u < BK_KS; ++u)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                accf[u][c] = 0.0f;
                acci[u][c] = 0;
            }
        // the lanes whose loads touch the clip end zero the samples past it
        const bool edge = __builtin_amdgcn_readfirstlane(
                              (int)(__builtin_amdgcn_ballot_w64(e_al + (int64_t)a.NLD * epg > nvalid) != 0)) != 0;
        for (int tr = 0; tr < j.n_tracks; ++tr) {
            // ---- stage the lane's window of track tr into its LDS row
            const char *tp = (const char *)xm_track_ptr(j, b, tr, es);
            const uint32_t nrec = (uint32_t)((nvalid * es + 3) & ~(int64_t)3);
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(tp, nvalid > 0 ? nrec : 0u);
            for (int g = 0; g < a.NLD; ++g) {
                const int64_t e = e_al + (int64_t)g * epg;     // first sample of this load
                // negative offsets wrap past num_records: zero (frames before 0)
                const uint32_t off = (uint32_t)(e * es);
                const i4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
                float f[8];
                if (IN16) {
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        f[2 * h] = (float)(int)(short)(v[h] & 0xffff);
                        f[2 * h + 1] = (float)(v[h] >> 16);
                    }
                } else {
                    // the whole vector at once (a bit_cast of one ext_vector
                    // element lost the other elements in this compiler)
                    const f4 vf = __builtin_bit_cast(f4, v);
#pragma unroll
                    for (int h = 0; h < 4; ++h) f[h] = vf[h];
                }
#pragma unroll
                for (int h = 0; h < epg; ++h) {
                    float x = f[h];
                    if (conv) x = S16 ? (float)xm_round_sat16(x * 32768.0f) : x * 0x1p-15f;
                    if (edge && e + h >= nvalid) x = 0.0f;      // the straddling dword's extra sample, or past N
                    f[h] = x;
                }
                float *d = row + g * epg;
                if (C == 2) {
#pragma unroll
                    for (int h = 0; h < epg; h += 2) *(f2 *)(d + h) = f2{f[h], f[h + 1]};
                } else {
#pragma unroll
                    for (int h = 0; h < epg; ++h) d[h] = f[h];
                }
            }
            // ---- the ks outputs of this sub-chunk (same wave: LDS in order)
            const XmhGain g = j.gains[tr];
            const int64_t m_lo = ob + i_wave + k0, m_hi = ob + i_wave + 63 * (int64_t)a.LB + k0 + ks - 1;
            const bool gconst = xm_gain_const(g, m_lo, m_hi);
            const float gfc = xm_gain_f32(g, m_lo);
            const int32_t gqc = xm_gain_q15(g, m_lo);
            int64_t q = qn;
            int r = rn;
            auto step = [&]() __attribute__((always_inline)) {   // to the next output
                r += a.dr;
                q += a.dq;
                if (r >= L) {
                    r -= L;
                    ++q;
                }
            };
            auto take = [&](int u, const float (&v)[2]) __attribute__((always_inline)) {   // gain, ordered sum
                const int64_t m = ob + i_lane + k0 + u;          // absolute output frame of this lane
                if (S16) {
                    const int32_t gq = gconst ? gqc : xm_gain_q15(g, m);
#pragma unroll
                    for (int c = 0; c < C; ++c) acci[u][c] += xm_q15_term(xm_round_sat16(v[c]), gq);
                } else {
                    const float gf = gconst ? gfc : xm_gain_f32(g, m);
#pragma unroll
                    for (int c = 0; c < C; ++c) accf[u][c] = accf[u][c] + gf * v[c];
                }
            };
            // outputs in pairs: when the second window starts 0 or 1 frame
            // after the first (every upsampling ratio; most frames of mild
            // downsampling) one LDS read per tap feeds both
#pragma unroll
            for (int u = 0; u < BK_KS; u += 2) {
                if (u >= ks) continue;   // wave-uniform
                const bool two = u + 1 < ks;
                const int ph0 = (int)__builtin_amdgcn_readfirstlane(r);
                const int off0 = (int)__builtin_amdgcn_readfirstlane((int)(q - qn));   // window offset (frames)
                step();
                const int ph1 = (int)__builtin_amdgcn_readfirstlane(r);
                const int off1 = (int)__builtin_amdgcn_readfirstlane((int)(q - qn));
                step();
                cfloat *h0 = (cfloat *)j.rs.H + (size_t)ph0 * T;
                cfloat *h1 = (cfloat *)j.rs.H + (size_t)ph1 * T;
                const float *x0 = row + sh + off0 * C;
                float v0[2] = {0.0f, 0.0f}, v1[2] = {0.0f, 0.0f};
                const int d = off1 - off0;
                if (two && (d == 0 || d == 1)) {
                    dot2<C>(x0, h0, h1, T, d, v0, v1);
                } else {
                    dot1<C>(x0, h0, T, v0);
                    if (two) dot1<C>(row + sh + off1 * C, h1, T, v1);
                }
                take(u, v0);
                if (two) take(u + 1, v1);
            }
        }
        // ---- store the lane's ks outputs
#pragma unroll
        for (int u = 0; u < BK_KS; ++u) {
            if (u >= ks) continue;
            const int64_t i = i_lane + k0 + u;
            if (i >= j.frames_out) continue;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int64_t o = (j.io_flags & XMH_IO_OUT_PLANAR) ? (int64_t)c * j.frames_out + i : i * C + c;
                if (S16 && PART) ((int32_t *)xm_out_ptr(j, b, 4))[o] = acci[u][c];
                else if (S16 && j.out_conv == 2) ((float *)xm_out_ptr(j, b, 4))[o] = (float)xm_sat16(acci[u][c]) * 0x1p-15f;
                else if (S16) ((int16_t *)xm_out_ptr(j, b, 2))[o] = xm_sat16(acci[u][c]);
                else if (j.out_conv == 1) ((int16_t *)xm_out_ptr(j, b, 2))[o] = (int16_t)xm_round_sat16(accf[u][c] * 32768.0f);
                else ((float *)xm_out_ptr(j, b, 4))[o] = accf[u][c] + 0.0f;   // -0 -> +0 (the contract's +0 seed)
            }
        }
        // next sub-chunk: num += KS * M
        rn += a.kr;
        qn += a.kq;
        if (rn >= L) {
            rn -= L;
            ++qn;
        }
    }
}

template <int C, bool S16, bool IN16, bool PART>
const void *blk_kern(int wpb)
{
    return wpb == 4 ? (const void *)k_rs_blk<C, S16, IN16, PART, 4> : (const void *)k_rs_blk<C, S16, IN16, PART, 1>;
}

}  // namespace

// The block kernel for a resampling mix job (rs.L != rs.M); XM_ENOSYS
// (-1003) when it does not take the job (planar input, s16 tracks that are
// not 4-B aligned, a ratio whose window does not fit LDS): the caller then
// runs the LDS-tile generic kernel.
extern "C" int xmg_launch_resample_blk(const XmhMixJob *j, void *stream, int *n_launches)
{
    const int C = j->channels;
    const bool s16 = j->fmt == 1;
    if (j->rs.L == j->rs.M || (C != 1 && C != 2) || (j->io_flags & XMH_IO_IN_PLANAR)) return -1003;
    if (j->partial && !s16) return -22;
    const bool conv = (j->io_flags & XMH_IO_IN_CONV) != 0;
    const int es = (conv != s16) ? 2 : 4;
    // 4-B aligned tracks (the dword range checks of the buffer loads)
    if (j->in_ptrs) {
        if (!j->in_ptrs_host) return -1003;
        for (int64_t i = 0; i < (int64_t)j->n_mix * j->n_tracks; ++i)
            if ((uintptr_t)j->in_ptrs_host[i] & 3) return -1003;
    } else if (((uintptr_t)j->in & 3) || ((j->in_track_stride * es) & 3) || ((j->in_mix_stride * es) & 3)) {
        return -1003;
    }
    const int64_t L = j->rs.L, M = j->rs.M, T = j->rs.T;
    if ((j->frames_in - j->in_base) * C * es >= ((int64_t)1 << 31)) return -1003;   // 32-bit buffer offsets
    // lane blocks of >= 64 outputs; KS outputs per sub-chunk with a window of
    // FS <= max(2T, 48) frames
    const int64_t q = (64 + L - 1) / L;
    const int64_t LB = q * L, MB = q * M;
    const int64_t budget = std::max<int64_t>(2 * T, 48);
    int64_t KS = ((budget - T) * L) / M + 1;
    KS = std::max<int64_t>(1, std::min<int64_t>(KS, BK_KS));
    const int64_t FS = ((KS - 1) * M + L - 1) / L + 1 + T;      // frames of one sub-chunk's window (upper bound)
    const int epg = 16 / es;
    const int64_t NLD = (FS * C + epg - 1) / epg + 1;           // 16-B loads per lane (any alignment)
    int64_t SE = NLD * epg;                                     // floats per row
    if (C == 2) SE = (SE / 2) | 1, SE *= 2;                     // 2 x odd: conflict-free b64 reads
    else SE |= 1;                                               // odd: conflict-free b32 reads
    const int64_t row_bytes = 64 * SE * 4;
    const int wpb = row_bytes * 4 <= 64 * 1024 ? 4 : 1;
    if (row_bytes * wpb > 160 * 1024) return -1003;
    const int64_t nblk = (j->frames_out + LB - 1) / LB;
    const int64_t waves = (nblk + 63) / 64;
    if (waves > 0x7fffffff || j->n_mix > 65535) return -1003;
    BlkArgs a;
    memset(&a, 0, sizeof a);
    a.j = *j;
    a.LB = (int32_t)LB;
    a.MB = (int32_t)MB;
    a.KS = (int32_t)KS;
    a.SE = (int32_t)SE;
    a.NLD = (int32_t)NLD;
    a.waves_per_mix = (int32_t)waves;
    a.dq = (int32_t)(M / L);
    a.dr = (int32_t)(M % L);
    a.kq = (int32_t)((KS * M) / L);
    a.kr = (int32_t)((KS * M) % L);
    const bool in16 = es == 2;
    const void *kern =
        C == 1 ? (s16 ? (j->partial ? (in16 ? blk_kern<1, true, true, true>(wpb) : blk_kern<1, true, false, true>(wpb))
                                    : (in16 ? blk_kern<1, true, true, false>(wpb) : blk_kern<1, true, false, false>(wpb)))
                      : (in16 ? blk_kern<1, false, true, false>(wpb) : blk_kern<1, false, false, false>(wpb)))
               : (s16 ? (j->partial ? (in16 ? blk_kern<2, true, true, true>(wpb) : blk_kern<2, true, false, true>(wpb))
                                    : (in16 ? blk_kern<2, true, true, false>(wpb) : blk_kern<2, true, false, false>(wpb)))
                      : (in16 ? blk_kern<2, false, true, false>(wpb) : blk_kern<2, false, false, false>(wpb)));
    const size_t lds = (size_t)(row_bytes * wpb);
    if (lds > 64 * 1024 && xmg_func_lds(kern, (int)lds)) return -1001;
    void *kargs[] = {&a};
    const dim3 grid((unsigned)((waves + wpb - 1) / wpb), (unsigned)j->n_mix);
    if (hipLaunchKernel(kern, grid, dim3(64 * wpb), kargs, lds, (hipStream_t)stream) != hipSuccess) return -1001;
    if (n_launches) *n_launches += 1;
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}
