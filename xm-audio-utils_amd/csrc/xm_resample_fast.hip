// xm_resample_fast.hip — the headline kernel: 48 kHz -> 44.1 kHz (L/M =
// 147/160) polyphase resample of stereo fp32 tracks + per-track gain ramp +
// in-order track sum, fused in one pass over HBM (SURVEY.md §8(a) a2+a4+a7).
//
// Arithmetic is scipy resample_poly's (include/xm_audio_common.h): per output
// acc = sum_t x[j0+t]*H[ph][t] in ascending t, each mul and add rounded
// separately (-ffp-contract=off), then mix = ((+0 + g0*r0) + g1*r1) + ...
// Exact shortcuts (DESIGN.md §"Exactness of the fast path"):
//  * tap 22 of every phase is an exact 0 for 147/160 (the 160-zero pre-pad),
//    so each output uses taps 0..21 (finite inputs);
//  * the +0 seeds of the dot product and of the mix are folded into one
//    final "+ 0.0f", which maps -0 to +0 and leaves every other value alone;
//  * inside a ramp g = gA + gS*(float)k with (gA, gS) = (g0, step) or, for a
//    crossfade-out, (1, -step): 1 + (-step)*k == 1 - (0 + step*k) bit for bit.
//
// Work decomposition (MI355X-first; measurements in DESIGN.md §fast kernel):
//  * super-period (SP) = 160 input frames -> 147 output frames.  The filter
//    phase of output k of an SP does not depend on the SP, so a wave whose
//    64 lanes are 64 SP streams runs one wave-uniform phase sequence: the 22
//    coefficients of each output are SGPR operands (scalar cache) of
//    v_pk_mul_f32 on stereo L/R pairs.
//  * lanes = NT tracks x S (=64/NT) stream slots of one mix.  Each lane walks
//    R consecutive SPs of its track, so its input is one contiguous stream
//    and the register window carries across SPs (43 frames moved per SP).
//  * input arrives by LDS-DMA (buffer_load ... lds) in 256-B segments per
//    stream: one DMA instruction = 4 streams x 256 B.  Measured on MI355X
//    (tools/ubench/mem_pattern.hip): 16 lanes per 256-B segment streams at
//    6.3 TB/s, whereas one 16-B stream per lane caps at 4.2 TB/s.  Chunks
//    are rotated per stream so the LDS->VGPR copy (ds_read_b128) is
//    bank-conflict free; buffer range checks plus explicit redirects
//    zero-fill frames outside [0, N).
//  * the ordered track sum is exchanged through 4 KiB of wave-private LDS
//    (rows rotated instead of padded): no workgroup barriers at all.
//  * LDS per wave = 16 KiB slot + 4 KiB exchange = 20 KiB -> 8 waves/CU,
//    leaving a 256-VGPR budget for the window.
#include <stdlib.h>
#include <string.h>
#include "xm_device.h"

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef const float __attribute__((address_space(4))) cfloat;   // -> s_load
typedef const f2 __attribute__((address_space(4))) cf2;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) char lds_char;

constexpr int L = 147, M = 160, RM = 11;   // reduced ratio, output offset rm
constexpr int TE = 22;                     // taps used (tap 22 is an exact zero)
constexpr int SPO = L;                     // outputs per super-period
constexpr int SPI = M;                     // input frames per super-period
constexpr int SEGF = 32;                   // frames per DMA segment (256 B)
constexpr int G = 8;                       // outputs per exchange round
constexpr int ROUNDS = (SPO + G - 1) / G;  // 19
constexpr int HK_STRIDE = 24;              // floats per output row of the k-ordered table
constexpr int CARRY0 = 21;                 // first rel frame an SP needs
constexpr int WIN = 7 * SEGF;              // 224 rel frames: SP s uses rel [21, 201]
constexpr int SLOT_BYTES = 64 * 256;       // one segment for 64 streams
constexpr int X_F2 = G * 64;               // exchange: 8 outputs x 64 lanes (f2)
constexpr int LDS_PER_WAVE = SLOT_BYTES + X_F2 * 8;   // 20 KiB
constexpr uint32_t OOB = 0x80000000u;      // voffset beyond every num_records

// rel frame (relative to 160*s - 32) of tap 0 of output k of SP s
// (scipy: j0 = floor((m+rm)*M/L) - T + 1, T = 23)
__host__ __device__ constexpr int rk(int k) { return ((k + RM) * M) / L - 22 + 32; }
// segment (0..6 of the SP's 7) holding the last frame output k needs
constexpr int last_seg(int k) { return (rk(k) + TE - 1) / SEGF; }
// last segment needed by the pair starting at even k / before it
constexpr int need_pair(int k) { return last_seg(k + 1 < SPO ? k + 1 : k); }
constexpr int need_before(int k) { return k == 0 ? 1 : last_seg(k - 1); }
static_assert(rk(0) == CARRY0, "window origin");
static_assert(last_seg(SPO - 1) == 6, "an SP spans 7 segments");
static_assert(last_seg(0) == 1, "first outputs need segments 0,1");

struct FastArgs {
    const float *in;                 // mix 0, track 0
    int64_t in_mix_stride;           // floats
    int64_t track_bytes;             // bytes between tracks of a mix (>= 8*N)
    float *out;
    int64_t out_mix_stride;          // floats
    const float *Hk;                 // [147][24] coefficients in output order
    int32_t n_mix, n_tracks;
    int32_t frames_in, frames_out;
    int32_t n_sp;                    // SPs per clip = ceil(frames_out / 147)
    int32_t R;                       // SPs per lane (consecutive)
    int32_t tasks_per_mix;
    int32_t unity;
    XmhGain g[8];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}

// exact contract gain (xm_audio_common.h) at output frame n
__device__ __forceinline__ float gain_exact(const XmhGain &g, int n)
{
    float v;
    if (g.len == 0) {
        v = n >= (int)g.start ? g.g1 : g.g0;
    } else {
        int k = n - (int)g.start;
        k = k < 0 ? 0 : (k > g.len ? g.len : k);
        v = g.g0 + g.step * (float)k;
    }
    return (g.flags & XMH_GAIN_XFADE_OUT) ? 1.0f - v : v;
}

template <int NT>
__global__ __launch_bounds__(64) void k_rs147_mix(FastArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int S = 64 / NT;                  // stream slots (SP runs) per track in a wave
    const int lane = threadIdx.x;
    const int tr = lane / S, spl = lane % S;    // compute mapping: lane = tr*S + spl
    const int mix = blockIdx.x / a.tasks_per_mix;
    const int task = blockIdx.x % a.tasks_per_mix;
    const int s_first = (task * S + spl) * a.R;                 // this lane's first SP
    char *slot = lds;
    // the same slot as an LDS-space pointer: M0 for the DMA is then a plain
    // constant (a generic->LDS cast would add a null check on SCC)
    lds_char *slot3 = (lds_char *)(lds_void *)lds;
    f2 *X = (f2 *)(lds + SLOT_BYTES);

    // one resource per mix, shifted 32 frames back so offsets stay >= 0
    const float *mixbase = a.in + (int64_t)mix * a.in_mix_stride;
    const uint32_t nrec = (uint32_t)((NT - 1) * a.track_bytes + ((int64_t)a.frames_in + 32) * 8);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(mixbase - 64, nrec);

    // ---- DMA addressing (loader role): instruction d covers streams
    // q = 4d..4d+3; lane l loads chunk j = ((l & 15) - q) & 15 of stream
    // q = 4d + (l >> 4), which the hardware lands at slot + d*1024 + l*16.
    // For S = 8 the byte offset splits into a wave-uniform part (soffset:
    // track d/2, slot group 4*(d&1), segment, SP) and one of 4 per-lane
    // parts (the chunk rotation depends on d only through d & 3).
    static_assert(S == 8, "DMA address split assumes 8 stream slots per track");
    const int lq = lane >> 4;                                   // stream within the 4 of an instruction
    uint32_t vl[4];
    int32_t fl[4];
#pragma unroll
    for (int d4 = 0; d4 < 4; ++d4) {
        const int j = ((lane & 15) - lq - 4 * d4) & 15;
        vl[d4] = (uint32_t)((task * S + lq) * a.R * (SPI * 8) + j * 16);
        fl[d4] = (task * S + lq) * a.R * SPI - 32 + 2 * j;
    }
    const uint32_t TB = __builtin_amdgcn_readfirstlane((uint32_t)a.track_bytes);
    const uint32_t GR = __builtin_amdgcn_readfirstlane((uint32_t)(4 * a.R * (SPI * 8)));   // slot group 4..7
    const int N = a.frames_in;
    // edge streams (clip start / end inside this task's span) need per-chunk redirects
    const bool edge = __builtin_amdgcn_ballot_w64(s_first == 0 || (s_first + a.R) * SPI + 64 > N) != 0;

    auto dma = [&](int r, int m) {   // segment m (0..6 rel to SP r) of every stream
        // soffset = track part + slot-group part + SP + segment.  Built with a
        // volatile s_add in place: left to itself LICM hoists all 112
        // (instruction, segment) constants out of the SP loop and spills SGPRs.
        const uint32_t rb0 = (uint32_t)(r * (SPI * 8) + m * 256);
        const uint32_t rb1 = rb0 + GR;
        if (!edge) {
#pragma unroll
            for (int d = 0; d < 16; ++d) {
                uint32_t so;
                asm volatile("s_mul_i32 %0, %1, %2\n\ts_add_u32 %0, %0, %3"
                             : "=&s"(so) : "s"(TB), "n"(d >> 1), "s"((d & 1) ? rb1 : rb0) : "scc");
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(slot3 + d * 1024), 16, vl[d & 3], so, 0, 0);
            }
        } else {
#pragma unroll
            for (int d = 0; d < 16; ++d) {
                uint32_t so;
                asm volatile("s_mul_i32 %0, %1, %2\n\ts_add_u32 %0, %0, %3"
                             : "=&s"(so) : "s"(TB), "n"(d >> 1), "s"((d & 1) ? rb1 : rb0) : "scc");
                const int f = fl[d & 3] + 4 * (d & 1) * a.R * SPI + r * SPI + m * SEGF;
                // out-of-clip chunks: push the whole offset past num_records
                const uint32_t v = (f >= 0 && f + 1 < N) ? vl[d & 3] : OOB;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(slot3 + d * 1024), 16, v, so, 0, 0);
            }
        }
    };
    // ---- register window: rel frames [0, 224) of the current SP, one array
    // per channel (kept scalar so nothing re-packs the VOP2 arithmetic)
    float xl[WIN], xr[WIN];
    auto copy_seg = [&](int m) {     // slot -> x[32m .. 32m+31] of this lane's stream
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");         // this wave's DMA landed
        const char *base = slot + (lane >> 2) * 1024 + (lane & 3) * 256;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float4 v = *(const float4 *)(base + (((j + lane) & 15) * 16));
            xl[SEGF * m + 2 * j] = v.x;
            xr[SEGF * m + 2 * j] = v.y;
            xl[SEGF * m + 2 * j + 1] = v.z;
            xr[SEGF * m + 2 * j + 1] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       // slot free for the next DMA
    };

    // ---- gain ramp of this lane's track
    XmhGain gp = a.g[0];
#pragma unroll
    for (int i = 1; i < NT; ++i)
        if (tr == i) gp = a.g[i];
    const bool xf = (gp.flags & XMH_GAIN_XFADE_OUT) != 0;

    float *outb = a.out + (int64_t)mix * a.out_mix_stride;
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(outb, (uint32_t)a.frames_out * 8u);
    cf2 *Hp = (cf2 *)a.Hk;   // [74][22] pairs (h_2i[t], h_2i+1[t])

    // prologue: segments 0, 1 of the first SP; segment 2 in flight
    dma(0, 0);
    copy_seg(0);
    dma(0, 1);
    copy_seg(1);
    dma(0, 2);

#pragma unroll 1
    for (int r = 0; r < a.R; ++r) {
        const int s = s_first + r;
        const int n_sp0 = s * SPO;
        // gain class of this lane over the SP: 0 constant, 1 linear (inside the
        // ramp, no clamp), 2 boundary (clamp or step inside the SP)
        int cls;
        float cA, cB = 0.0f, fkb = 0.0f;
        {
            const int st = (int)gp.start, ln = gp.len;
            const int lo = n_sp0, hi = n_sp0 + SPO - 1;
            const bool konst = ln == 0 ? !(lo < st && hi >= st) : (hi <= st || lo >= st + ln);
            if (konst) {
                cls = 0;
                cA = gain_exact(gp, lo);
            } else if (ln > 0 && lo >= st && hi <= st + ln) {
                cls = 1;
                cA = xf ? 1.0f : gp.g0;
                cB = xf ? -gp.step : gp.step;
                fkb = (float)(lo - st);
            } else {
                cls = 2;
                cA = 0.0f;
            }
        }
        const bool any_lin = __builtin_amdgcn_readfirstlane((int)(__builtin_amdgcn_ballot_w64(cls == 1) != 0));
        const bool any_bnd = __builtin_amdgcn_readfirstlane((int)(__builtin_amdgcn_ballot_w64(cls == 2) != 0));

#pragma unroll
        for (int q = 0; q < ROUNDS; ++q) {
            const int k0 = q * G;
            const int kend = k0 + G < SPO ? k0 + G : SPO;
            float gk[G];
#pragma unroll
            for (int i = 0; i < G; ++i) gk[i] = cA;
            if (any_bnd) {
#pragma unroll
                for (int i = 0; i < G; ++i) gk[i] = gain_exact(gp, n_sp0 + k0 + i);
            } else if (any_lin) {
#pragma unroll
                for (int i = 0; i < G; ++i) gk[i] = cA + cB * (fkb + (float)(k0 + i));
            }
#pragma unroll
            for (int k = k0; k < kend; k += 2) {
                const bool two = k + 1 < kend;
                // bring in the segments this pair needs (static schedule):
                // copy segment m, then start the DMA of the next one
#pragma unroll
                for (int m = need_before(k) + 1; m <= need_pair(k); ++m) {
                    copy_seg(m);
                    if (m < 6) dma(r, m + 1);
                    else if (r + 1 < a.R) dma(r + 1, 2);          // next SP's segment 2
                }
                // one s_load_dwordx2 pair (h_k[t], h_k+1[t]) feeds both outputs.
                // Per-channel VOP2 v_mul_f32/v_add_f32 with a single-SGPR
                // coefficient: the same VALU cycles as v_pk_* on the stereo
                // pair (4 x 2 vs 2 x 4 per tap) but no SGPR-pair broadcasts,
                // which the compiler otherwise materialises with s_mov and spills.
                cf2 *hp = Hp + (k >> 1) * TE;
                const int ra = rk(k), rb = rk(two ? k + 1 : k);
                f2 h = hp[0];
                float l0 = xl[ra] * h.x, r0 = xr[ra] * h.x;
                float l1 = xl[rb] * h.y, r1 = xr[rb] * h.y;
#pragma unroll
                for (int t = 1; t < TE; ++t) {
                    h = hp[t];
                    l0 = l0 + xl[ra + t] * h.x;
                    r0 = r0 + xr[ra + t] * h.x;
                    if (two) {
                        l1 = l1 + xl[rb + t] * h.y;
                        r1 = r1 + xr[rb + t] * h.y;
                    }
                }
                const f2 acc0 = f2{l0, r0}, acc1 = f2{l1, r1};
                // exchange row kk: (track t, slot sp) at (t*S + sp + 4*kk) & 63
                const int kk0 = k - k0, kk1 = k + 1 - k0;
                X[kk0 * 64 + ((lane + 4 * kk0) & 63)] = acc0 * gk[kk0];
                if (two) X[kk1 * 64 + ((lane + 4 * kk1) & 63)] = acc1 * gk[kk1];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // ordered track sum: lane' = (slot sp', output kk'), NT tracks each;
            // 8 consecutive lanes store 8 consecutive frames (64 B) of one SP
            {
                constexpr int OPL = G * S / 64;            // outputs per lane (1 for NT = 8)
#pragma unroll
                for (int o = 0; o < OPL; ++o) {
                    const int idx = o * 64 + lane;
                    const int spo = idx / G, kk = idx % G;
                    if (k0 + kk < kend) {
                        f2 sum = X[kk * 64 + ((spo + 4 * kk) & 63)];
#pragma unroll
                        for (int t2 = 1; t2 < NT; ++t2) sum = sum + X[kk * 64 + ((t2 * S + spo + 4 * kk) & 63)];
                        sum = sum + f2{0.0f, 0.0f};        // -0 -> +0 (scipy seeds are +0)
                        const int64_t n = (int64_t)((task * S + spo) * a.R + r) * SPO + k0 + kk;
                        if (n < a.frames_out)
                            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, sum), ro,
                                                                  (uint32_t)n * 8u, 0, 0);
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // carry: the next SP's rel frames [21, 64) are this SP's [181, 224)
#pragma unroll
        for (int f = CARRY0; f < 2 * SEGF; ++f) {
            xl[f] = xl[f + SPI];
            xr[f] = xr[f + SPI];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA outstanding at exit
}

}  // namespace

// Host-side coefficient table for the fast path, pair-interleaved in output
// order: Hp[i][t] = (H[ph(2i)][t], H[ph(2i+1)][t]), t < 22, ph(k) =
// ((k+rm)*M) % L; the unpaired last output (k = 146) gets (h, 0).
// 74 * 22 * 2 floats (13 KiB) — the table xm_table_build() uploads.
extern "C" int xmh_fast_table_147_160(const float *H, int T, float *Hk /* >= 147*24 floats */)
{
    if (T != 23) return -1003;
    for (int ph = 0; ph < L; ++ph)
        if (H[ph * T + 22] != 0.0f) return -1003;   // tap 22 must be an exact zero
    for (int i = 0; i < (SPO + 1) / 2; ++i)
        for (int t = 0; t < TE; ++t) {
            const int k0 = 2 * i, k1 = 2 * i + 1;
            Hk[(i * TE + t) * 2 + 0] = H[(((k0 + RM) * M) % L) * T + t];
            Hk[(i * TE + t) * 2 + 1] = k1 < SPO ? H[(((k1 + RM) * M) % L) * T + t] : 0.0f;
        }
    return 0;
}

extern "C" int xmh_launch_mix_fast(const XmhMixJob *j, void *stream, int *n_launches)
{
    const int NT = j->n_tracks;
    const int64_t N = j->frames_in;
    if (!(j->rs.L == L && j->rs.M == M && j->rs.rm == RM && j->rs.T == 23 && j->rs.Hrun) ||
        j->fmt != 2 || j->channels != 2 || NT != 8 || j->in_ptrs || j->out_ptrs || !j->gains_host ||
        N <= 0 || (N & 1) || N >= (1 << 26) || j->n_mix <= 0)
        return -1003;   // not this kernel's job: generic path
    const int64_t tb = j->in_track_stride * 4;
    if (tb < N * 8 || (tb & 15) || ((uintptr_t)j->in & 15) || ((j->in_mix_stride * 4) & 15) ||
        (NT - 1) * tb + (N + 32) * 8 >= ((int64_t)1 << 31))
        return -1003;
    FastArgs a;
    memset(&a, 0, sizeof a);
    a.in = (const float *)j->in;
    a.in_mix_stride = j->in_mix_stride;
    a.track_bytes = tb;
    a.out = (float *)j->out;
    a.out_mix_stride = j->out_mix_stride;
    a.Hk = j->rs.Hrun;
    a.n_mix = j->n_mix;
    a.n_tracks = NT;
    a.frames_in = (int32_t)N;
    a.frames_out = (int32_t)j->frames_out;
    a.n_sp = (int32_t)((j->frames_out + SPO - 1) / SPO);
    const int S = 64 / NT;
    // SPs per lane: long runs amortise the per-task prologue; keep enough
    // tasks to fill the 2048 wave slots (8 per CU) several times over
    int R = 25;
    while (R > 1 && (int64_t)a.n_mix * ((a.n_sp + S * R - 1) / (S * R)) < 4 * 2048) R = (R + 1) / 2;
    a.R = R;
    a.tasks_per_mix = (a.n_sp + S * R - 1) / (S * R);
    a.unity = j->unity;
    for (int i = 0; i < NT; ++i) {
        a.g[i] = j->gains_host[i];
        const int64_t lim = (int64_t)1 << 28;   // outputs < 2^26: keeps clamp(n-start) unchanged
        a.g[i].start = a.g[i].start < -lim ? -lim : (a.g[i].start > lim ? lim : a.g[i].start);
    }
    const size_t lds = LDS_PER_WAVE;
    const int64_t blocks = (int64_t)a.n_mix * a.tasks_per_mix;
    if (blocks > 0x7fffffff) return -1003;
    auto kern = k_rs147_mix<8>;
    static bool attr_done;
    if (!attr_done) {
        if (hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return -1001;
        attr_done = true;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64), lds, (hipStream_t)stream, a);
    if (n_launches) *n_launches += 1;
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}
