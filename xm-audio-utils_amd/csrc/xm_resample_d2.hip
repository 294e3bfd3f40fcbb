// xm_resample_d2.hip — the fused resample + mix kernel at L/M = 147/320
// (96 kHz -> 44.1 kHz and every pair with that reduced ratio; round 5,
// SURVEY.md §8(f)2), stereo f32 interleaved mixes of 2-8 tracks.
//
// The same design as k_rs147_mix (csrc/xm_resample_fast.hip):
// a super-period (SP) is 320 input frames -> 147 outputs; a wave's 64 lanes
// are 8 track rows x 8 SP-run slots of one mix; input arrives by LDS-DMA in
// 256-B segments per stream into a 16-KiB slot; packed taps on (L, R) pairs of
// two outputs with the coefficient pair in an SGPR pair; the ordered track sum
// through 4 KiB of wave-private LDS.  What 147/320 changes:
//  * each output runs 43 or 44 used taps (kOffD2 / kNumD2, tools/gen_coefs.c
//    emit_offsets_t): an SP spans 12 segments (a 384-frame window, the last
//    64 frames carried to the next SP) and 10 of them are loaded per SP;
//  * TWO PHASES per output pair: taps 0..21 (phase A) when the pair's window
//    starts, taps 22.. (phase B) one round (8 outputs, 17.4 input frames)
//    later, when phase A of the pair 8 outputs on reads about the same frames.
//    The accumulators of four pairs wait between the phases.  Each output's
//    chain is still tap 0, 1, ..., n-1 in order, every product and add
//    separately rounded (the contract's order); the register window stays
//    ~29 frames of taps wide instead of 44 (44 at once would not fit two
//    waves per SIMD: VGPR-bound);
//  * outputs are complete one round after their phase A: the exchange writes
//    lag one round and the track sum stores round q - 2 at the start of round
//    q; every SP adds one drain round (phase B of its last round);
//  * coefficients are instruction literals (XM_LK_* blocks: s_mov_b32 into
//    s96-s99 ahead of the taps): the 26 KB pair table does not stay in the
//    scalar cache (the 320/147 kernel lost 40 % to those misses,
//    profiles/r5_h_u2_coef.txt);
//  * a segment's DMA goes out over 4 pairs (two parts per pair): an SP loads
//    10 segments over 80 pairs, so one part per pair would issue a segment's
//    last part right before its copy.
// Every vmcnt wait is an exact static count (Sched below).
#include <stdlib.h>
#include <string.h>
#include "xm_device.h"
#include "xm_coefs_147_160.h"   // generated: XM_FAST_RM_D2, kOffD2, kNumD2, kPtD2, XM_KHPD2_INIT
#include "xm_pk_taps.h"         // generated: XM_LK_* literal-coefficient blocks

#pragma clang diagnostic ignored "-Winline-asm"

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int SEGF = 32;                   // frames per DMA segment (256 B)
constexpr int NW = 12;                     // window segments
constexpr int WIN = NW * SEGF;             // 384 rel frames (relative to SPI*s - 32)
constexpr int L = 147, M = 320, T = 46, RM = XM_FAST_RM_D2;
constexpr int SPO = 147, SPI = 320;
constexpr int G = 8;                       // outputs per exchange round
constexpr int ROUNDS = (SPO + G - 1) / G;  // 19 rounds of phase A
constexpr int QN = ROUNDS + 1;             // + the drain round (phase B of round 18)
constexpr int KS = QN * G;                 // 160 output slots per SP
constexpr int TA = 22;                     // phase-A taps
constexpr int DLY = G;                     // phase B of output k runs at slot k + 8
constexpr int SLOT_BYTES = 64 * 256;
constexpr int X_F2 = G * 64;
constexpr int LDS_PER_WAVE = SLOT_BYTES + X_F2 * 8;   // 20 KiB
// (8 waves per CU, as the fused kernel: the split is xmg_pick_split's)
constexpr int WPB = 8;
constexpr uint32_t OOB = 0x80000000u;
constexpr int DMA_PARTS = 8;               // a segment's 16 DMA instructions, 2 per part
constexpr int PPP = 2;                     // DMA parts per output pair
constexpr int NPP = DMA_PARTS / PPP;       // pairs a segment's DMA spans

// first used tap's rel frame of output k
constexpr int rk(int k) { return ((k + RM) * M) / L - (T - 1) + 32 + kOffD2[k]; }
constexpr int imax(int a, int b) { return a > b ? a : b; }

// the last rel frame slot k's work reads: phase A of outputs k, k+1 (k <
// SPO), phase B of outputs k-8, k-7.  A pair runs kPtD2 taps for both of its
// outputs (the shorter one with +0 coefficients), so its frames reach rk + pt - 1
constexpr int last_frame_at(int k)
{
    int f = -1;
    if (k < SPO) f = imax(f, rk(k) + TA - 1);
    if (k + 1 < SPO) f = imax(f, rk(k + 1) + TA - 1);
    const int j = k - DLY;
    if (j >= 0 && j < SPO) f = imax(f, rk(j) + kPtD2[j / 2] - 1);
    if (j + 1 >= 0 && j + 1 < SPO) f = imax(f, rk(j + 1) + kPtD2[j / 2] - 1);
    return f;
}
constexpr int need_at(int k) { return k + 2 >= KS ? NW - 1 : (last_frame_at(k) < 0 ? 0 : last_frame_at(k) / SEGF); }
// segments copied by slot k: running maximum of the needs (copies only grow),
// tabulated once (a search per call site exceeds the constexpr step limit)
struct NeedTab {
    int v[KS / 2];
};
constexpr NeedTab make_need()
{
    NeedTab t{};
    int n = 1;
    for (int i = 0; i < KS; i += 2) {
        n = imax(n, need_at(i));
        t.v[i / 2] = n;
    }
    return t;
}
constexpr NeedTab NEED = make_need();
constexpr int needc(int k) { return NEED.v[k / 2]; }
constexpr int have_before(int k) { return k == 0 ? 1 : needc(k - 2); }
struct Tab {
    int v[NW + 1];
};
constexpr Tab make_kc()
{
    Tab t{};
    for (int m = 0; m <= NW; ++m) {
        t.v[m] = -1;
        for (int k = KS - 2; k >= 0; k -= 2)
            if (needc(k) >= m) t.v[m] = k;
    }
    return t;
}
constexpr Tab KC = make_kc();
constexpr int kc(int m) { return KC.v[m]; }
// the frames before an SP: its first slots need segments 0, 1 only (carried)
constexpr int carry0()
{
    int c = WIN;
    for (int k = 0; k < SPO; ++k) c = rk(k) < c ? rk(k) : c;
    return c;
}
constexpr int CARRY0 = carry0();
static_assert(CARRY0 >= 0 && need_at(0) <= 1, "an SP's first taps read the carried segments");
static_assert(2 * SEGF + SPI <= WIN, "the carry's source lies inside the window");
static_assert(rk(SPO - 1) + kPtD2[(SPO - 1) / 2] - 1 < WIN, "an SP's taps lie inside the window");

// store events: slot q*G of round q, except round 1 (nothing completed yet);
// round q stores output round q - 2 (q == 0: the previous SP's round 18)
constexpr bool store_at(int k) { return k % G == 0 && k / G != 1; }
constexpr int dma_start(int m) { return m == 2 ? kc(NW - 1) : kc(m - 1); }
constexpr int dma_last(int m) { return dma_start(m) + 2 * (NPP - 1) - (m == 2 ? KS : 0); }
// first of the PPP parts of segment m issued at slot k (-1: none); for m == 2
// `next` selects the parts of the following SP's segment 2
constexpr int part_at(int k, int m, bool next)
{
    if (m != 2 || next) {
        const int j = (k - dma_start(m)) / 2;
        return k >= dma_start(m) && j < NPP ? j * PPP : -1;
    }
    const int j = (k + KS - dma_start(2)) / 2;   // tail parts of this SP's own segment 2
    return j < NPP ? j * PPP : -1;
}
constexpr int stores_in(int lo, int hi)
{
    int n = 0;
    for (int k = 0; k < KS; k += 2) {
        if (store_at(k) && k >= lo && k < hi) ++n;
        if (store_at(k) && k - KS >= lo) ++n;   // lo < 0: the previous SP's store events from it on
    }
    return n;
}
constexpr int vm_after(int m) { return stores_in(dma_last(m), kc(m)); }
constexpr int prologue_stores()
{
    int n = 0;
    for (int k = 0; k < KS; k += 2)
        if (store_at(k) && k - KS >= dma_last(2)) ++n;
    return n;
}
constexpr bool sched_ok()
{
    for (int m = 2; m < NW; ++m) {
        if (kc(m) < 0 || dma_last(m) >= kc(m) || vm_after(m) >= 64) return false;
        int seen = 0;
        for (int k = 0; k < KS; k += 2)
            for (int nx = 0; nx < (m == 2 ? 2 : 1); ++nx) {
                const int p = part_at(k, m, nx != 0);
                if (p < 0) continue;
                if (p >= DMA_PARTS) return false;
                ++seen;
            }
        if (seen != NPP) return false;
    }
    return true;
}
static_assert(sched_ok(), "every segment's DMA issued once, within the slot, before its copy; vmcnt fits");
constexpr bool sched8_ok()   // 1-track rows: 8 stores per store event
{
    for (int m = 2; m < NW; ++m)
        if (8 * vm_after(m) >= 64) return false;
    return true;
}
static_assert(sched8_ok(), "1-track rows: vmcnt fits 8 stores per store event");

struct D2Args {
    const float *in;
    int64_t in_mix_stride;     // samples
    int64_t track_bytes;
    float *out;
    int64_t out_mix_stride;    // samples
    int32_t n_mix, n_tracks;
    int32_t frames_in, frames_out;
    int32_t n_sp, R, tasks_per_mix;
    int32_t out_s16;           // 1: the f32 mix stored as s16 = sat16(rint(y * 32768)) (out strides in s16 samples)
    XmhGain g[8];
    const float *const *in_ptrs;
    float *const *out_ptrs;
};

static constexpr float kHpD2h[75][88] = XM_KHPD2_INIT;   // host copy: the literals

__device__ __forceinline__ unsigned lit(int e) { return __builtin_bit_cast(unsigned, (&kHpD2h[0][0])[e]); }

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

#define XM_AL ".p2align 3\n\t"

// ODD: odd frames_in or row bases off the 128-B grid (copy_seg zeroes frame N
// of a chunk straddling it; the DMA keeps the line two segments share in L2)
// SPL (round 5): 1-track rows, eight resample-only clips per wave (a
// timeline's per-track resampling, batches of clips): row t is clip
// 8 * mix + t (mix = the wave's pseudo-mix), each stored to its own output
// (8 stores per store event: vm_after is at most 2 events, 16 < 64)
template <bool ODD, bool SPL>
__global__ __launch_bounds__(64 * WPB) void k_rs_d2_mix(D2Args a)
{
    constexpr int NS = SPL ? 8 : 1;             // stores per store event
    extern __shared__ __attribute__((aligned(16))) char lds_all[];
    const int wib = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char *lds = lds_all + wib * LDS_PER_WAVE;
    const int gw = (int)blockIdx.x * WPB + wib;
    constexpr int S = 8, TR = 8;
    const int lane = threadIdx.x & 63;
    const int tr = lane / S, spl = lane % S;
    const int mix = gw / a.tasks_per_mix;
    const int task = gw % a.tasks_per_mix;
    const int s_first = (task * S + spl) * a.R;
    const char *slot = lds;
    f2 *X = (f2 *)(lds + SLOT_BYTES);
    const uint32_t ldsb = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void *)lds);

    // one resource per mix, based 32 frames before its lowest track
    uint64_t mb;
    uint32_t toff[TR], span;
    {
        uint64_t p[TR], lo = ~0ull, hi = 0;
        bool ok[TR];
#pragma unroll
        for (int t = 0; t < TR; ++t) {
            const int64_t ci = (int64_t)mix * TR + t;   // SPL: this row's clip
            ok[t] = SPL ? ci < a.n_mix : (t < a.n_tracks && mix < a.n_mix);
            if (a.in_ptrs)
                p[t] = ok[t] ? (uint64_t)(uintptr_t)a.in_ptrs[SPL ? ci : (int64_t)mix * a.n_tracks + t] : 0;
            else if (SPL)
                p[t] = (uint64_t)(uintptr_t)((const char *)a.in + ci * a.in_mix_stride * 4);
            else
                p[t] = (uint64_t)(uintptr_t)((const char *)a.in + (int64_t)mix * a.in_mix_stride * 4 + (int64_t)t * a.track_bytes);
            if (ok[t]) {
                lo = p[t] < lo ? p[t] : lo;
                hi = p[t] > hi ? p[t] : hi;
            }
        }
        if (lo > hi) lo = hi = (uint64_t)(uintptr_t)a.in;   // a padding wave
        mb = lo - 32 * 8;
#pragma unroll
        for (int t = 0; t < TR; ++t) toff[t] = __builtin_amdgcn_readfirstlane(ok[t] ? (uint32_t)(p[t] - lo) : OOB);
        span = (uint32_t)(hi - lo);
    }
    i4 rs;
    rs.x = (int)__builtin_amdgcn_readfirstlane((uint32_t)mb);
    rs.y = (int)__builtin_amdgcn_readfirstlane((uint32_t)(mb >> 32) & 0xffffu);
    rs.z = (int)__builtin_amdgcn_readfirstlane((uint32_t)(span + ((int64_t)a.frames_in + 32) * 8));
    rs.w = 0x00020000;

    // DMA addressing: instruction d covers streams 4d..4d+3; lane l loads
    // chunk ((l & 15) - q) & 15 of stream q = 4d + (l >> 4) (rotated: the copy's
    // ds_read_b128 are conflict-free)
    const int lq = lane >> 4;
    uint32_t vl[4];
#pragma unroll
    for (int d4 = 0; d4 < 4; ++d4) {
        const int j = ((lane & 15) - lq - 4 * d4) & 15;
        vl[d4] = (uint32_t)((task * S + lq) * a.R * (SPI * 8) + j * 16);
    }
    const uint32_t GR = __builtin_amdgcn_readfirstlane((uint32_t)(4 * a.R * (SPI * 8)));
    const int N = a.frames_in;
    const int RH = a.R;

    auto edge_of = [&](int r) __attribute__((always_inline)) {
        const bool e = s_first + r == 0 || (s_first + r) * SPI + (WIN - 32) > N;
        return __builtin_amdgcn_readfirstlane((int)(__builtin_amdgcn_ballot_w64(e) != 0)) != 0;
    };
    auto dma_part = [&](int r, int m, int jp, bool edge) __attribute__((always_inline)) {
        const uint32_t rb0 = (uint32_t)(r * (SPI * 8) + m * (SEGF * 8));
        const uint32_t rb1 = rb0 + GR;
        if (jp == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous copy's reads of the slot
#pragma unroll
        for (int d = 2 * jp; d < 2 * jp + 2; ++d) {
            uint32_t so;
            uint32_t v = vl[d & 3];
            if (__builtin_expect(edge, 0)) {
                const int f = (int)(vl[d & 3] >> 3) - 32 + 4 * (d & 1) * a.R * SPI + r * SPI + m * SEGF;
                v = (f >= 0 && f < N) ? v : OOB;   // a chunk wholly outside [0, N): zero-filled
            }
#define XM_D2_DMA(POL)                                                                                          \
    asm volatile("s_add_u32 %0, %1, %2\n\t"                                                                     \
                 "s_add_u32 m0, %3, %4\n\t"                                                                     \
                 "s_nop 0\n\t"                                                                                  \
                 "buffer_load_dwordx4 %5, %6, %0 offen" POL " lds"                                              \
                 : "=&s"(so)                                                                                    \
                 : "s"(toff[d / 2]), "s"((d & 1) ? rb1 : rb0), "s"(ldsb), "n"(d * 1024), "v"(v), "s"(rs)       \
                 : "memory", "scc", "m0")
            if constexpr (ODD) XM_D2_DMA(" sc1");
            else XM_D2_DMA(" nt");
#undef XM_D2_DMA
        }
    };
    auto dma = [&](int r, int m, bool edge) __attribute__((always_inline)) {
#pragma unroll
        for (int jp = 0; jp < DMA_PARTS; ++jp) dma_part(r, m, jp, edge);
    };
    f2 x2[WIN];
    auto copy_seg = [&](int m, auto vm, int r, bool edge) __attribute__((always_inline)) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(vm)::value) : "memory");
        const char *base = slot + (lane >> 2) * 1024 + (lane & 3) * 256;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float4 v = *(const float4 *)(base + (((j + lane) & 15) * 16));
            x2[SEGF * m + 2 * j] = f2{v.x, v.y};
            x2[SEGF * m + 2 * j + 1] = f2{v.z, v.w};
        }
        if (ODD && __builtin_expect(edge, 0)) {   // odd N: frame N of the chunk straddling it reads as zero
            const int nrel = N - ((s_first + r) * SPI - 32 + m * SEGF);
#pragma unroll
            for (int j = 0; j < 16; ++j) x2[SEGF * m + 2 * j + 1] = 2 * j + 1 >= nrel ? f2{0.0f, 0.0f} : x2[SEGF * m + 2 * j + 1];
        }
    };

    XmhGain gp = a.g[0];
#pragma unroll
    for (int i = 1; i < TR; ++i)
        if (!SPL && tr == i) gp = a.g[i];
    const bool xf = (gp.flags & XMH_GAIN_XFADE_OUT) != 0;

    const bool mix_ok = (int64_t)mix * (SPL ? TR : 1) < a.n_mix;
    // output f32 (L, R) pairs, or with out_s16 the s16 pairs of the converted mix
    const int osz = a.out_s16 ? 2 : 4;          // bytes per output sample
    // SPL: the clips of this wave at outb + g * clip_bytes (g < n_grp)
    const int n_grp = SPL ? (int)min((int64_t)TR, a.n_mix - (int64_t)mix * TR) : 1;
    const uint32_t clip_bytes = SPL ? (uint32_t)a.out_mix_stride * (uint32_t)osz : 0u;
    char *outb = a.out_ptrs ? (mix_ok ? (char *)a.out_ptrs[mix] : (char *)a.out)
                            : (char *)a.out + (int64_t)mix * (SPL ? TR : 1) * a.out_mix_stride * osz;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        outb, (short)0, mix_ok ? (int)((uint32_t)(n_grp - 1) * clip_bytes + (uint32_t)a.frames_out * 2u * (uint32_t)osz) : 0,
        0x00020000);
    // f32 -> s16 store epilogue (XM_MIXER_OUT_CONVERT; the fused and generic
    // kernels' xm_round_sat16(y * 32768)), both channels in one dword
    auto pack_s16 = [](f2 v) __attribute__((always_inline)) {
        const int32_t l = xm_round_sat16(v.x * 32768.0f), r = xm_round_sat16(v.y * 32768.0f);
        return ((uint32_t)l & 0xffffu) | ((uint32_t)r << 16);
    };
    // one store per (group, store event) either way: the vmcnt counts hold
    auto store_pair = [&](f2 v, bool ok, uint32_t base, int n) __attribute__((always_inline)) {
        if (a.out_s16)   // wave-uniform
            __builtin_amdgcn_raw_buffer_store_b32(pack_s16(v), ro, ok ? base + (uint32_t)n * 4u : OOB, 0, 0);
        else
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), ro, ok ? base + (uint32_t)n * 8u : OOB, 0, 0);
    };

    // track sum: lane' = (slot spo, output kk of the round); rows of every
    // track in track order (phantom rows add +-0)
    const int spo = (lane / G) % S, kkp = lane % G;
    f2 pend[TR];
    auto sum_store = [&](int rp, int qp, bool valid) __attribute__((always_inline)) {
#pragma unroll
        for (int t2 = 0; t2 < TR; ++t2) pend[t2] = X[kkp * 64 + ((t2 * S + spo + 4 * kkp) & 63)];
        if constexpr (SPL) {   // each row its own 1-track mix (+ 0), all 8 stores issued (vmcnt)
            const int kq = qp * G + kkp;
            const int n = ((task * S + spo) * a.R + rp) * SPO + kq;
            const bool ok = valid && kq < SPO && n < a.frames_out;
#pragma unroll
            for (int g = 0; g < TR; ++g) store_pair(pend[g] + f2{0.0f, 0.0f}, ok, (uint32_t)g * clip_bytes, n);
            return;
        }
        f2 v = pend[0];
#pragma unroll
        for (int k = 1; k < TR; ++k) v = v + pend[k];
        v = v + f2{0.0f, 0.0f};   // -0 -> +0 (scipy seeds are +0)
        const int kq = qp * G + kkp;
        const int n = ((task * S + spo) * a.R + rp) * SPO + kq;
        store_pair(v, valid && kq < SPO && n < a.frames_out, 0u, n);
    };

    // prologue: segments 0, 1 in registers; segment 2's parts a previous SP
    // would have issued, and as many (dropped) stores as it issues after them
    const bool edge0 = edge_of(0);
    dma(0, 0, edge0);
    copy_seg(0, std::integral_constant<int, 0>{}, 0, edge0);
    dma(0, 1, edge0);
    copy_seg(1, std::integral_constant<int, 0>{}, 0, edge0);
#pragma unroll
    for (int i = 0; i < NPP; ++i)
        if (part_at(dma_start(2) + 2 * i, 2, true) == i * PPP && dma_start(2) + 2 * i < KS)
#pragma unroll
            for (int q = 0; q < PPP; ++q) dma_part(0, 2, i * PPP + q, edge0);
#pragma unroll
    for (int i = 0; i < NS * prologue_stores(); ++i) __builtin_amdgcn_raw_buffer_store_b32(0u, ro, OOB, 0, 0);

    f2 acc[4][2];   // phase-A results of the pairs waiting for phase B (pair index % 4)
#pragma unroll 1
    for (int r = 0; r < RH; ++r) {
        const int s = s_first + r;
        const int n_sp0 = s * SPO;
        // gain class of this lane over the SP: 0 constant, 1 linear, 2 boundary
        int cls;
        float cA, cB = 0.0f, fkb = 0.0f;
        {
            const int st = (int)gp.start, ln = gp.len;
            const int lo = n_sp0, hi = lo + SPO - 1;
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
        const bool edge_cur = edge_of(r), edge_next = edge_of(r + 1);
        f2 gpr[G / 2];
#pragma unroll
        for (int p = 0; p < G / 2; ++p) gpr[p] = f2{cA, cA};

#pragma unroll
        for (int q = 0; q < QN; ++q) {
            const int k0 = q * G;
            // gains of the outputs completing in this round: round q - 1
            if (q >= 1) {
                const int o0 = k0 - G;
                if (any_bnd) {
#pragma unroll
                    for (int p = 0; p < G / 2; ++p)
                        gpr[p] = f2{gain_exact(gp, n_sp0 + o0 + 2 * p), gain_exact(gp, n_sp0 + o0 + 2 * p + 1)};
                } else if (any_lin) {
#pragma unroll
                    for (int p = 0; p < G / 2; ++p) {
                        const f2 kf = f2{fkb, fkb} + f2{(float)(o0 + 2 * p), (float)(o0 + 2 * p + 1)};
                        gpr[p] = f2{cA, cA} + f2{cB, cB} * kf;
                    }
                }
            }
#pragma unroll
            for (int k = k0; k < k0 + G; k += 2) {
                // 1. the segments this slot's taps need
#pragma unroll
                for (int m = have_before(k) + 1; m <= needc(k); ++m) {
                    if (m == 2) copy_seg(2, std::integral_constant<int, NS * vm_after(2)>{}, r, edge_cur);
                    if (m == 3) copy_seg(3, std::integral_constant<int, NS * vm_after(3)>{}, r, edge_cur);
                    if (m == 4) copy_seg(4, std::integral_constant<int, NS * vm_after(4)>{}, r, edge_cur);
                    if (m == 5) copy_seg(5, std::integral_constant<int, NS * vm_after(5)>{}, r, edge_cur);
                    if (m == 6) copy_seg(6, std::integral_constant<int, NS * vm_after(6)>{}, r, edge_cur);
                    if (m == 7) copy_seg(7, std::integral_constant<int, NS * vm_after(7)>{}, r, edge_cur);
                    if (m == 8) copy_seg(8, std::integral_constant<int, NS * vm_after(8)>{}, r, edge_cur);
                    if (m == 9) copy_seg(9, std::integral_constant<int, NS * vm_after(9)>{}, r, edge_cur);
                    if (m == 10) copy_seg(10, std::integral_constant<int, NS * vm_after(10)>{}, r, edge_cur);
                    if (m == 11) copy_seg(11, std::integral_constant<int, NS * vm_after(11)>{}, r, edge_cur);
                }
                f2 p0, p1, p2, p3;
                // 2. phase B of outputs k-8, k-7: taps 22.. continuing their chains
                const int j = k - DLY;
                const bool hasB = j >= 0 && j < SPO;
                f2 w0 = f2{0.0f, 0.0f}, w1 = f2{0.0f, 0.0f};
                if (hasB) {
                    const int pi = j >> 1, ps = pi & 3;
                    const bool two = j + 1 < SPO;
                    const int ra = rk(j), rb = rk(two ? j + 1 : j);
                    const int pt = kPtD2[pi];
                    const int rowb = pi * 88;
                    f2 a0 = acc[ps][0], a1 = acc[ps][1];
#define XM_LKB(t) "i"(lit(rowb + 2 * (t))), "i"(lit(rowb + 2 * (t) + 1)), "v"(x2[ra + (t)]), "v"(x2[rb + (t)])
#define XM_LKB1(t) "i"(lit(rowb + 2 * (t))), "v"(x2[ra + (t)])
#pragma unroll
                    for (int b = TA; b < TA + 24; b += 4) {
                        if (b >= pt) break;
                        const int n = pt - b < 4 ? pt - b : 4;
                        if (two) {
                            if (n == 4)
                                asm volatile(XM_AL XM_LK_R4_TWO : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB(b), XM_LKB(b + 1), XM_LKB(b + 2), XM_LKB(b + 3) : XM_LK_CLOBBER);
                            else if (n == 3)
                                asm volatile(XM_AL XM_LK_R3_TWO : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB(b), XM_LKB(b + 1), XM_LKB(b + 2) : XM_LK_CLOBBER);
                            else if (n == 2)
                                asm volatile(XM_AL XM_LK_R2_TWO : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB(b), XM_LKB(b + 1) : XM_LK_CLOBBER);
                            else
                                asm volatile(XM_AL XM_LK_R1_TWO : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB(b) : XM_LK_CLOBBER);
                        } else {
                            if (n == 4)
                                asm volatile(XM_AL XM_LK_R4_ONE : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB1(b), XM_LKB1(b + 1), XM_LKB1(b + 2), XM_LKB1(b + 3) : XM_LK_CLOBBER);
                            else if (n == 3)
                                asm volatile(XM_AL XM_LK_R3_ONE : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB1(b), XM_LKB1(b + 1), XM_LKB1(b + 2) : XM_LK_CLOBBER);
                            else if (n == 2)
                                asm volatile(XM_AL XM_LK_R2_ONE : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB1(b), XM_LKB1(b + 1) : XM_LK_CLOBBER);
                            else
                                asm volatile(XM_AL XM_LK_R1_ONE : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB1(b) : XM_LK_CLOBBER);
                        }
                    }
                    // outputs j, j+1 complete: (L, R) times their gains (packed, op_sel)
                    const int pp = (j - (k0 - G)) >> 1;
                    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(w0) : "v"(a0), "v"(gpr[pp]));
                    if (two) asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(w1) : "v"(a1), "v"(gpr[pp]));
                }
                // 3. phase A of outputs k, k+1: taps 0..21, new chains
                if (k < SPO) {
                    const int pi = k >> 1, ps = pi & 3;
                    const bool two = k + 1 < SPO;
                    const int ra = rk(k), rb = rk(two ? k + 1 : k);
                    const int rowb = pi * 88;
                    f2 a0, a1 = f2{0.0f, 0.0f};
#pragma unroll
                    for (int b = 0; b < TA; b += 4) {
                        const int n = TA - b < 4 ? TA - b : 4;
                        if (two) {
                            if (b == 0)
                                asm volatile(XM_AL XM_LK_F4_TWO : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "=&v"(a0), "=&v"(a1)
                                             : XM_LKB(0), XM_LKB(1), XM_LKB(2), XM_LKB(3) : XM_LK_CLOBBER);
                            else if (n == 4)
                                asm volatile(XM_AL XM_LK_R4_TWO : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB(b), XM_LKB(b + 1), XM_LKB(b + 2), XM_LKB(b + 3) : XM_LK_CLOBBER);
                            else
                                asm volatile(XM_AL XM_LK_R2_TWO : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB(b), XM_LKB(b + 1) : XM_LK_CLOBBER);
                        } else {
                            if (b == 0)
                                asm volatile(XM_AL XM_LK_F4_ONE : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "=&v"(a0), "=&v"(a1)
                                             : XM_LKB1(0), XM_LKB1(1), XM_LKB1(2), XM_LKB1(3) : XM_LK_CLOBBER);
                            else if (n == 4)
                                asm volatile(XM_AL XM_LK_R4_ONE : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB1(b), XM_LKB1(b + 1), XM_LKB1(b + 2), XM_LKB1(b + 3) : XM_LK_CLOBBER);
                            else
                                asm volatile(XM_AL XM_LK_R2_ONE : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                             : XM_LKB1(b), XM_LKB1(b + 1) : XM_LK_CLOBBER);
                        }
                    }
#undef XM_LKB
#undef XM_LKB1
                    acc[ps][0] = a0;
                    acc[ps][1] = a1;
                }
                // 4. refill: this SP's segments 3..11, the tail of its segment
                // 2 and the head of the next SP's segment 2 (ahead of the stores)
#pragma unroll
                for (int m = 3; m < NW; ++m)
                    if (part_at(k, m, false) >= 0)
#pragma unroll
                        for (int qq = 0; qq < PPP; ++qq) dma_part(r, m, part_at(k, m, false) + qq, edge_cur);
                if (part_at(k, 2, false) >= 0)
#pragma unroll
                    for (int qq = 0; qq < PPP; ++qq) dma_part(r, 2, part_at(k, 2, false) + qq, edge_cur);
                if (part_at(k, 2, true) >= 0 && r + 1 < RH)
#pragma unroll
                    for (int qq = 0; qq < PPP; ++qq) dma_part(r + 1, 2, part_at(k, 2, true) + qq, edge_next);
                // 5. the track sum of output round q - 2 (its rows were written
                // during round q - 1), before this round's rows overwrite them
                if (k == k0 && store_at(k)) {
                    if (q == 0) sum_store(r - 1, ROUNDS - 1, r > 0);
                    else sum_store(r, q - 2, true);
                }
                // 6. exchange rows of the completed outputs
                if (hasB) {
                    const int kk0 = k - k0, kk1 = kk0 + 1;
                    X[kk0 * 64 + ((lane + 4 * kk0) & 63)] = w0;
                    if (j + 1 < SPO) X[kk1 * 64 + ((lane + 4 * kk1) & 63)] = w1;
                }
            }
        }
        // carry: the next SP's rel frames [CARRY0, 64) are this SP's [CARRY0 + 320, 384)
#pragma unroll
        for (int f = CARRY0; f < 2 * SEGF; ++f) x2[f] = x2[f + SPI];
        asm volatile("s_barrier" ::: "memory");
    }
    sum_store(RH - 1, ROUNDS - 1, true);   // round 18 of the last SP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the wave's LDS is gone
}

}  // namespace

// the pair table as baked must be the run-time design's (both come from
// xm_resample_design; this guards against a stale build): output k runs taps
// kOffD2[k] .. + kNumD2[k] - 1, every other tap of its phase +0
extern "C" int xmg_d2_table_check(const float *H, int Lr, int Mr, int Tr)
{
    if (Lr != L || Mr != M || Tr != T) return -1003;
    for (int k = 0; k < L; ++k) {
        const int ph = (int)(((long)(k + RM) * M) % L);
        for (int t = 0; t < T; ++t) {
            const int e = t - kOffD2[k];
            const float want = e >= 0 && e < kNumD2[k] ? kHpD2h[k / 2][2 * e + (k & 1)] : 0.0f;
            if (__builtin_bit_cast(uint32_t, H[ph * T + t]) != __builtin_bit_cast(uint32_t, want)) return -1003;
        }
    }
    return 0;
}

// SPs per lane and tasks per mix: the fused kernel's split (xmg_pick_split,
// csrc/xm_resample_fast.hip; 8 waves per CU here too) and its test override
static void d2_split(int64_t n_mix, int n_sp, int *R_out, int *tpm_out)
{
    const int S = 8;
    xmg_pick_split(n_mix, n_sp, S, R_out, tpm_out);
    if (const int fR = xmg_forced_split_r()) {
        *R_out = fR;
        *tpm_out = (n_sp + S * fR - 1) / (S * fR);
    }
}

// -1003: not this kernel's job (the caller tries the others); R, tpm: the split
extern "C" int xmg_launch_mix_d2(const XmhMixJob *j, void *stream, int *n_launches, int *R_out, int *tpm_out)
{
    const int NT = j->n_tracks;
    const int64_t Nf = j->frames_in;
    if (j->rs.L != L || j->rs.M != M || j->rs.T != T || j->rs.rm != RM || !j->rs.fast) return -1003;
    if (j->channels != 2 || j->fmt != 2 || j->io_flags || j->out_conv > 1 || j->out_conv < 0 || j->window || j->in_base || j->out_base ||
        j->partial || !j->gains_host || NT < 1 || NT > 8 || Nf <= 0 || Nf >= (1 << 26) || j->n_mix <= 0 ||
        (j->in_ptrs && !j->in_ptrs_host))
        return -1003;
    const bool spl = NT == 1;   // 1-track rows: eight clips per wave
    if (spl && j->out_ptrs) return -1003;   // per-clip output tables: generic path
    const int64_t npm = spl ? (j->n_mix + 7) / 8 : j->n_mix;   // the waves' pseudo-mixes
    const int64_t lim = ((int64_t)1 << 31) - (Nf + 32) * 8;
    uintptr_t mis = 0;
    if (j->in_ptrs) {
        for (int64_t mi = 0; mi < npm; ++mi) {
            uintptr_t lo = UINTPTR_MAX, hi = 0;
            for (int t = 0; t < (spl ? 8 : NT); ++t) {
                if (spl && mi * 8 + t >= j->n_mix) break;
                const uintptr_t p = (uintptr_t)j->in_ptrs_host[spl ? mi * 8 + t : mi * NT + t];
                if (p & 3) return -1003;
                mis |= p;
                lo = p < lo ? p : lo;
                hi = p > hi ? p : hi;
            }
            if (lo < 256 || (int64_t)(hi - lo) >= lim) return -1003;
        }
    } else {
        const int64_t tb = j->in_track_stride * 4, mb = j->in_mix_stride * 4;
        const int64_t atb = tb < 0 ? -tb : tb;
        const int64_t amb = mb < 0 ? -mb : mb;
        if ((atb & 3) || (mb & 3) || ((uintptr_t)j->in & 3) || (!spl && atb < Nf * 8)) return -1003;
        if (!spl && (int64_t)(NT - 1) * atb >= lim) return -1003;
        if (spl && j->n_mix > 1 && (amb < Nf * 8 || 7 * amb >= lim)) return -1003;
        mis = (uintptr_t)j->in | (uintptr_t)atb | (uintptr_t)(j->n_mix > 1 ? (mb < 0 ? -mb : mb) : 0);
    }
    const int64_t osz = j->out_conv == 1 ? 2 : 4;   // bytes per output sample (s16 out: XM_MIXER_OUT_CONVERT)
    if (j->frames_out * 2 * osz >= ((int64_t)1 << 31)) return -1003;
    if (spl && (j->out_mix_stride < j->frames_out * 2 || 7 * j->out_mix_stride * osz + j->frames_out * 2 * osz >= ((int64_t)1 << 31)))
        return -1003;
    D2Args a;
    memset(&a, 0, sizeof a);
    a.in = (const float *)j->in;
    a.in_ptrs = (const float *const *)j->in_ptrs;
    a.out_ptrs = (float *const *)j->out_ptrs;
    a.in_mix_stride = j->in_mix_stride;
    a.track_bytes = j->in_track_stride * 4;
    a.out = (float *)j->out;
    a.out_mix_stride = j->out_mix_stride;
    a.out_s16 = j->out_conv == 1;
    a.n_mix = j->n_mix;
    a.n_tracks = NT;
    a.frames_in = (int32_t)Nf;
    a.frames_out = (int32_t)j->frames_out;
    a.n_sp = (int32_t)((j->frames_out + SPO - 1) / SPO);
    d2_split(npm, a.n_sp, &a.R, &a.tasks_per_mix);
    for (int i = 0; i < NT; ++i) {
        a.g[i] = j->gains_host[i];
        const int64_t glim = (int64_t)1 << 28;
        a.g[i].start = a.g[i].start < -glim ? -glim : (a.g[i].start > glim ? glim : a.g[i].start);
    }
    const int64_t waves = npm * a.tasks_per_mix;
    const int64_t blocks = (waves + WPB - 1) / WPB;
    if (blocks > 0x7fffffff / WPB) return -1003;
    const bool odd = (Nf & 1) != 0 || (mis & 127) != 0;
    const void *kern = spl ? (odd ? (const void *)k_rs_d2_mix<true, true> : (const void *)k_rs_d2_mix<false, true>)
                           : (odd ? (const void *)k_rs_d2_mix<true, false> : (const void *)k_rs_d2_mix<false, false>);
    if (xmg_func_lds(kern, WPB * LDS_PER_WAVE)) return -1001;
    void *kargs[] = {&a};
    if (hipLaunchKernel(kern, dim3((unsigned)blocks), dim3(64 * WPB), kargs, (size_t)(WPB * LDS_PER_WAVE),
                        (hipStream_t)stream) != hipSuccess)
        return -1001;
    if (n_launches) *n_launches += 1;
    if (hipGetLastError() != hipSuccess) return -1001;
    if (R_out) *R_out = a.R;
    if (tpm_out) *tpm_out = a.tasks_per_mix;
    return 0;
}
