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
//    phase of output k of an SP does not depend on the SP, so a wave whose 64
//    lanes are 64 SP streams runs one wave-uniform, fully unrolled sequence of
//    v_mul_f32 / v_add_f32 whose coefficients are instruction literals (the
//    table is baked at build time by tools/gen_coefs.c from the same design
//    code the host runs; the host checks they agree before using this kernel).
//    No scalar loads, so no lgkmcnt stalls in the tap loop: with 2 waves per
//    SIMD a single stalled wave halves VALU issue (tools/ubench/dep_latency.hip).
//  * lanes = 8 tracks x 8 stream slots of one mix.  Each lane walks R
//    consecutive SPs of its track, so its input is one contiguous stream and
//    the register window carries across SPs (43 frames moved per SP).
//  * input arrives by LDS-DMA (buffer_load_dwordx4 ... lds) in 256-B segments
//    per stream: one DMA instruction = 4 streams x 256 B.  Measured on MI355X
//    (tools/ubench/mem_pattern.hip): 16 lanes per 256-B segment streams at
//    6.3 TB/s, whereas one 16-B stream per lane caps at 4.2 TB/s.  Chunks are
//    rotated per stream so the LDS->VGPR copy (ds_read_b128) is bank-conflict
//    free; buffer range checks plus explicit redirects zero-fill frames outside
//    [0, N).  The DMA is issued from inline asm so the compiler's conservative
//    "vmcnt(0) before any LDS read" is not inserted; this file owns every
//    vmcnt wait, with exact static counts (stores are never predicated off:
//    out-of-range offsets are dropped by the buffer descriptor instead).
//  * the ordered track sum is exchanged through 4 KiB of wave-private LDS
//    (rows rotated instead of padded), software-pipelined one round deep: the
//    reads of round q are issued at the start of round q+1 and consumed after
//    its first output pair.  No barriers: LDS ops of one wave execute in order.
//  * LDS per wave = 16 KiB slot + 4 KiB exchange = 20 KiB -> 8 waves/CU.
#include <stdlib.h>
#include <string.h>
#include <type_traits>
#include "xm_device.h"
#include "xm_coefs_147_160.h"   // generated: kH147[147][22], XM_FAST_RM

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int L = 147, M = 160, RM = XM_FAST_RM;   // reduced ratio, output offset rm
static_assert(RM == 11, "48k->44.1k design");
constexpr int TE = 22;                     // taps used (tap 22 is an exact zero)
constexpr int SPO = L;                     // outputs per super-period
constexpr int SPI = M;                     // input frames per super-period
constexpr int SEGF = 32;                   // frames per DMA segment (256 B)
constexpr int G = 8;                       // outputs per exchange round
constexpr int ROUNDS = (SPO + G - 1) / G;  // 19
constexpr int CARRY0 = 21;                 // first rel frame an SP needs
constexpr int WIN = 7 * SEGF;              // 224 rel frames: SP s uses rel [21, 201]
constexpr int SLOT_BYTES = 64 * 256;       // one segment for 64 streams
constexpr int X_F2 = G * 64;               // exchange: 8 outputs x 64 lanes (f2)
constexpr int LDS_PER_WAVE = SLOT_BYTES + X_F2 * 8;   // 20 KiB
constexpr int WAVES_PER_CU = 8;            // LDS-bound: 160 KiB / 20 KiB
constexpr uint32_t OOB = 0x80000000u;      // offset beyond every num_records

// rel frame (relative to 160*s - 32) of tap 0 of output k of SP s
// (scipy: j0 = floor((m+rm)*M/L) - T + 1, T = 23)
__host__ __device__ constexpr int rk(int k) { return ((k + RM) * M) / L - 22 + 32; }
// segment (0..6 of the SP's 7) holding the last frame output k needs
constexpr int last_seg(int k) { return (rk(k) + TE - 1) / SEGF; }
// last segment needed by the pair starting at even k
constexpr int need_pair(int k) { return last_seg(k + 1 < SPO ? k + 1 : k); }
static_assert(rk(0) == CARRY0, "window origin");
static_assert(last_seg(SPO - 1) == 6, "an SP spans 7 segments");
static_assert(last_seg(0) == 1, "first outputs need segments 0,1");

// ---- static per-SP schedule.  Within output pair k (even) the order is:
//   copies of newly needed segments (LDS -> VGPR)
//   compute of outputs k, k+1
//   if k % G == 0: track sum + store of the previous round
//   DMA of the segment after each one copied here
//   exchange writes of outputs k, k+1
// E = how many segments ahead of need a segment is copied into registers.
template <int E>
struct Sched {
    static constexpr int needc(int k) { return need_pair(k) + E > 6 ? 6 : need_pair(k) + E; }
    static constexpr int have_before(int k) { return k == 0 ? 1 : needc(k - 2); }
    static constexpr int kc(int m)   // pair whose copies include segment m (m >= 2)
    {
        for (int k = 0; k < SPO; k += 2)
            if (needc(k) >= m) return k;
        return -1;
    }
    static constexpr int stores_in(int lo, int hi)   // store events at pairs lo < k < hi
    {
        int n = 0;
        for (int k = 0; k < SPO; k += G)
            if (k > lo && k < hi) ++n;
        return n;
    }
    // vector-memory instructions issued after dma(m) and before copy_seg(m):
    // only stores (one DMA segment is in flight at a time)
    static constexpr int vm_after(int m)
    {
        return m == 2 ? stores_in(kc(6), SPO) + stores_in(-1, kc(2)) : stores_in(kc(m - 1), kc(m));
    }
    static constexpr int prologue_pad() { return stores_in(kc(6), SPO); }
};

struct FastArgs {
    const float *in;                 // mix 0, track 0
    int64_t in_mix_stride;           // floats
    int64_t track_bytes;             // bytes between tracks of a mix (>= 8*N)
    float *out;
    int64_t out_mix_stride;          // floats
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

// coefficient bits as an integer (an "i" asm operand once k, t are unrolled)
__device__ __forceinline__ constexpr int hbits(int k, int t) { return __builtin_bit_cast(int, kH147[k][t]); }

#ifdef XM_FAST_ABLATION
// per-launch cycle attribution (ABL & 16): [0] wave cycles, [1] cycles in
// copy_seg's vmcnt waits, [2] waves, [3] cycles in the prologue
__device__ unsigned long long g_fast_prof[4];
#endif

// ABL: ablation bits for performance attribution (dev builds only, see
// `make ablate`; results are wrong by design): 1 no DMA/copies, 2 no taps,
// 4 no exchange/track sum (a checksum is stored instead), 8 constant gains,
// 16 cycle attribution into g_fast_prof (results stay exact).
template <int NT, bool ASM, int ABL = 0>
__global__ __launch_bounds__(64) void k_rs147_mix(FastArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char lds[];
    using SC = Sched<0>;
    constexpr int S = 64 / NT;                  // stream slots (SP runs) per track in a wave
    static_assert(S == 8, "DMA address split and exchange assume 8 tracks x 8 slots");
    const int lane = threadIdx.x;
    const int tr = lane / S, spl = lane % S;    // compute mapping: lane = tr*S + spl
    const int mix = blockIdx.x / a.tasks_per_mix;
    const int task = blockIdx.x % a.tasks_per_mix;
    const int s_first = (task * S + spl) * a.R;                 // this lane's first SP
    const char *slot = lds;
    f2 *X = (f2 *)(lds + SLOT_BYTES);
    const uint32_t ldsb = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void *)lds);

    // one resource per mix, shifted 32 frames back so offsets stay >= 0
    const float *mixbase = a.in + (int64_t)mix * a.in_mix_stride - 64;
    const uint64_t mb = (uint64_t)(uintptr_t)mixbase;
    i4 rs;
    rs.x = (int)__builtin_amdgcn_readfirstlane((uint32_t)mb);
    rs.y = (int)__builtin_amdgcn_readfirstlane((uint32_t)(mb >> 32) & 0xffffu);
    rs.z = (int)__builtin_amdgcn_readfirstlane(
        (uint32_t)((NT - 1) * a.track_bytes + ((int64_t)a.frames_in + 32) * 8));
    rs.w = 0x00020000;

    // ---- DMA addressing (loader role): instruction d covers streams
    // q = 4d..4d+3; lane l loads chunk j = ((l & 15) - q) & 15 of stream
    // q = 4d + (l >> 4), which the hardware lands at slot + d*1024 + l*16.
    // The byte offset splits into a wave-uniform part (soffset: track d/2,
    // slot group 4*(d&1), segment, SP) and one of 4 per-lane parts (the chunk
    // rotation depends on d only through d & 3).
    const int lq = lane >> 4;
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

    // segment m (0..6 relative to SP r) of every stream of the wave -> slot.
    // s_waitcnt lgkmcnt(0) first: the previous copy's ds_reads of the slot
    // must be done before the DMA can land on it.
    auto dma = [&](int r, int m) {
        if (ABL & 1) return;
        const uint32_t rb0 = (uint32_t)(r * (SPI * 8) + m * 256);
        const uint32_t rb1 = rb0 + GR;
        // streams touching the clip start or end in this SP need per-chunk redirects
        const bool edge = __builtin_amdgcn_ballot_w64(s_first + r == 0 || (s_first + r + 1) * SPI + 32 > N) != 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            uint32_t v = vl[d & 3];
            if (edge) {
                const int f = fl[d & 3] + 4 * (d & 1) * a.R * SPI + r * SPI + m * SEGF;
                v = (f >= 0 && f + 1 < N) ? v : OOB;   // out-of-clip chunk: zero-filled
            }
            uint32_t so;
            asm volatile("s_mul_i32 %0, %1, %2\n\t"
                         "s_add_u32 %0, %0, %3\n\t"
                         "s_add_u32 m0, %4, %5\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dwordx4 %6, %7, %0 offen lds"
                         : "=&s"(so)
                         : "s"(TB), "n"(d >> 1), "s"((d & 1) ? rb1 : rb0), "s"(ldsb), "n"(d * 1024), "v"(v), "s"(rs)
                         : "memory", "scc", "m0");
        }
    };
    // ---- register window: rel frames [0, 224) of the current SP, one array
    // per channel (kept scalar so nothing re-packs the VOP2 arithmetic)
    uint64_t t_wait = 0;
    const uint64_t t_begin = (ABL & 16) ? __builtin_amdgcn_s_memtime() : 0;
    float xl[WIN], xr[WIN];
    if (ABL & 1)
        for (int f = 0; f < WIN; ++f) xl[f] = xr[f] = (float)(lane + f);
    auto copy_seg = [&](int m, auto vm) {   // slot -> x[32m .. 32m+31] of this lane's stream
        if (ABL & 1) return;
        uint64_t tw0 = 0;
        if (ABL & 16) tw0 = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(vm)::value) : "memory");   // dma(m) landed
        if (ABL & 16) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            t_wait += __builtin_amdgcn_s_memtime() - tw0;
        }
        const char *base = slot + (lane >> 2) * 1024 + (lane & 3) * 256;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float4 v = *(const float4 *)(base + (((j + lane) & 15) * 16));
            xl[SEGF * m + 2 * j] = v.x;
            xr[SEGF * m + 2 * j] = v.y;
            xl[SEGF * m + 2 * j + 1] = v.z;
            xr[SEGF * m + 2 * j + 1] = v.w;
        }
    };

    // ---- gain ramp of this lane's track
    XmhGain gp = a.g[0];
#pragma unroll
    for (int i = 1; i < NT; ++i)
        if (tr == i) gp = a.g[i];
    const bool xf = (gp.flags & XMH_GAIN_XFADE_OUT) != 0;

    float *outb = a.out + (int64_t)mix * a.out_mix_stride;
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(outb, (uint32_t)a.frames_out * 8u);

    // ---- track-sum role: lane' = (slot spo, output kk of the round)
    const int spo = lane / G, kkp = lane % G;
    f2 pend[NT];
    f2 chk = f2{0.0f, 0.0f};
    auto sum_reads = [&]() {          // the previous round's exchange rows
        if (ABL & 4) return;
#pragma unroll
        for (int t2 = 0; t2 < NT; ++t2) pend[t2] = X[kkp * 64 + ((t2 * S + spo + 4 * kkp) & 63)];
    };
    auto sum_store = [&](int rp, int qp, bool valid) {
        if (ABL & 4) return;
        f2 sum = pend[0];
#pragma unroll
        for (int t2 = 1; t2 < NT; ++t2) sum = sum + pend[t2];
        sum = sum + f2{0.0f, 0.0f};              // -0 -> +0 (scipy seeds are +0)
        const int kq = qp * G + kkp;
        const int n = ((task * S + spo) * a.R + rp) * SPO + kq;   // >= frames_out: dropped by range check
        const uint32_t off = (valid && kq < SPO) ? (uint32_t)n * 8u : OOB;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, sum), ro, off, 0, 0);
    };

    // prologue: segments 0, 1 of the first SP in registers; segment 2 in
    // flight, followed by as many (dropped) stores as a steady-state SP issues
    // after its own dma(., 2), so copy_seg(2)'s vmcnt is exact from r = 0 on
    dma(0, 0);
    copy_seg(0, std::integral_constant<int, 0>{});
    dma(0, 1);
    copy_seg(1, std::integral_constant<int, 0>{});
    dma(0, 2);
#pragma unroll
    for (int i = 0; i < SC::prologue_pad(); ++i)
        __builtin_amdgcn_raw_buffer_store_b64(v2u{0u, 0u}, ro, OOB, 0, 0);

    const uint64_t t_pro = (ABL & 16) ? __builtin_amdgcn_s_memtime() - t_begin : 0;
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
            if (ABL & 8) {
            } else if (any_bnd) {
#pragma unroll
                for (int i = 0; i < G; ++i) gk[i] = gain_exact(gp, n_sp0 + k0 + i);
            } else if (any_lin) {
#pragma unroll
                for (int i = 0; i < G; ++i) gk[i] = cA + cB * (fkb + (float)(k0 + i));
            }
            sum_reads();   // previous round (round 18 of the previous SP when q == 0)
#pragma unroll
            for (int k = k0; k < kend; k += 2) {
                const bool two = k + 1 < kend;
                // 1. bring in the segments this pair's schedule copies
#pragma unroll
                for (int m = SC::have_before(k) + 1; m <= SC::needc(k); ++m) {
                    if (m == 2) copy_seg(2, std::integral_constant<int, SC::vm_after(2)>{});
                    if (m == 3) copy_seg(3, std::integral_constant<int, SC::vm_after(3)>{});
                    if (m == 4) copy_seg(4, std::integral_constant<int, SC::vm_after(4)>{});
                    if (m == 5) copy_seg(5, std::integral_constant<int, SC::vm_after(5)>{});
                    if (m == 6) copy_seg(6, std::integral_constant<int, SC::vm_after(6)>{});
                }
                // 2. outputs k, k+1: 22 taps each, literal coefficients, four
                // independent mul/add chains (L, R of two outputs)
                const int ra = rk(k), rb = rk(two ? k + 1 : k);
                float l0, r0, l1 = 0.0f, r1 = 0.0f;
                if (ASM) {
                    // one opaque block per tap: 4 products into 4 temps, then
                    // the 4 dependent adds (mul->add distance 4, see
                    // tools/ubench/dep_latency.hip); coefficient bits inline
                    if (two) {
                        asm("v_mul_f32 %0, %4, %6\n\tv_mul_f32 %1, %4, %7\n\t"
                            "v_mul_f32 %2, %5, %8\n\tv_mul_f32 %3, %5, %9"
                            : "=&v"(l0), "=&v"(r0), "=&v"(l1), "=&v"(r1)
                            : "i"(hbits(k, 0)), "i"(hbits(k + 1, 0)), "v"(xl[ra]), "v"(xr[ra]), "v"(xl[rb]), "v"(xr[rb]));
                    } else {
                        asm("v_mul_f32 %0, %2, %3\n\tv_mul_f32 %1, %2, %4"
                            : "=&v"(l0), "=&v"(r0) : "i"(hbits(k, 0)), "v"(xl[ra]), "v"(xr[ra]));
                    }
#pragma unroll
                    for (int t = 1; t < TE; ++t) {
                        float p0, p1, p2, p3;
                        if (two) {
                            asm("v_mul_f32 %0, %8, %10\n\tv_mul_f32 %1, %8, %11\n\t"
                                "v_mul_f32 %2, %9, %12\n\tv_mul_f32 %3, %9, %13\n\t"
                                "v_add_f32 %4, %4, %0\n\tv_add_f32 %5, %5, %1\n\t"
                                "v_add_f32 %6, %6, %2\n\tv_add_f32 %7, %7, %3"
                                : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(l0), "+v"(r0), "+v"(l1), "+v"(r1)
                                : "i"(hbits(k, t)), "i"(hbits(k + 1, t)), "v"(xl[ra + t]), "v"(xr[ra + t]),
                                  "v"(xl[rb + t]), "v"(xr[rb + t]));
                        } else {
                            asm("v_mul_f32 %0, %4, %5\n\tv_mul_f32 %1, %4, %6\n\t"
                                "v_add_f32 %2, %2, %0\n\tv_add_f32 %3, %3, %1"
                                : "=&v"(p0), "=&v"(p1), "+v"(l0), "+v"(r0)
                                : "i"(hbits(k, t)), "v"(xl[ra + t]), "v"(xr[ra + t]));
                        }
                    }
                } else if (ABL & 2) {
                    l0 = xl[ra];
                    r0 = xr[ra];
                    l1 = xl[rb];
                    r1 = xr[rb];
                } else {
                    l0 = xl[ra] * kH147[k][0];
                    r0 = xr[ra] * kH147[k][0];
                    if (two) {
                        l1 = xl[rb] * kH147[k + 1][0];
                        r1 = xr[rb] * kH147[k + 1][0];
                    }
#pragma unroll
                    for (int t = 1; t < TE; ++t) {
                        l0 = l0 + xl[ra + t] * kH147[k][t];
                        r0 = r0 + xr[ra + t] * kH147[k][t];
                        if (two) {
                            l1 = l1 + xl[rb + t] * kH147[k + 1][t];
                            r1 = r1 + xr[rb + t] * kH147[k + 1][t];
                        }
                    }
                }
                // 3. the previous round's track sum (its reads were issued
                // before this pair's compute, so their latency is hidden)
                if (k == k0) {
                    if (q == 0) sum_store(r - 1, ROUNDS - 1, r > 0);
                    else sum_store(r, q - 1, true);
                }
                // 4. refill the slot behind each copy made above
#pragma unroll
                for (int m = SC::have_before(k) + 1; m <= SC::needc(k); ++m) {
                    if (m < 6) dma(r, m + 1);
                    else if (r + 1 < a.R) dma(r + 1, 2);          // next SP's segment 2
                }
                // 5. exchange row kk: (track t, slot sp) at (t*S + sp + 4*kk) & 63
                const int kk0 = k - k0, kk1 = k + 1 - k0;
                if (ABL & 4) {
                    chk = chk + f2{l0, r0} * gk[kk0] + f2{l1, r1} * gk[kk1];
                    continue;
                }
                X[kk0 * 64 + ((lane + 4 * kk0) & 63)] = f2{l0, r0} * gk[kk0];
                if (two) X[kk1 * 64 + ((lane + 4 * kk1) & 63)] = f2{l1, r1} * gk[kk1];
            }
        }
        // carry: the next SP's rel frames [21, 64) are this SP's [181, 224)
#pragma unroll
        for (int f = CARRY0; f < 2 * SEGF; ++f) {
            xl[f] = xl[f + SPI];
            xr[f] = xr[f + SPI];
        }
    }
    if (ABL & 4) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, chk), ro, (uint32_t)lane * 8u, 0, 0);
    // last round of the last SP
    sum_reads();
    sum_store(a.R - 1, ROUNDS - 1, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the wave's LDS is gone
#ifdef XM_FAST_ABLATION
    if ((ABL & 16) && lane == 0) {
        atomicAdd(&g_fast_prof[0], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_begin));
        atomicAdd(&g_fast_prof[1], (unsigned long long)t_wait);
        atomicAdd(&g_fast_prof[2], 1ull);
        atomicAdd(&g_fast_prof[3], (unsigned long long)t_pro);
    }
#endif
}

}  // namespace

#ifdef XM_FAST_ABLATION
// dev builds: read and clear the cycle attribution counters
extern "C" __attribute__((visibility("default"))) int xm_dev_fast_prof(unsigned long long *out4)
{
    static const unsigned long long zero[4] = {0, 0, 0, 0};
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_fast_prof), sizeof zero) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_fast_prof), zero, sizeof zero) != hipSuccess)
        return -1001;
    return 0;
}
#endif

// The kernel's coefficients are compile-time literals: accept a runtime table
// only if it is bit-identical (both come from xm_resample_design; this guards
// against a stale build).  Tap 22 of every phase must be an exact zero.
extern "C" int xmh_fast_table_check(const float *H, int Lr, int Mr, int T)
{
    if (Lr != L || Mr != M || T != 23) return -1003;
    for (int ph = 0; ph < L; ++ph)
        if (__builtin_bit_cast(uint32_t, H[ph * T + 22]) != 0u) return -1003;
    for (int k = 0; k < SPO; ++k) {
        const int ph = ((k + RM) * M) % L;
        for (int t = 0; t < TE; ++t)
            if (__builtin_bit_cast(uint32_t, H[ph * T + t]) != __builtin_bit_cast(uint32_t, kH147[k][t]))
                return -1003;
    }
    return 0;
}

// SPs per lane and tasks per mix: every wave costs ~ (R + 1) SP-times (the +1
// is the prologue / first-SP overhead) and the grid runs in ceil(waves /
// slots) generations; pick the split with the least total.
static void pick_split(int64_t n_mix, int n_sp, int S, int *R_out, int *tpm_out)
{
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    const int64_t slots = (int64_t)cus * WAVES_PER_CU;
    const int max_tpm = (n_sp + S - 1) / S;
    int bestR = (n_sp + S - 1) / S, bestT = 1;
    double best = 1e300;
    for (int tpm = 1; tpm <= max_tpm && tpm <= 4096; ++tpm) {
        const int R = (n_sp + S * tpm - 1) / (S * tpm);
        if (tpm > 1 && (n_sp + S * R - 1) / (S * R) != tpm) continue;   // same R with fewer tasks exists
        const int64_t waves = n_mix * tpm;
        const double cost = (double)((waves + slots - 1) / slots) * (R + 1);
        if (cost < best) {
            best = cost;
            bestR = R;
            bestT = tpm;
        }
    }
    *R_out = bestR;
    *tpm_out = bestT;
}

extern "C" int xmh_launch_mix_fast(const XmhMixJob *j, void *stream, int *n_launches)
{
    const int NT = j->n_tracks;
    const int64_t N = j->frames_in;
    if (!(j->rs.L == L && j->rs.M == M && j->rs.rm == RM && j->rs.T == 23 && j->rs.fast) ||
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
    a.n_mix = j->n_mix;
    a.n_tracks = NT;
    a.frames_in = (int32_t)N;
    a.frames_out = (int32_t)j->frames_out;
    a.n_sp = (int32_t)((j->frames_out + SPO - 1) / SPO);
    const int S = 64 / NT;
    pick_split(a.n_mix, a.n_sp, S, &a.R, &a.tasks_per_mix);
    if (const char *fr = getenv("XM_FAST_R")) {   // dev knob: force SPs per lane
        const int R = atoi(fr);
        if (R >= 1) {
            a.R = R;
            a.tasks_per_mix = (a.n_sp + S * R - 1) / (S * R);
        }
    }
    a.unity = j->unity;
    for (int i = 0; i < NT; ++i) {
        a.g[i] = j->gains_host[i];
        const int64_t lim = (int64_t)1 << 28;   // outputs < 2^26: keeps clamp(n-start) unchanged
        a.g[i].start = a.g[i].start < -lim ? -lim : (a.g[i].start > lim ? lim : a.g[i].start);
    }
    const int64_t blocks = (int64_t)a.n_mix * a.tasks_per_mix;
    if (blocks > 0x7fffffff) return -1003;
    const char *ab = getenv("XM_FAST_TAPS");   // "c": compiler-scheduled taps (A/B only)
    const bool c_taps = ab && ab[0] == 'c';
    auto kern = c_taps ? k_rs147_mix<8, false> : k_rs147_mix<8, true>;
#ifdef XM_FAST_ABLATION
    const char *abl = getenv("XM_FAST_ABLATE");
    switch (abl ? atoi(abl) : 0) {
    case 1: kern = k_rs147_mix<8, false, 1>; break;
    case 2: kern = k_rs147_mix<8, false, 2>; break;
    case 4: kern = k_rs147_mix<8, false, 4>; break;
    case 8: kern = k_rs147_mix<8, false, 8>; break;
    case 5: kern = k_rs147_mix<8, false, 5>; break;
    case 6: kern = k_rs147_mix<8, false, 6>; break;
    case 12: kern = k_rs147_mix<8, false, 12>; break;
    case 13: kern = k_rs147_mix<8, false, 13>; break;
    case 16: kern = k_rs147_mix<8, false, 16>; break;
    case 17: kern = k_rs147_mix<8, false, 17>; break;
    case 18: kern = k_rs147_mix<8, false, 18>; break;
    case 24: kern = k_rs147_mix<8, false, 24>; break;
    default: break;
    }
#endif
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64), LDS_PER_WAVE, (hipStream_t)stream, a);
    if (n_launches) *n_launches += 1;
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}
