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
#include "xm_pk_taps.h"         // generated: packed-tap asm blocks (tools/gen_pk_asm.py)

// cache policy of the once-read input stream (XM_DMA_NT=0 at build: default policy)
#ifndef XM_DMA_NT_OFF
#define XM_DMA_NT " nt"
#else
#define XM_DMA_NT ""
#endif

// every packed-tap asm block starts 8-byte aligned, so no VOP3P instruction
// straddles an 8-byte boundary (MI355X_MICROARCH.md: hand-asm streams lose
// at 4-mod-8 placement; measured here -0.5 %)
#define XM_AL ".p2align 3\n\t"

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
constexpr int DMA_PARTS = 8;               // a segment's 16 DMA instructions, 2 per output pair

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
template <int E, int NSTORE = 1>   // NSTORE: vector stores per store event
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
    // DMA of segment m is spread over DMA_PARTS pairs (2 instructions each),
    // starting at the pair that copied segment m-1 (segment 2: at kc(6) of
    // the previous SP, wrapping into the next SP's first pairs)
    static constexpr int dma_start(int m) { return m == 2 ? kc(6) : kc(m - 1); }
    // pair (in the copying SP's coordinates) of segment m's last DMA part
    static constexpr int dma_last(int m) { return dma_start(m) + 2 * (DMA_PARTS - 1) - (m == 2 ? 2 * ((SPO + 1) / 2) : 0); }
    // part of segment m's DMA issued at pair k of an SP (-1: none); for m == 2
    // `next` selects the parts that belong to the following SP's segment 2
    static constexpr int part_at(int k, int m, bool next)
    {
        if (m != 2) {
            const int j = (k - dma_start(m)) / 2;
            return k >= dma_start(m) && j < DMA_PARTS ? j : -1;
        }
        if (next) return k >= dma_start(2) ? (k - dma_start(2)) / 2 : -1;
        const int j = (k + 2 * ((SPO + 1) / 2) - dma_start(2)) / 2;   // tail parts of this SP's own segment 2
        return j < DMA_PARTS ? j : -1;
    }
    // vector-memory instructions issued after segment m's last DMA part and
    // before copy_seg(m): only round stores (part windows never overlap)
    static constexpr int vm_after(int m) { return NSTORE * stores_in(dma_last(m), kc(m)); }
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
    int64_t out_clip_stride;         // SPLIT: floats between the 8 clips' outputs
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

// the same coefficients pair-interleaved for the packed taps (TAPS == 2):
// g_kHp[i][t] = (h_2i[t], h_2i+1[t]), read with scalar loads
typedef const f2 __attribute__((address_space(4))) cf2;
__constant__ float g_kHp[75][44] = XM_KHP147_INIT;   // + 1 zero row: prefetch past the end stays in bounds

// coefficient groups of the packed taps: pair i = outputs (2i, 2i+1), group
// g covers taps 8g .. min(8g+7, 21); 74 pairs x 3 groups per SP
constexpr int CG_TAPS = 8;
constexpr int CG_PER_PAIR = 3;
__host__ __device__ constexpr int cg_ntaps(int g) { return g < 2 ? CG_TAPS : TE - 2 * CG_TAPS; }

// coefficient bits as an integer (an "i" asm operand once k, t are unrolled)
__device__ __forceinline__ constexpr int hbits(int k, int t) { return __builtin_bit_cast(int, kH147[k][t]); }

#ifdef XM_FAST_ABLATION
// per-launch cycle attribution (ABL & 16): [0] wave cycles, [1] cycles in
// copy_seg's vmcnt waits, [2] waves, [3] cycles issuing DMA (incl. back-pressure),
// [4] cycles from copy issue to data in VGPRs, [5] cycles in the track-sum store step
__device__ unsigned long long g_fast_prof[8];
#endif

// ABL: ablation bits for performance attribution (dev builds only, see
// `make ablate`; results are wrong by design): 1 no DMA/copies, 2 no taps,
// 4 no exchange/track sum (a checksum is stored instead), 8 constant gains,
// 16 cycle attribution into g_fast_prof (results stay exact).
// TAPS: 0 compiler-scheduled VOP2 with literal coefficients, 1 the same as
// opaque asm blocks, 2 packed v_pk_mul/v_pk_add on (L, R) with the
// coefficient pair (h_k, h_k+1) in an SGPR pair selected by op_sel.
// SPLIT: resample only (config 2) — the 8 "tracks" are 8 independent clips
// at unity gain and each is stored to its own output instead of being summed
// (out = r + 0, the contract's 1-track mix).
template <int NT, int TAPS, int ABL = 0, bool SPLIT = false, int WPB = 1>
__global__ __launch_bounds__(64 * WPB) void k_rs147_mix(FastArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char lds_all[];
    // WPB > 1: WPB independent waves per workgroup, each with its own LDS
    // slice, kept in step by one s_barrier per super-period (shared
    // instruction-cache lines: the SP body is ~100 KB of code)
    const int wib = WPB > 1 ? (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
    char *lds = lds_all + wib * LDS_PER_WAVE;
    const int gw = (int)blockIdx.x * WPB + wib;
    using SC = Sched<0, SPLIT ? NT : 1>;
    static_assert(SC::vm_after(2) < 64 && SC::vm_after(3) < 64 && SC::vm_after(4) < 64 && SC::vm_after(5) < 64 &&
                      SC::vm_after(6) < 64, "vmcnt is 6 bits");
    static_assert(SC::dma_last(2) < SC::kc(2) && SC::dma_last(3) < SC::kc(3) && SC::dma_last(4) < SC::kc(4) &&
                      SC::dma_last(5) < SC::kc(5) && SC::dma_last(6) < SC::kc(6),
                  "a segment's DMA parts must all be issued before its copy");
    constexpr int S = 64 / NT;                  // stream slots (SP runs) per track in a wave
    static_assert(S == 8, "DMA address split and exchange assume 8 tracks x 8 slots");
    const int lane = threadIdx.x & 63;
    const int tr = lane / S, spl = lane % S;    // compute mapping: lane = tr*S + spl
    const int mix = gw / a.tasks_per_mix;
    const int task = gw % a.tasks_per_mix;
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

    // part j (instructions 2j, 2j+1) of segment m (0..6 relative to SP r) of
    // every stream of the wave -> slot.  Part 0 waits lgkmcnt(0) first: the
    // previous copy's ds_reads of the slot must be done before DMA lands on it.
    uint64_t t_wait = 0, t_issue = 0, t_copy = 0, t_sum = 0;
    auto dma_part = [&](int r, int m, int jp) {
        if (ABL & 1) return;
        uint64_t ti0 = 0;
        if (ABL & 16) ti0 = __builtin_amdgcn_s_memtime();
        const uint32_t rb0 = (uint32_t)(r * (SPI * 8) + m * 256);
        const uint32_t rb1 = rb0 + GR;
        // streams touching the clip start or end in this SP need per-chunk redirects
        const bool edge = __builtin_amdgcn_ballot_w64(s_first + r == 0 || (s_first + r + 1) * SPI + 32 > N) != 0;
        if (jp == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int d = 2 * jp; d < 2 * jp + 2; ++d) {
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
                         "buffer_load_dwordx4 %6, %7, %0 offen" XM_DMA_NT " lds"
                         : "=&s"(so)
                         : "s"(TB), "n"(d >> 1), "s"((d & 1) ? rb1 : rb0), "s"(ldsb), "n"(d * 1024), "v"(v), "s"(rs)
                         : "memory", "scc", "m0");
        }
        if (ABL & 16) t_issue += __builtin_amdgcn_s_memtime() - ti0;
    };
    auto dma = [&](int r, int m) {   // a whole segment at once (prologue)
#pragma unroll
        for (int jp = 0; jp < DMA_PARTS; ++jp) dma_part(r, m, jp);
    };
    // ---- register window: rel frames [0, 224) of the current SP, one array
    // per channel (kept scalar so nothing re-packs the VOP2 arithmetic)
    const uint64_t t_begin = (ABL & 16) ? __builtin_amdgcn_s_memtime() : 0;
    float xl[WIN], xr[WIN];   // TAPS 0/1
    f2 x2[WIN];               // TAPS 2: (L, R) in an aligned VGPR pair
    if (ABL & 1)
#pragma unroll
        for (int f = 0; f < WIN; ++f) {
            if (TAPS == 2) x2[f] = f2{(float)(lane + f), (float)(lane - f)};
            else xl[f] = xr[f] = (float)(lane + f);
        }
    float fake = 0.0f;   // ABL & 1: SP-dependent window contents, so nothing can be hoisted
    auto copy_seg = [&](int m, auto vm) {   // slot -> x[32m .. 32m+31] of this lane's stream
        if (ABL & 1) {
#pragma unroll
            for (int j = 0; j < SEGF; ++j) {
                if (TAPS == 2) {
                    x2[SEGF * m + j] = f2{fake + (float)j, fake - (float)j};
                } else {
                    xl[SEGF * m + j] = fake + (float)j;
                    xr[SEGF * m + j] = fake - (float)j;
                }
            }
            return;
        }
        uint64_t tw0 = 0;
        if (ABL & 16) tw0 = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(vm)::value) : "memory");   // dma(m) landed
        uint64_t tw1 = 0;
        if (ABL & 16) {
            tw1 = __builtin_amdgcn_s_memtime();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            t_wait += tw1 - tw0;
        }
        const char *base = slot + (lane >> 2) * 1024 + (lane & 3) * 256;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float4 v = *(const float4 *)(base + (((j + lane) & 15) * 16));
            if (TAPS == 2) {
                x2[SEGF * m + 2 * j] = f2{v.x, v.y};
                x2[SEGF * m + 2 * j + 1] = f2{v.z, v.w};
            } else {
                xl[SEGF * m + 2 * j] = v.x;
                xr[SEGF * m + 2 * j] = v.y;
                xl[SEGF * m + 2 * j + 1] = v.z;
                xr[SEGF * m + 2 * j + 1] = v.w;
            }
        }
        if (ABL & 16) {   // all 16 ds_read_b128 landed (serialises the copy: attribution only)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            t_copy += __builtin_amdgcn_s_memtime() - tw1;
        }
    };

    // ---- gain ramp of this lane's track
    XmhGain gp = a.g[0];
#pragma unroll
    for (int i = 1; i < NT; ++i)
        if (tr == i) gp = a.g[i];
    const bool xf = (gp.flags & XMH_GAIN_XFADE_OUT) != 0;

    float *outb = a.out + (int64_t)mix * a.out_mix_stride;
    const uint32_t clip_bytes = SPLIT ? (uint32_t)a.out_clip_stride * 4u : 0u;
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(outb, (NT - 1) * clip_bytes + (uint32_t)a.frames_out * 8u);

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
        uint64_t ts0 = 0;
        if (ABL & 16) ts0 = __builtin_amdgcn_s_memtime();
        const int kq = qp * G + kkp;
        const int n = ((task * S + spo) * a.R + rp) * SPO + kq;   // >= frames_out: dropped by range check
        if constexpr (SPLIT) {
            // one store per clip, every one issued (vmcnt accounting); n past
            // the clip end would land in the next clip: send it out of range
            const bool ok = valid && kq < SPO && n < a.frames_out;
#pragma unroll
            for (int t2 = 0; t2 < NT; ++t2) {
                const f2 v = pend[t2] + f2{0.0f, 0.0f};   // -0 -> +0 (scipy seeds are +0)
                const uint32_t off = ok ? (uint32_t)t2 * clip_bytes + (uint32_t)n * 8u : OOB;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), ro, off, 0, 0);
            }
        } else {
            f2 sum = pend[0];
#pragma unroll
            for (int t2 = 1; t2 < NT; ++t2) sum = sum + pend[t2];
            sum = sum + f2{0.0f, 0.0f};              // -0 -> +0 (scipy seeds are +0)
            const uint32_t off = (valid && kq < SPO) ? (uint32_t)n * 8u : OOB;
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, sum), ro, off, 0, 0);
        }
        if (ABL & 16) t_sum += __builtin_amdgcn_s_memtime() - ts0;
    };

    // ---- packed taps: the coefficient group in flight, one s_load_dwordx16
    // (8 SGPR pairs (h_k[t], h_k+1[t])) per 8-tap group, double-buffered by
    // group parity.  The loads are asm the compiler cannot see as pending, so
    // every consumer sits behind an explicit lgkmcnt(0) (volatile asm keeps
    // program order).  One dwordx16 instead of eight dwordx2: -4.5 % time.
    const uint64_t hp_base = (uint64_t)(uintptr_t)&g_kHp[0][0];
    typedef float f16v __attribute__((ext_vector_type(16)));
    f16v cgb[2];   // double buffer by group parity (222 groups per SP: the parity pattern repeats)
    auto cg_load16 = [&](int buf, int pi, int g) {
        const uint32_t off = (uint32_t)(pi * 44 + g * 2 * CG_TAPS) * 4u;
        asm volatile("s_load_dwordx16 %0, %1, %2" : "=s"(cgb[buf]) : "s"(hp_base), "s"(off) : "memory");
    };

    // prologue: segments 0, 1 of the first SP in registers; segment 2 in
    // flight, followed by as many (dropped) stores as a steady-state SP issues
    // after its own dma(., 2), so copy_seg(2)'s vmcnt is exact from r = 0 on
    dma(0, 0);
    copy_seg(0, std::integral_constant<int, 0>{});
    dma(0, 1);
    copy_seg(1, std::integral_constant<int, 0>{});
    // segment 2's parts a previous SP would have issued; the first SP's own
    // pairs issue the rest, so every copy_seg's vmcnt count is the steady one
#pragma unroll
    for (int jp = 0; jp < DMA_PARTS; ++jp)
        if (SC::part_at(SC::dma_start(2) + 2 * jp, 2, true) == jp && SC::dma_start(2) + 2 * jp < SPO) dma_part(0, 2, jp);

#pragma unroll 1
    for (int r = 0; r < a.R; ++r) {
        const int s = s_first + r;
        if (ABL & 1) fake = (float)(s * 3 + lane);
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
        if (TAPS == 2) cg_load16(0, 0, 0);
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
                for (int i = 0; i < G; i += 2) {   // (k, k+1) as one packed pair: same ops, same rounding
                    const f2 kf = f2{fkb, fkb} + f2{(float)(k0 + i), (float)(k0 + i + 1)};
                    const f2 g2 = f2{cA, cA} + f2{cB, cB} * kf;
                    gk[i] = g2.x;
                    gk[i + 1] = g2.y;
                }
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
                if (TAPS == 2 && !(ABL & 2)) {
                    // (L, R) of outputs k and k+1; c = (h_k[t], h_k+1[t]) in
                    // an SGPR pair: op_sel picks h_k for both halves of the
                    // first product, h_k+1 for the second.  Per tap 2 pk_mul
                    // + 2 pk_add instead of 4 + 4 VOP2.  Coefficients arrive
                    // by explicit s_load one 8-tap group ahead (cg_load).
                    const int pi = k >> 1;
                    f2 a0, a1 = f2{0.0f, 0.0f};
#define XM_X2(t) "v"(x2[ra + (t)]), "v"(x2[rb + (t)])
#define XM_X1(t) "v"(x2[ra + (t)])
#define XM_SP(i) "s"(__builtin_shufflevector(cv, cv, 2 * (i), 2 * (i) + 1))
#define XM_CUR XM_SP(0), XM_SP(1), XM_SP(2), XM_SP(3), XM_SP(4), XM_SP(5), XM_SP(6), XM_SP(7)
#pragma unroll
                    for (int g = 0; g < CG_PER_PAIR; ++g) {
                        // wait for this group, then prefetch the next one
                        // (the next pair's first group; none past pair 73)
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        const int gi = 3 * pi + g;
                        const f16v cv = cgb[gi & 1];
                        if (g + 1 < CG_PER_PAIR) cg_load16((gi + 1) & 1, pi, g + 1);
                        else if (pi + 1 < 74) cg_load16((gi + 1) & 1, pi + 1, 0);
                        f2 p0, p1, p2, p3;
                        const int b = g * CG_TAPS;
                        if (two && g == 0)
                            asm volatile(XM_AL XM_PK_G0_TWO
                                         : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "=&v"(a0), "=&v"(a1)
                                         : XM_CUR, XM_X2(0), XM_X2(1), XM_X2(2), XM_X2(3), XM_X2(4), XM_X2(5),
                                           XM_X2(6), XM_X2(7));
                        else if (two && g == 1)
                            asm volatile(XM_AL XM_PK_G1_TWO
                                         : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                         : XM_CUR, XM_X2(b + 0), XM_X2(b + 1), XM_X2(b + 2), XM_X2(b + 3),
                                           XM_X2(b + 4), XM_X2(b + 5), XM_X2(b + 6), XM_X2(b + 7));
                        else if (two)
                            asm volatile(XM_AL XM_PK_G2_TWO
                                         : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                         : XM_CUR, XM_X2(b + 0), XM_X2(b + 1), XM_X2(b + 2), XM_X2(b + 3),
                                           XM_X2(b + 4), XM_X2(b + 5));
                        else if (g == 0)
                            asm volatile(XM_AL XM_PK_G0_ONE
                                         : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "=&v"(a0), "=&v"(a1)
                                         : XM_CUR, XM_X1(0), XM_X1(1), XM_X1(2), XM_X1(3), XM_X1(4), XM_X1(5),
                                           XM_X1(6), XM_X1(7));
                        else if (g == 1)
                            asm volatile(XM_AL XM_PK_G1_ONE
                                         : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                         : XM_CUR, XM_X1(b + 0), XM_X1(b + 1), XM_X1(b + 2), XM_X1(b + 3),
                                           XM_X1(b + 4), XM_X1(b + 5), XM_X1(b + 6), XM_X1(b + 7));
                        else
                            asm volatile(XM_AL XM_PK_G2_ONE
                                         : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "+v"(a0), "+v"(a1)
                                         : XM_CUR, XM_X1(b + 0), XM_X1(b + 1), XM_X1(b + 2), XM_X1(b + 3),
                                           XM_X1(b + 4), XM_X1(b + 5));
                    }
#undef XM_X2
#undef XM_X1
#undef XM_CUR
#undef XM_SP
                    l0 = a0.x;
                    r0 = a0.y;
                    l1 = a1.x;
                    r1 = a1.y;
                } else if (TAPS == 2) {   // ABL & 2
                    l0 = x2[ra].x;
                    r0 = x2[ra].y;
                    l1 = x2[rb].x;
                    r1 = x2[rb].y;
                } else if (TAPS == 1) {
                    // VOP2 with literal coefficients, 4 taps per opaque block
                    // (tools/gen_pk_asm.py): products of tap t+1 issue before
                    // the adds of tap t; adds stay in tap order.
#define XM_T2(t) "i"(hbits(k, t)), "i"(hbits(k + 1, t)), "v"(xl[ra + (t)]), "v"(xr[ra + (t)]), "v"(xl[rb + (t)]), "v"(xr[rb + (t)])
#define XM_T1(t) "i"(hbits(k, t)), "v"(xl[ra + (t)]), "v"(xr[ra + (t)])
                    float q0, q1, q2, q3, q4, q5, q6, q7;
                    if (two) {
                        asm volatile(XM_V2_F4_TWO
                                     : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "=&v"(q4), "=&v"(q5), "=&v"(q6),
                                       "=&v"(q7), "=&v"(l0), "=&v"(r0), "=&v"(l1), "=&v"(r1)
                                     : XM_T2(0), XM_T2(1), XM_T2(2), XM_T2(3));
#pragma unroll
                        for (int b = 4; b < 20; b += 4)
                            asm volatile(XM_V2_R4_TWO
                                         : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "=&v"(q4), "=&v"(q5), "=&v"(q6),
                                           "=&v"(q7), "+v"(l0), "+v"(r0), "+v"(l1), "+v"(r1)
                                         : XM_T2(b), XM_T2(b + 1), XM_T2(b + 2), XM_T2(b + 3));
                        asm volatile(XM_V2_R2_TWO
                                     : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "=&v"(q4), "=&v"(q5), "=&v"(q6),
                                       "=&v"(q7), "+v"(l0), "+v"(r0), "+v"(l1), "+v"(r1)
                                     : XM_T2(20), XM_T2(21));
                    } else {
                        asm volatile(XM_V2_F4_ONE
                                     : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "=&v"(l0), "=&v"(r0)
                                     : XM_T1(0), XM_T1(1), XM_T1(2), XM_T1(3));
#pragma unroll
                        for (int b = 4; b < 20; b += 4)
                            asm volatile(XM_V2_R4_ONE
                                         : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "+v"(l0), "+v"(r0)
                                         : XM_T1(b), XM_T1(b + 1), XM_T1(b + 2), XM_T1(b + 3));
                        asm volatile(XM_V2_R2_ONE
                                     : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "+v"(l0), "+v"(r0)
                                     : XM_T1(20), XM_T1(21));
                    }
#undef XM_T2
#undef XM_T1
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
                // 4. refill the slot, 2 DMA instructions per pair: segments
                // 3..6 of this SP, the tail of this SP's segment 2, and the
                // head of the next SP's segment 2
#pragma unroll
                for (int m = 3; m <= 6; ++m)
                    if (SC::part_at(k, m, false) >= 0) dma_part(r, m, SC::part_at(k, m, false));
                if (SC::part_at(k, 2, false) >= 0) dma_part(r, 2, SC::part_at(k, 2, false));
                if (SC::part_at(k, 2, true) >= 0 && r + 1 < a.R) dma_part(r + 1, 2, SC::part_at(k, 2, true));
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
            if (TAPS == 2) {
                x2[f] = x2[f + SPI];
            } else {
                xl[f] = xl[f + SPI];
                xr[f] = xr[f + SPI];
            }
        }
        // (measured alternatives, both slower: a barrier every exchange round;
        // waves 4..7 staggered half an SP behind their SIMD partners)
        if constexpr (WPB > 1) asm volatile("s_barrier" ::: "memory");
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
        atomicAdd(&g_fast_prof[3], (unsigned long long)t_issue);
        atomicAdd(&g_fast_prof[4], (unsigned long long)t_copy);
        atomicAdd(&g_fast_prof[5], (unsigned long long)t_sum);
    }
#endif
}

}  // namespace

#ifdef XM_FAST_ABLATION
// dev builds: read and clear the cycle attribution counters
extern "C" __attribute__((visibility("default"))) int xm_dev_fast_prof(unsigned long long *out8)
{
    static const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_fast_prof), sizeof zero) != hipSuccess ||
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

extern "C" int xmh_launch_mix_generic(const XmhMixJob *j, void *stream, int *n_launches);

extern "C" int xmh_launch_mix_fast(const XmhMixJob *j, void *stream, int *n_launches)
{
    const int NT = j->n_tracks;
    const int64_t N = j->frames_in;
    if (!(j->rs.L == L && j->rs.M == M && j->rs.rm == RM && j->rs.T == 23 && j->rs.fast) || j->in_base ||
        j->out_base || j->out_conv ||
        j->fmt != 2 || j->channels != 2 || j->in_ptrs || j->out_ptrs || !j->gains_host ||
        N <= 0 || (N & 1) || N >= (1 << 26) || j->n_mix <= 0)
        return -1003;   // not this kernel's job: generic path
    // 8-track mixes, or (split) 1-track unity-gain resampling of >= 8 clips,
    // taken 8 clips at a time as the 8 "tracks" of a pseudo-mix
    const bool split = NT == 1 && j->unity && j->n_mix >= 8;
    if (NT != 8 && !split) return -1003;
    const int64_t tb = split ? j->in_mix_stride * 4 : j->in_track_stride * 4;
    const int64_t in_mix = split ? 8 * j->in_mix_stride : j->in_mix_stride;
    if (tb < N * 8 || (tb & 15) || ((uintptr_t)j->in & 15) || ((in_mix * 4) & 15) ||
        7 * tb + (N + 32) * 8 >= ((int64_t)1 << 31))
        return -1003;
    if (split && (j->out_mix_stride < j->frames_out * 2 || 7 * j->out_mix_stride * 4 + j->frames_out * 8 >= ((int64_t)1 << 31)))
        return -1003;
    FastArgs a;
    memset(&a, 0, sizeof a);
    a.in = (const float *)j->in;
    a.in_mix_stride = in_mix;
    a.track_bytes = tb;
    a.out = (float *)j->out;
    a.out_mix_stride = split ? 8 * j->out_mix_stride : j->out_mix_stride;
    a.out_clip_stride = split ? j->out_mix_stride : 0;
    a.n_mix = split ? j->n_mix / 8 : j->n_mix;
    a.n_tracks = 8;
    a.frames_in = (int32_t)N;
    a.frames_out = (int32_t)j->frames_out;
    a.n_sp = (int32_t)((j->frames_out + SPO - 1) / SPO);
    const int S = 64 / 8;
    pick_split(a.n_mix, a.n_sp, S, &a.R, &a.tasks_per_mix);
    if (const char *fr = getenv("XM_FAST_R")) {   // dev knob: force SPs per lane
        const int R = atoi(fr);
        if (R >= 1) {
            a.R = R;
            a.tasks_per_mix = (a.n_sp + S * R - 1) / (S * R);
        }
    }
    a.unity = j->unity;
    for (int i = 0; i < 8; ++i) {
        if (split) {
            memset(&a.g[i], 0, sizeof a.g[i]);
            a.g[i].g0 = a.g[i].g1 = 1.0f;
            continue;
        }
        a.g[i] = j->gains_host[i];
        const int64_t lim = (int64_t)1 << 28;   // outputs < 2^26: keeps clamp(n-start) unchanged
        a.g[i].start = a.g[i].start < -lim ? -lim : (a.g[i].start > lim ? lim : a.g[i].start);
    }
    const int64_t blocks = (int64_t)a.n_mix * a.tasks_per_mix;
    if (blocks > 0x7fffffff) return -1003;
    // XM_FAST_TAPS (A/B only): "c" compiler-scheduled VOP2, "a" asm VOP2, default packed
    const char *ab = getenv("XM_FAST_TAPS");
    auto kern = k_rs147_mix<8, 2>;
    if (ab && ab[0] == 'c') kern = k_rs147_mix<8, 0>;
    if (ab && ab[0] == 'a') kern = k_rs147_mix<8, 1>;
#ifdef XM_FAST_ABLATION
    const char *abl = getenv("XM_FAST_ABLATE");
    const int tm = ab && ab[0] == 'c' ? 0 : (ab && ab[0] == 'a' ? 1 : 2);
#define XM_ABL_CASE(n) \
    case n: kern = tm == 0 ? k_rs147_mix<8, 0, n> : (tm == 1 ? k_rs147_mix<8, 1, n> : k_rs147_mix<8, 2, n>); break;
    switch (abl ? atoi(abl) : 0) {
    XM_ABL_CASE(1) XM_ABL_CASE(2) XM_ABL_CASE(16) XM_ABL_CASE(17) XM_ABL_CASE(18)
    default: break;
    }
#undef XM_ABL_CASE
#endif
    if (split) kern = k_rs147_mix<8, 2, 0, true>;
    // 8 waves per workgroup kept in step by one barrier per SP: measured -7 %
    // (4.52 -> 4.21 ms at the headline).  XM_FAST_WPB=1 (dev A/B) and the
    // tap-form / ablation variants run one wave per workgroup.
    int wpb = blocks % 8 == 0 ? 8 : 1;
    if (const char *w = getenv("XM_FAST_WPB")) wpb = (atoi(w) == 1 || (atoi(w) == 4 && blocks % 4 == 0)) ? atoi(w) : wpb;
    if (ab) wpb = 1;
#ifdef XM_FAST_ABLATION
    if (getenv("XM_FAST_ABLATE")) wpb = 1;
#endif
    if (wpb == 4 && !split) {   // dev A/B only
        kern = k_rs147_mix<8, 2, 0, false, 4>;
        if (hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * LDS_PER_WAVE) !=
            hipSuccess)
            return -1001;
        hipLaunchKernelGGL(kern, dim3((unsigned)(blocks / 4)), dim3(256), 4 * LDS_PER_WAVE, (hipStream_t)stream, a);
    } else if (wpb == 8) {
        kern = split ? k_rs147_mix<8, 2, 0, true, 8> : k_rs147_mix<8, 2, 0, false, 8>;
        if (hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * LDS_PER_WAVE) !=
            hipSuccess)
            return -1001;
        hipLaunchKernelGGL(kern, dim3((unsigned)(blocks / 8)), dim3(512), 8 * LDS_PER_WAVE, (hipStream_t)stream, a);
    } else {
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64), LDS_PER_WAVE, (hipStream_t)stream, a);
    }
    if (n_launches) *n_launches += 1;
    if (hipGetLastError() != hipSuccess) return -1001;
    if (split && j->n_mix % 8) {   // the last n_mix % 8 clips: generic kernel
        XmhMixJob r = *j;
        const int64_t done = (int64_t)a.n_mix * 8;
        r.n_mix = (int32_t)(j->n_mix - done);
        r.in = (const float *)j->in + done * j->in_mix_stride;
        r.out = (float *)j->out + done * j->out_mix_stride;
        return xmh_launch_mix_generic(&r, stream, n_launches);
    }
    return 0;
}
