// xm_fx.hip — effects chain kernels for gfx950 (biquad cascade, FIR) and the
// synthetic PCM generator.
//
// Biquad: scipy sosfilt order (transposed DF-II, _signaltools.py:4601),
// sections in order, state zero at clip start.  The recurrence is serial in
// time, so exactness (SURVEY.md §7 hard part 3) limits the parallelism to
// clips x sections x channels: k_biquad_pc (cascades of up to 16 sections)
// gives each (clip, section, channel) its own lane on a chain wave that forms
// its feed-forward products itself, k_biquad_pipe (longer cascades) each
// (clip, section) with stereo packed; both chain the sections through LDS (see
// the comments at the kernels).  Earlier designs (k_biquad_lane, the LDS-tap
// FIR k_fir, round 3's producer wave) and their dev switches left the product
// in round 4; git history keeps them.
// FIR: upfirdn order (_upfirdn.py:107), register-blocked over an LDS tile.
#include <stdlib.h>
#include <algorithm>
#include "xm_device.h"

// The LDS-DMA asm blocks set M0 themselves and list it as clobbered; clang
// warns because M0 is reserved.  Nothing else in these kernels uses M0 (no
// indirect register indexing, no ds_*_addtid / GWS: checked in the ISA).
#pragma clang diagnostic ignored "-Winline-asm"

namespace {

constexpr int BQ_MAXSEC = 64;   // XM_MAX_SOS (src/xm_internal.h): a cascade fills at most one wave of lanes

// Section-pipelined cascade.  The recurrence of one section is serial in
// time, so the only parallelism that keeps sosfilt's rounding is across
// clips and across sections: lane = (clip k, section s), lane = k*NS + s,
// KPW = min(64 / NS, 16) clips per workgroup (stereo (L, R) ride in one
// packed v_pk_* pair).  Time advances in chunks of BQ_G = 64 granules (16 B
// each: FPL = 4 / C frames); at step i lane s filters chunk i - s, so the NS
// sections of a clip work on NS consecutive chunks at once and the
// per-sample recurrence is the only serial chain.
//
// Two waves per workgroup.  The compute wave runs only the recurrences:
// section 0 reads granule g of its input at inb[i & 1][k][g], section s > 0
// at sec[L - 1][g] (the previous section's output row), the last section
// writes outb[i & 1][k][g], the others sec[L][g].  A lane reads granule g
// (two granules ahead of its use) before its left neighbour overwrites it
// with the next chunk: one wave, program order.  The copy wave does every
// HBM access: per step, chunk i + 1 of each clip by one LDS-DMA instruction
// (global_load_lds_dwordx4: 64 lanes x 16 B = the clip's whole 1 KB chunk,
// a wave-uniform base, landing straight in its inb row) and the stores of
// the chunk the last sections finished one step earlier (outb[(i - 1) & 1]);
// it waits for its DMA and meets the compute wave at one s_barrier per step.
// Rows are padded by one granule, so a wave's 64 row accesses of one granule
// are bank-conflict free.  The DMA is issued from inline asm (the compiler
// would otherwise put a vmcnt(0) before every LDS read); a partial last
// chunk is loaded and stored element by element, with bounds.
//
// Measured on MI355X, config-4 biquad stage (1024 stereo clips x 441000
// frames x 5 sections, tools/dev/bq_load.py): 22.3 ms for the previous
// design (32-granule chunks, per-item exec-masked loads, register staging,
// scattered 16-B items); 16.0 ms with one wave doing both jobs; 14.1 ms with
// the copy wave.  The compute wave spends ~58 cycles per frame (9 packed
// VALU ops + 1 LDS access per frame; tools/ubench/bq_chain.hip: ~51 cycles
// for the bare recurrence with its LDS traffic), against a floor of
// 36 cycles for 9 wave64 VALU issues.
template <int C>
struct BqVec;
template <>
struct BqVec<1> { typedef float T; };
template <>
struct BqVec<2> { typedef float T __attribute__((ext_vector_type(2))); };
typedef float bq_f4 __attribute__((ext_vector_type(4)));
typedef float bq_f2 __attribute__((ext_vector_type(2)));
// 4-B aligned 16-B vector: clip bases are only float-aligned
typedef float bq_f4u __attribute__((ext_vector_type(4), aligned(4)));

// One stereo granule (two frames A, B) of one section, hand-scheduled: the
// per-frame chain z0 -> o -> a1*o -> u -> z0 is four dependent packed ops,
// and every one of them has an independent op between it and its producer,
// so a lone wave never stalls on the VALU forwarding latency and needs no
// s_nop (the compiler's order put each product right before its consumer).
// Same operations as the scalar form in k_biquad_pipe, bit for bit:
// o = b0*v + z0, z0 = (b1*v - a1*o) + z1, z1 = b2*v - a2*o, with -(a*o) as a
// negated product and the adds commuted (IEEE add is commutative).
__device__ __forceinline__ bq_f4 bq_step2(bq_f4 v4, bq_f2 &z0, bq_f2 &z1, bq_f2 b0, bq_f2 b1, bq_f2 b2,
                                          bq_f2 a1, bq_f2 a2)
{
    const bq_f2 va = {v4[0], v4[1]}, vb = {v4[2], v4[3]};
    bq_f2 oa, ob, p0, p1, p2, t, u;
    asm volatile(
        "v_pk_mul_f32 %[p0], %[b0], %[va]\n\t"
        "v_pk_mul_f32 %[p1], %[b1], %[va]\n\t"
        "v_pk_add_f32 %[oa], %[z0], %[p0]\n\t"
        "v_pk_mul_f32 %[p2], %[b2], %[va]\n\t"
        "v_pk_mul_f32 %[t], %[a1], %[oa] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[p0], %[b0], %[vb]\n\t"
        "v_pk_add_f32 %[t], %[p1], %[t]\n\t"
        "v_pk_mul_f32 %[u], %[a2], %[oa] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %[z0], %[z1], %[t]\n\t"
        "v_pk_add_f32 %[z1], %[p2], %[u]\n\t"
        "v_pk_add_f32 %[ob], %[z0], %[p0]\n\t"
        "v_pk_mul_f32 %[p1], %[b1], %[vb]\n\t"
        "v_pk_mul_f32 %[t], %[a1], %[ob] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[p2], %[b2], %[vb]\n\t"
        "v_pk_add_f32 %[t], %[p1], %[t]\n\t"
        "v_pk_mul_f32 %[u], %[a2], %[ob] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %[z0], %[z1], %[t]\n\t"
        "v_pk_add_f32 %[z1], %[p2], %[u]"
        : [oa] "=&v"(oa), [ob] "=&v"(ob), [p0] "=&v"(p0), [p1] "=&v"(p1), [p2] "=&v"(p2), [t] "=&v"(t),
          [u] "=&v"(u), [z0] "+v"(z0), [z1] "+v"(z1)
        : [va] "v"(va), [vb] "v"(vb), [b0] "v"(b0), [b1] "v"(b1), [b2] "v"(b2), [a1] "v"(a1), [a2] "v"(a2));
    return bq_f4{oa.x, oa.y, ob.x, ob.y};
}

constexpr int BQ_G = 64;     // granules per chunk = lanes per DMA instruction
constexpr int BQ_KPW = 16;   // clips per wave at most (16 DMA + 16 stores per step)
constexpr int BQ_RP = 80;    // granules per input / output row: 65 + up to 15 of bank skew
constexpr size_t BQ_LDS = ((size_t)4 * BQ_KPW * BQ_RP + 64 * (BQ_G + 1)) * 16;   // 148,480 B


// The copy wave shared by both biquad kernels: every HBM access of the
// workgroup.  inb_row(p, k) / outb_row(p, k) give the LDS granule (16 B) where
// clip k's input / output chunk of parity p starts; chunks are 1 KB (64
// granules) of interleaved PCM, CH frames.
template <int C, class InRow, class OutRow>
__device__ __forceinline__ void bq_copy_wave(const XmhFxJob &j, int clip0, int nclip, int64_t steps, int ns,
                                             InRow inb_row, OutRow outb_row)
{
    typedef const __attribute__((address_space(1))) float gcf;
    typedef __attribute__((address_space(1))) float gf;
    typedef __attribute__((address_space(1))) bq_f4u gf4u;
    typedef __attribute__((address_space(3))) void lds_void;
    extern __shared__ bq_f4 bq_lds[];
    constexpr int FPL = 4 / C;                     // frames per 16-B granule
    constexpr int CH = BQ_G * FPL;                 // frames per chunk
    const int lane = threadIdx.x & 63;
    const int64_t N = j.frames;
    const int64_t nchunk = (N + CH - 1) / CH;
    const int64_t nfull = N / CH;                  // chunks with no frame past N
    {
        // The clip bases.  Lane k < nclip holds clip k's pointers; when the
        // clips lie within 4 GB of the lowest one (one tensor, or any compact
        // table) every access is a wave-uniform base (SGPR: the lowest pointer
        // + the chunk offset) plus a 32-bit per-lane offset precomputed per
        // clip.  Otherwise each access broadcasts its clip's 64-bit pointer.
        const int kl = min(lane, nclip - 1);
        const uint64_t xl = (uint64_t)(uintptr_t)j.in_ptrs[clip0 + kl];
        const uint64_t yl = (uint64_t)(uintptr_t)j.out_ptrs[clip0 + kl];
        auto bcast = [&](uint64_t v, int k) __attribute__((always_inline)) {
            // (readlane returns int: cast through uint32_t, no sign extension)
            return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), k) << 32) |
                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, k);
        };
        uint64_t xmin = bcast(xl, 0), xmax = xmin, ymin = bcast(yl, 0), ymax = ymin;
#pragma unroll
        for (int k = 1; k < BQ_KPW; ++k) {
            const uint64_t xk = bcast(xl, k), yk = bcast(yl, k);
            xmin = xk < xmin ? xk : xmin; xmax = xk > xmax ? xk : xmax;
            ymin = yk < ymin ? yk : ymin; ymax = yk > ymax ? yk : ymax;
        }
        const bool narrow = xmax - xmin < (1ull << 32) - 1024 && ymax - ymin < (1ull << 32) - 1024;
        uint32_t dx[BQ_KPW], dy[BQ_KPW];          // per clip: offset from the base + this lane's granule
#pragma unroll
        for (int k = 0; k < BQ_KPW; ++k) {
            dx[k] = (uint32_t)(bcast(xl, k) - xmin) + (uint32_t)lane * 16u;
            dy[k] = (uint32_t)(bcast(yl, k) - ymin) + (uint32_t)lane * 16u;
        }
        const uint32_t loff = (uint32_t)lane * 16u;
        const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void *)bq_lds);

        // input chunk c of every clip -> inb[c & 1]: one LDS-DMA instruction per
        // clip (64 lanes x 16 B = the clip's whole chunk, straight into its row)
        auto load_chunk = [&](int64_t c) __attribute__((always_inline)) {
            if (c >= nchunk) return;
            const int par = (int)(c & 1);
            if (c < nfull) {
                const uint64_t cbb = (uint64_t)c * CH * C * 4;
                if (narrow) {
#pragma unroll
                    for (int k = 0; k < BQ_KPW; ++k) {
                        if (k >= nclip) break;     // wave-uniform
                        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                                     :
                                     : "s"(lds0 + (uint32_t)inb_row(par, k) * 16u), "v"(dx[k]), "s"(xmin + cbb)
                                     : "memory", "m0");
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < BQ_KPW; ++k) {
                        if (k >= nclip) break;
                        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                                     :
                                     : "s"(lds0 + (uint32_t)inb_row(par, k) * 16u), "v"(loff), "s"(bcast(xl, k) + cbb)
                                     : "memory", "m0");
                    }
                }
                return;
            }
            // partial last chunk: element loads with bounds, zero past N
            const int64_t f0 = c * CH + lane * FPL;
#pragma unroll
            for (int k = 0; k < BQ_KPW; ++k) {
                if (k >= nclip) break;
                const float *x = (const float *)(uintptr_t)bcast(xl, k) + (size_t)f0 * C;
                bq_f4 v = bq_f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (f0 * C + e < N * C) v[e] = ((gcf *)x)[e];
                bq_lds[inb_row(par, k) + lane] = v;
            }
        };
        // the last sections' chunk c (in outb[p]) -> HBM
        auto store_chunk = [&](int64_t c, int p) __attribute__((always_inline)) {
            if (c < 0 || c >= nchunk) return;
            bq_f4 sv[BQ_KPW];
#pragma unroll
            for (int k = 0; k < BQ_KPW; ++k) sv[k] = bq_lds[outb_row(p, min(k, nclip - 1)) + lane];
            if (c < nfull) {
                const uint64_t cbb = (uint64_t)c * CH * C * 4;
#pragma unroll
                for (int k = 0; k < BQ_KPW; ++k) {
                    if (k >= nclip) break;
                    if (narrow) *(gf4u *)((char *)(uintptr_t)(ymin + cbb) + dy[k]) = sv[k];
                    else *(gf4u *)((char *)(uintptr_t)(bcast(yl, k) + cbb) + loff) = sv[k];
                }
                return;
            }
            const int64_t f0 = c * CH + lane * FPL;
#pragma unroll
            for (int k = 0; k < BQ_KPW; ++k) {
                if (k >= nclip) break;
                float *y = (float *)(uintptr_t)bcast(yl, k) + (size_t)f0 * C;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (f0 * C + e < N * C) ((gf *)y)[e] = sv[k][e];
            }
        };

        load_chunk(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int64_t i = 0; i < steps; ++i) {
            // the compute wave filters step i meanwhile
            load_chunk(i + 1);
            store_chunk(i - ns, (int)((i - 1) & 1));   // finished in step i - 1
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // chunk i + 1 landed
            __syncthreads();
        }
        store_chunk(steps - ns, (int)((steps - 1) & 1));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may land after the LDS is gone
    }
}

template <int C, bool ST>
__global__ __launch_bounds__(128) void k_biquad_pipe(XmhFxJob j)
{
    typedef typename BqVec<C>::T V;
    constexpr int G = BQ_G;
    constexpr int FPL = 4 / C;                     // frames per 16-B granule
    constexpr int CH = G * FPL;                    // frames per chunk
    // dynamic LDS (BQ_LDS bytes), in granules:
    //   inb rows  [parity][clip], BQ_RP apart   input chunks (DMA targets, below 64 KB)
    //   outb rows [parity][clip], BQ_RP apart   the last sections' output chunks
    //   sec[lane][granule], rows G + 1 apart     the other sections' output chunks
    // sec rows land on successive 16-B bank slots (65 = 1 mod 16), so a wave's
    // 64 reads of sec[L-1][g] (and writes of sec[L][g]) are conflict-free.  The
    // inb / outb row of clip k is skewed to the bank slot of the sec row its
    // lane would otherwise use (section 0 reads "row L - 1", the last section
    // writes "row L"), which keeps the mixed accesses conflict-free too (PMC
    // without the skew: 43 % of LDS cycles were bank conflicts).
    extern __shared__ bq_f4 bq_lds[];
    const int ns = j.n_sos;
    constexpr int SEC0 = 4 * BQ_KPW * BQ_RP;      // first sec row, granules (a multiple of 16)
    bq_f4 (*sec)[G + 1] = (bq_f4 (*)[G + 1])(bq_lds + SEC0);
    auto inb_row = [=](int p, int k) __attribute__((always_inline)) {
        return (p * BQ_KPW + k) * BQ_RP + ((k * ns - 1) * (G + 1) & 15);
    };
    auto outb_row = [=](int p, int k) __attribute__((always_inline)) {
        return ((2 + p) * BQ_KPW + k) * BQ_RP + ((k * ns + ns - 1) * (G + 1) & 15);
    };
    const int kpw = min(64 / ns, BQ_KPW);          // clips per workgroup
    const int lane = threadIdx.x & 63;
    const int clip0 = blockIdx.x * kpw;
    const int nclip = min(kpw, j.n_clips - clip0);
    const int64_t N = j.frames;
    const int64_t nchunk = (N + CH - 1) / CH;
    const int64_t steps = nchunk + ns - 1;

    if (threadIdx.x >= 64) {
        bq_copy_wave<C>(j, clip0, nclip, steps, ns, inb_row, outb_row);
        return;
    }

    // ---------------- compute wave: the recurrences -------------------------
    const int s = lane % ns, kk = lane / ns;
    const bool valid = kk < nclip;
    const float *q = j.sos + 6 * s;                // this lane's section, state zero at clip start
    const float b0 = q[0], b1 = q[1], b2 = q[2], a1 = q[4], a2 = q[5];
    const bq_f2 cb0 = {b0, b0}, cb1 = {b1, b1}, cb2 = {b2, b2}, ca1 = {a1, a1}, ca2 = {a2, a2};
    V z0 = V(0.0f), z1 = V(0.0f);
    float *st = (ST && valid) ? j.state + ((size_t)(clip0 + kk) * ns + s) * 2 * C : nullptr;
    if (ST && st) {                                // streaming: continue from the previous block
        if constexpr (C == 2) { z0 = V{st[0], st[1]}; z1 = V{st[2], st[3]}; }
        else { z0 = st[0]; z1 = st[1]; }
    }
    const int kc = min(kk, BQ_KPW - 1);
    const bq_f4 *srow = &sec[(lane + 63) & 63][0];
    const bool last = s == ns - 1 && valid;        // idle lanes write their own (unread) sec row
    __syncthreads();
    for (int64_t i = 0; i < steps; ++i) {
        const int64_t c = i - s;                   // chunk this lane filters
        // every lane runs the chunk (uniform control flow); a lane outside its
        // chunk range keeps its state and its outputs are never stored
        const bool act = valid && c >= 0 && c < nchunk;
        const V z0s = z0, z1s = z1;
        // the last chunk's frames past N are zero padding: with a state to
        // carry they must not advance the recurrence
        const bool tail = ST && st && act && (c + 1) * CH > N;
        const bq_f4 *src = s ? srow : bq_lds + inb_row((int)(i & 1), kc);
        bq_f4 *dst = last ? bq_lds + outb_row((int)(i & 1), kc) : &sec[lane][0];
        // fully unrolled over the chunk: granule g + 2 is read while granule
        // g is filtered, so the LDS latency hides behind two granules
        bq_f4 n0 = src[0], n1 = src[1];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const bq_f4 v4 = n0;
            n0 = n1;
            if (g + 2 < G) n1 = src[g + 2];
            auto scalar = [&]() __attribute__((always_inline)) {
                bq_f4 r;
#pragma unroll
                for (int e = 0; e < FPL; ++e) {
                    V v;
                    if constexpr (C == 2) v = V{v4[2 * e], v4[2 * e + 1]};
                    else v = v4[e];
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
                return r;
            };
            bq_f4 r;
            if constexpr (C == 2) r = tail ? scalar() : bq_step2(v4, z0, z1, cb0, cb1, cb2, ca1, ca2);
            else r = scalar();
            dst[g] = r;
        }
        if (!act) { z0 = z0s; z1 = z1s; }
        __syncthreads();                           // chunk i + 1 staged; outputs visible to the copy wave
    }
    if (ST && st) {
        if constexpr (C == 2) { st[0] = z0.x; st[1] = z0.y; st[2] = z1.x; st[3] = z1.y; }
        else { st[0] = z0; st[1] = z1; }
    }
}

// ---- chain / load / store split: k_biquad_pc -------------------------------
// The recurrence of one (clip, section, channel) needs 4 dependent ops per
// frame; sosfilt's other ops are the 3 feed-forward products b_r * x, which do
// not depend on the state.  Lane = (clip, section, channel): the sections of a
// cascade are a pipeline across lanes, section s filtering chunk i - s at
// step i from section s-1's output row of step i - 1 (section 0: the planar
// input row).  The chain lane forms the products itself (v_mul_f32 /
// v_pk_mul_f32, IEEE-exact: the very products sosfilt takes) in the issue
// slots the dependent chain leaves idle, so per frame it issues 6 VALU (p0 =
// b0*x; (p1, p2) = (b1, b2)*x; o = p0 + z0; (t, u) = (-a1, -a2)*o; (t, z1') =
// (p1, p2) + (t, u); z0 = z1 + t: sosfilt's ops bit for bit, IEEE negation
// being exact) and moves 2 floats through LDS (its source frame in, its
// output out).  Round 3 handed the products from a producer wave through LDS
// (3 floats written and 3 read per frame, 13 of the workgroup's LDS floats per
// lane-frame against 4 here): the chain ran 39 cycles per frame, LDS-bound,
// against 24.4 for the bare recurrence (tools/ubench/bq_pk_chain.hip).
// Waves per workgroup:
//   chain (wave 0): section s filters chunk c = i - s from its source row
//     (16 ds_read_b128, the whole 64-frame chunk read first) into its own
//     planar output row O[lane][i & 1] (ds_write_b128 per 4 frames);
//   load (wave 3): the DMA of chunk i + 2 (global_load_lds_dwordx4 by per-lane
//     64-bit addresses, 4 / C clips per instruction) into inb[i & 1], waiting
//     only for chunk i + 1, which it then splits into the planar rows
//     PL[(i + 1) & 1] -- every chunk has two steps to land;
//   store (wave 2): the last section's rows O[(i - 1) & 1] (chunk i - ns),
//     interleaved in registers, to HBM, never waiting for a store;
//   wave 1 only keeps the barrier count (the SIMD order 0, 2, 1, 3 puts the
//     store wave beside the chain wave on the LDS store path).
// One barrier per step; chunks are 64 frames.  Rows are skewed by 4 floats
// per row so the 16-B row accesses of a wave are bank-conflict free.
constexpr int PC_CH = 64;                          // frames per chunk (per channel)
constexpr int PC_KPW = 12;                         // clips per workgroup at most
constexpr int PC_OS = 2 * PC_CH + 4;               // floats per lane: O[parity][frame] + skew
constexpr int PC_RS = PC_CH + 4;                   // floats per planar input row + skew
constexpr int PC_O0 = 0;                           // O rows (floats)
constexpr int PC_IN0 = PC_O0 + 64 * PC_OS;         // inb[chunk & 1][clip]: chunks of PC_CH * C floats, contiguous
constexpr int PC_PL0 = PC_IN0 + 2 * PC_KPW * PC_CH * 2;   // PL[chunk & 1][clip][ch]: rows of PC_RS floats
constexpr size_t PC_LDS = (size_t)(PC_PL0 + 2 * PC_KPW * 2 * PC_RS) * 4;   // 59,136 B
// two workgroups per CU (src/xm_audio_mixer.c run_fx_pipelined sizes its CU
// partition for that; 128-frame chunks, 116 KB: bq 7.07 ms against 7.36, but
// one workgroup per CU)
static_assert(PC_LDS <= 80 * 1024, "two workgroups per CU");
static_assert(PC_OS % 64 == 4 && PC_RS % 64 == 4 && PC_IN0 % 4 == 0 && PC_PL0 % 4 == 0,
              "16-B rows, 4-float skew per row");

// vmcnt(n) for a wave-uniform n <= 12 (the DMA groups of one chunk)
__device__ __forceinline__ void pc_vm_wait(int n)
{
    switch (n) {
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// The load wave: the DMA of chunk i + 2 into inb[(i + 2) % 3] at step i, so
// every chunk has two steps to land; only loads are in flight on this wave,
// and they return in order, so vmcnt(ng) at the end of step i leaves just
// chunk i + 2's ng DMAs outstanding (chunk i + 1 is in LDS).
template <int C>
__device__ __forceinline__ void pc_load_wave(const XmhFxJob &j, int clip0, int nclip, int64_t steps, float *lf)
{
    typedef const __attribute__((address_space(1))) float gcf;
    typedef __attribute__((address_space(3))) void lds_void;
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int CB = PC_CH * C * 4;              // chunk bytes per clip
    constexpr int LPC = CB / 16;                   // lanes per clip chunk
    constexpr int CPI = 64 / LPC;                  // clips per DMA instruction
    constexpr int NG = PC_KPW / CPI;               // instruction groups at most
    static_assert(NG <= 12, "pc_vm_wait covers 12 groups");
    const int lane = threadIdx.x & 63;
    const int64_t N = j.frames;
    const int64_t nchunk = (N + PC_CH - 1) / PC_CH, nfull = N / PC_CH;
    const int ng = (nclip + CPI - 1) / CPI;
    const int kl = lane / LPC;                     // this lane's clip within a group
    uint64_t xa[NG];
    const float *xp[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int k = min(g * CPI + kl, nclip - 1);   // loads of missing clips fill unused rows
        xp[g] = j.in_ptrs[clip0 + k];
        xa[g] = (uint64_t)(uintptr_t)xp[g] + (uint64_t)(lane % LPC) * 16u;
    }
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void *)lf);
    // issue chunk c; returns the DMAs left in flight (0: none, or loaded synchronously)
    auto load_chunk = [&](int64_t c) __attribute__((always_inline)) -> int {
        if (c >= nchunk) return 0;
        const int p = (int)(c & 1);
        if (c < nfull) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                if (g >= ng) break;                // wave-uniform
                const uint32_t m0 = lds0 + (uint32_t)(PC_IN0 + (p * PC_KPW + g * CPI) * PC_CH * C) * 4u;
                asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                             :
                             : "s"(m0), "v"(xa[g] + (uint64_t)c * CB)
                             : "memory", "m0");
            }
            return ng;
        }
        // partial last chunk: element loads with bounds, zero past N (the
        // compiler waits for these before the LDS writes)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            if (g >= ng) break;
            const int64_t s0 = c * PC_CH * C + (int64_t)(lane % LPC) * 4;
            f4 v = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (s0 + e < N * C) v[e] = ((gcf *)xp[g])[s0 + e];
            *(f4 *)(lf + PC_IN0 + (p * PC_KPW + g * CPI) * PC_CH * C + lane * 4) = v;
        }
        return 0;
    };
    // chunk c (landed in inb[c & 1]) -> planar rows PL[c & 1][clip][ch]
    auto planarize = [&](int64_t c) __attribute__((always_inline)) {
        if (c >= nchunk) return;
        const int p = (int)(c & 1);
        const f4 *ib = (const f4 *)(lf + PC_IN0 + p * PC_KPW * PC_CH * C);
        float *pl = lf + PC_PL0 + p * PC_KPW * 2 * PC_RS;
        for (int t = lane; t < nclip * (PC_CH / 4); t += 64) {   // (clip, frame quad)
            const int k = t / (PC_CH / 4), qd = t % (PC_CH / 4);
            if (C == 2) {
                const f4 u = ib[k * (PC_CH / 2) + 2 * qd], v = ib[k * (PC_CH / 2) + 2 * qd + 1];
                *(f4 *)(pl + (2 * k) * PC_RS + 4 * qd) = f4{u[0], u[2], v[0], v[2]};
                *(f4 *)(pl + (2 * k + 1) * PC_RS + 4 * qd) = f4{u[1], u[3], v[1], v[3]};
            } else {
                *(f4 *)(pl + (2 * k) * PC_RS + 4 * qd) = ib[k * (PC_CH / 4) + qd];
            }
        }
    };
    load_chunk(0);
    load_chunk(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    planarize(0);
    __syncthreads();
    for (int64_t i = 0; i < steps; ++i) {
        pc_vm_wait(load_chunk(i + 2));             // chunk i + 1 landed (inb[i & 1] was split at step i - 1)
        planarize(i + 1);
        __syncthreads();
    }
}

// The store wave: at step i the last section's output rows O[(i - 1) & 1]
// (chunk i - ns) -> interleaved 16-B segments -> HBM; it never waits for a
// store.
template <int C>
__device__ __forceinline__ void pc_store_wave(const XmhFxJob &j, int clip0, int nclip, int64_t steps, int ns,
                                              float *lf)
{
    typedef __attribute__((address_space(1))) float gf;
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    constexpr int CB = PC_CH * C * 4;
    constexpr int LPC = CB / 16;
    constexpr int CPI = 64 / LPC;
    constexpr int NG = PC_KPW / CPI;
    constexpr int CPG = 4 / C;                     // clips per 4-lane block
    const int lane = threadIdx.x & 63;
    const int64_t N = j.frames;
    const int64_t nchunk = (N + PC_CH - 1) / PC_CH, nfull = N / PC_CH;
    const int ng = (nclip + CPI - 1) / CPI;
    const int kl = lane / LPC, sg = lane % LPC;    // clip within a group, 16-B segment within its chunk
    uint64_t ya[NG];
    float *yp[NG];
    int orow[NG];                                  // O row (float offset) of the clip's channel 0
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int k = min(g * CPI + kl, nclip - 1);
        yp[g] = j.out_ptrs[clip0 + k];
        ya[g] = (uint64_t)(uintptr_t)yp[g] + (uint64_t)sg * 16u;
        const int ln = ((k / CPG) * ns + ns - 1) * 4 + (k % CPG) * C;   // the chain lane of (clip, last, ch 0)
        orow[g] = PC_O0 + ln * PC_OS;
    }
    __syncthreads();
    for (int64_t i = 0; i < steps; ++i) {
        const int64_t c = i - ns;
        if (c >= 0 && c < nchunk) {
            const int p = (int)((i - 1) & 1);
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                if (g >= ng) break;
                const float *o = lf + orow[g] + p * PC_CH;
                f4 v;
                if (C == 2) {                      // frames 2 sg, 2 sg + 1 of both channels
                    const f2 a = *(const f2 *)(o + 2 * sg), b = *(const f2 *)(o + PC_OS + 2 * sg);
                    v = f4{a[0], b[0], a[1], b[1]};
                } else {
                    v = *(const f4 *)(o + 4 * sg);
                }
                if (g * CPI + kl >= nclip) continue;   // a clamped lane: not its clip
                if (c < nfull) {
                    asm volatile("global_store_dwordx4 %0, %1, off" : : "v"(ya[g] + (uint64_t)c * CB), "v"(v) : "memory");
                } else {
                    const int64_t s0 = c * PC_CH * C + (int64_t)sg * 4;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (s0 + e < N * C) ((gf *)yp[g])[s0 + e] = v[e];
                }
            }
        }
        __syncthreads();
    }
}

template <int C, bool ST>
__global__ __launch_bounds__(256) void k_biquad_pc(XmhFxJob j)
{
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    constexpr int CPG = 4 / C;                     // clips per group (a block of 4 lanes)
    extern __shared__ bq_f4 bq_lds[];
    float *lf = (float *)bq_lds;
    const int ns = j.n_sos;
    const int gpw = 16 / ns;                       // groups per wave
    const int kpw = min(gpw * CPG, PC_KPW);        // clips per workgroup
    const int clip0 = blockIdx.x * kpw;
    const int nclip = min(kpw, j.n_clips - clip0);
    const int64_t N = j.frames;
    const int64_t nchunk = (N + PC_CH - 1) / PC_CH;
    const int64_t steps = nchunk + ns + 1;
    const int wave = threadIdx.x >> 6;
    // the store wave (LDS reads only) as wave 2: a workgroup's waves take the
    // SIMDs in the cyclic order 0, 2, 1, 3, so wave 2 shares the chain wave's
    // half of the LDS store path, which the load wave's writes no longer
    // contend for (7.36 -> 7.26-7.29 ms same box)
    constexpr int W_LOAD = 3, W_STORE = 2;
    if (wave == W_LOAD) {
        pc_load_wave<C>(j, clip0, nclip, steps, lf);
        return;
    }
    if (wave == W_STORE) {
        pc_store_wave<C>(j, clip0, nclip, steps, ns, lf);
        return;
    }
    if (wave == 1) {   // barriers only
        __syncthreads();
        for (int64_t i = 0; i < steps; ++i) __syncthreads();
        return;
    }
    const int lane = threadIdx.x & 63;
    const int blk = lane >> 2, r = lane & 3;
    const int grp = blk / ns, s = blk % ns, ci = r / C, ch = r % C;
    const int kk = grp * CPG + ci;
    const bool valid = blk < gpw * ns && kk < nclip;
    const int kq = valid ? kk : 0;
    const float *q = j.sos + 6 * (valid ? s : 0);
    const float b0 = q[0], b1 = q[1], b2 = q[2], a1 = q[4], a2 = q[5];
    const int O_lane = PC_O0 + lane * PC_OS;

    // ---------------- chain: 6 VALU per frame ---------------------------------
    const float na1 = -a1, na2 = -a2;              // (-a)*o == -(a*o): IEEE negation is exact
    const f2 nA = f2{na1, na2}, B12 = f2{b1, b2};
    float z0 = 0.0f, z1 = 0.0f;
    float *st = (ST && valid) ? j.state + ((size_t)(clip0 + kk) * ns + s) * 2 * C : nullptr;
    if (ST && st) {
        z0 = st[ch];
        z1 = st[C + ch];
    }
    __syncthreads();
    for (int64_t i = 0; i < steps; ++i) {
        const int64_t c = i - s;                   // chunk this lane filters
        const bool act = valid && c >= 0 && c < nchunk;
        const float z0s = z0, z1s = z1;
        const int par = (int)(i & 1);
        // chunk c: section s-1's output row (written at step i - 1), or the
        // planar input row (chunk i, split by the load wave at step i - 1)
        const float *src = valid && s == 0 ? lf + PC_PL0 + ((par * PC_KPW + kq) * 2 + ch) * PC_RS
                                           : lf + (valid ? O_lane - 4 * PC_OS : O_lane) + (par ^ 1) * PC_CH;
        float *Ow = lf + O_lane + par * PC_CH;
        // the whole source chunk first (the compiler cannot move these reads
        // past the output writes: same LDS array)
        f4 X[PC_CH / 4];
#pragma unroll
        for (int qd = 0; qd < PC_CH / 4; ++qd) X[qd] = ((const f4 *)src)[qd];
        const bool tail = ST && st && act && (c + 1) * PC_CH > N;
        if (__builtin_amdgcn_ballot_w64(tail) != 0) {
            // a streamed block's last chunk: frames past N are padding and must
            // not advance the state (wave-uniform branch)
#pragma unroll
            for (int f = 0; f < PC_CH; ++f) {
                const float x = X[f >> 2][f & 3];
                const float p0 = b0 * x, p1 = b1 * x, p2 = b2 * x;
                const float o = p0 + z0;
                if (!(tail && c * PC_CH + f >= N)) {
                    z0 = z1 + (p1 + na1 * o);
                    z1 = p2 + na2 * o;
                }
                Ow[f] = o;
            }
        } else {
            // quads of 4 frames.  Per frame 4 instructions on the 4-op
            // dependence: o = p0 + z0; (t, u) = (-a1, -a2) * o (v_pk_mul_f32);
            // (t, z1') = (p1, p2) + (t, u) (v_pk_add_f32); z0 = z1 + t -- each
            // half the very operation sosfilt takes; the products off it
#pragma unroll
            for (int qd = 0; qd < PC_CH / 4; ++qd) {
                // o of frames (0, 1) and (2, 3) built in place as register pairs: the
                // product (t, u) broadcasts o from the pair's low or high half by
                // op_sel, so no o is copied into the store pair (the compiler-
                // scheduled form moved every odd frame's o: 7.72-7.74 ms against
                // 7.32-7.33 ms on one box)
                f2 op[2];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float x = X[qd][e];
                    const float p0 = b0 * x;
                    const f2 p12 = B12 * f2{x, x};
                    f2 &oo = op[e >> 1];
                    f2 tu;
                    if (e & 1) {
                        oo.y = p0 + z0;
                        asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(tu) : "v"(nA), "v"(oo));
                    } else {
                        oo.x = p0 + z0;
                        asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(tu) : "v"(nA), "v"(oo));
                    }
                    const f2 rr = p12 + tu;
                    z0 = z1 + rr.x;
                    z1 = rr.y;
                }
                ((f4 *)Ow)[qd] = f4{op[0].x, op[0].y, op[1].x, op[1].y};
            }
        }
        if (!act) { z0 = z0s; z1 = z1s; }
        __syncthreads();                           // chunk i + 1's source rows ready; outputs visible
    }
    if (ST && st) {
        st[ch] = z0;
        st[C + ch] = z1;
    }
}

// ---- FIR, register-blocked: k_fir_rb ----------------------------------------
// upfirdn order per output: acc = +0, then acc = acc + x[n-K+1+t] * h[K-1-t]
// for t ascending.  A workgroup (4 waves) stages the input tile of its 1792
// output frames plus the K-1 frames before them in LDS with 16-B loads (the
// chunk grid of the absolute address: no per-element division), the left edge
// zero (or the streamed history).  Lane l of wave w owns FU = 7 consecutive
// outputs, so the 7 outputs of a tap share 6 of their 7 window frames: the
// window lives in registers (two 7-frame halves A, B that swap roles every
// 7-tap block, no moves), one LDS read per frame per 7 outputs x 7 taps, and
// each tap's coefficient h[K-1-t] is wave-uniform (scalar loads, an SGPR
// operand).  Stereo (L, R) ride in packed pairs: per output and tap one
// v_pk_mul_f32 + one v_pk_add_f32.  A lane stride of 7 frames (an odd number
// of 8-B frames) puts the 32 lanes of each ds_read_b64 half-wave on 32
// distinct bank pairs.  Outputs go back through wave-private LDS so the
// stores are whole 16-B chunks in frame order.
constexpr int FR_U = 7;                            // outputs per lane (odd: conflict-free reads)
constexpr int FR_WAVES = 4;
constexpr int FR_TILE = 64 * FR_U * FR_WAVES;      // output frames per workgroup (1792)

template <int C>
struct FrV;
template <>
struct FrV<1> { typedef float T; };
template <>
struct FrV<2> { typedef float T __attribute__((ext_vector_type(2))); };

template <int C>
__global__ __launch_bounds__(64 * FR_WAVES) void k_fir_rb(XmhFxJob j)
{
    typedef typename FrV<C>::T V;
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(1))) f4 gcf4;
    typedef __attribute__((address_space(1))) f4 gf4;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int K = j.fir_len;
    const int clip = blockIdx.y;
    const float *x = j.in_ptrs[clip];
    float *y = j.out_ptrs[clip];
    const int64_t N = j.frames;
    const int64_t n0 = (int64_t)blockIdx.x * FR_TILE;
    const int64_t f0 = n0 - K + 1;                 // first tile frame
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // the tile: floats [f0*C, (n0 + FR_TILE + 14)*C) of the clip (14 frames of
    // slack for the window's read-ahead), on the 16-B grid of absolute addresses
    const uint64_t xa = (uint64_t)(uintptr_t)x;
    // tile float i <-> clip float g0 + i, at LDS float i + sh, where sh puts
    // the LDS 16-B chunks on the 16-B grid of absolute addresses; a stereo
    // clip that is not 8-B aligned (frames would straddle) loads float by float
    const bool al = C == 1 || (xa & 7) == 0;
    const int64_t g0 = f0 * C;                     // clip float of tile float 0
    const int sh = al ? (int)((((int64_t)((xa >> 2) & 3) + g0) % 4 + 4) % 4) : 0;
    const int tile_f = (FR_TILE + K - 1 + 14) * C;
    float *tile = lds;                             // LDS floats [0, sh + tile_f) (rounded to 16 B)
    const int nchunk = (sh + tile_f + 3) / 4;
    const int64_t clip_hi = N * C;                 // clip floats
    for (int q = tid; q < nchunk; q += 64 * FR_WAVES) {
        const int64_t gi = g0 - sh + 4 * (int64_t)q;   // clip float of the chunk's first float
        f4 v;
        if (al && gi >= 0 && gi + 4 <= clip_hi) {
            v = *(gcf4 *)(x + gi);                 // a 16-B aligned chunk of the clip
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t g = gi + e;
                float u = 0.0f;
                if (g >= 0 && g < clip_hi) u = x[g];
                else if (g < 0 && g >= g0 && j.hist_in)   // streaming: the K-1 frames before this block
                    u = j.hist_in[(int64_t)clip * (K - 1) * C + (K - 1) * C + g];
                v[e] = u;
            }
        }
        *(f4 *)(tile + 4 * q) = v;
    }
    __syncthreads();

    const V *tv = (const V *)(tile + sh);          // tile frames (V = one frame)
    const int base = w * 64 * FR_U + lane * FR_U;  // tile frame of tap 0 of this lane's first output
    const float *h = j.fir;
    V acc[FR_U], A[FR_U], B[FR_U];
#pragma unroll
    for (int u = 0; u < FR_U; ++u) {
        acc[u] = V(0.0f);
        A[u] = tv[base + u];
        B[u] = tv[base + FR_U + u];
    }
    // one 7-tap block: acc[u] += W[u + t] * hb[t], W = P ++ Q (frames tb .. tb+13)
    auto block = [&](const V (&P)[FR_U], const V (&Q)[FR_U], const float *hb) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < FR_U; ++t) {
            const float hv = hb[t];                // wave-uniform (SGPR)
#pragma unroll
            for (int u = 0; u < FR_U; ++u) {
                const V xv = u + t < FR_U ? P[u + t] : Q[u + t - FR_U];
                acc[u] = acc[u] + xv * hv;
            }
        }
    };
    // the 14 coefficients of a loop iteration, h[K-1-t] for t = tb .. tb+13:
    // the contiguous taps h[K-14-tb .. K-1-tb] by wide scalar loads, issued
    // one iteration ahead of their use (past the last iteration the block
    // start clamps to tap 0: loaded, never used)
    auto coefs = [&](float (&hc)[2 * FR_U], int tb) __attribute__((always_inline)) {
        const float *hb = h + max(K - 2 * FR_U - tb, 0);
        float blk[2 * FR_U];
#pragma unroll
        for (int i = 0; i < 2 * FR_U; ++i) blk[i] = hb[i];
#pragma unroll
        for (int i = 0; i < 2 * FR_U; ++i) hc[i] = blk[2 * FR_U - 1 - i];
    };
    int tb = 0;
    float hc[2 * FR_U];
    coefs(hc, 0);
    for (; tb + 2 * FR_U <= K; tb += 2 * FR_U) {
        float hn[2 * FR_U];
        coefs(hn, tb + 2 * FR_U);
        block(A, B, hc);
#pragma unroll
        for (int u = 0; u < FR_U; ++u) A[u] = tv[base + tb + 2 * FR_U + u];
        block(B, A, hc + FR_U);
#pragma unroll
        for (int u = 0; u < FR_U; ++u) B[u] = tv[base + tb + 3 * FR_U + u];
#pragma unroll
        for (int i = 0; i < 2 * FR_U; ++i) hc[i] = hn[i];
    }
    if (tb + FR_U <= K) {                          // one more whole block: then the window is B ++ next
        // (hc was loaded with a clamped block start here: the taps come
        // straight from h)
        float hl[FR_U];
#pragma unroll
        for (int t = 0; t < FR_U; ++t) hl[t] = h[K - 1 - (tb + t)];
        block(A, B, hl);
#pragma unroll
        for (int u = 0; u < FR_U; ++u) {
            A[u] = B[u];
            B[u] = tv[base + tb + 2 * FR_U + u];
        }
        tb += FR_U;
    }
    // the last K - tb (< 7) taps, window A ++ B
    const int rem = K - tb;
#pragma unroll
    for (int t = 0; t < FR_U - 1; ++t) {
        if (t >= rem) break;                       // wave-uniform
        const float hv = h[K - 1 - (tb + t)];
#pragma unroll
        for (int u = 0; u < FR_U; ++u) {
            const V xv = u + t < FR_U ? A[u + t] : B[u + t - FR_U];
            acc[u] = acc[u] + xv * hv;
        }
    }
    // (measured and dropped: storing whole aligned tiles straight from the
    // registers, 7 x 8-B frames per lane, saved 1.5 % at K = 63 but cost 22 %
    // at K = 15, where the partial-line writes set the pace)
    // outputs -> wave-private LDS (after the whole workgroup is done with the
    // tile) -> whole 16-B chunks in frame order
    __syncthreads();
    V *ov = (V *)lds + w * 64 * FR_U;
#pragma unroll
    for (int u = 0; u < FR_U; ++u) ov[lane * FR_U + u] = acc[u];
    const int64_t wn0 = n0 + w * 64 * FR_U;        // this wave's first output frame
    const float *of = (const float *)ov;
    const int64_t og0 = wn0 * C;                   // clip float of the wave's first output float
    constexpr int OWF = 64 * FR_U * C;             // floats per wave
    const int osh = (int)(((uint64_t)(uintptr_t)(y + og0) >> 2) & 3);   // floats before a 16-B boundary
    const int lead = osh ? 4 - osh : 0;
    for (int i = lane; i < lead; i += 64)          // unaligned head, element by element
        if (og0 + i < N * C) y[og0 + i] = of[i];
    for (int q = lane; 4 * q + lead + 4 <= OWF; q += 64) {
        const int i = lead + 4 * q;
        if (og0 + i + 4 <= N * C) {
            *(gf4 *)(y + og0 + i) = f4{of[i], of[i + 1], of[i + 2], of[i + 3]};
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (og0 + i + e < N * C) y[og0 + i + e] = of[i + e];
        }
    }
    const int body = lead + ((OWF - lead) / 4) * 4;
    for (int i = body + lane; i < OWF; i += 64)    // tail
        if (og0 + i < N * C) y[og0 + i] = of[i];
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

extern "C" int xmg_launch_fx_biquad(const XmhFxJob *j, void *stream)
{
    if (j->n_sos < 1 || j->n_sos > BQ_MAXSEC || (j->channels != 1 && j->channels != 2)) return -1003;
    if (j->n_clips == 0 || j->frames == 0) return 0;

    // cascades of up to 16 sections: chain / load / store waves
    // (k_biquad_pc); longer ones: the section-pipelined k_biquad_pipe
    if (j->n_sos <= 16) {
        auto pk = j->channels == 2 ? (j->state ? k_biquad_pc<2, true> : k_biquad_pc<2, false>)
                                   : (j->state ? k_biquad_pc<1, true> : k_biquad_pc<1, false>);
        const int kpw = std::min(16 / j->n_sos * (4 / j->channels), PC_KPW);
        // dev knob XM_BQ_LDS=bytes: a larger LDS request (>= 81920: one
        // workgroup per CU) for placement experiments
        static const int lds_req = [] {
            const char *e = getenv("XM_BQ_LDS");
            const int v = e ? atoi(e) : 0;
            return v > (int)PC_LDS && v <= 160 * 1024 ? v : (int)PC_LDS;
        }();
        if (xmg_func_lds((const void *)pk, lds_req)) return -1001;   // once per (kernel, device)
        XmhFxJob jj = *j;
        hipLaunchKernelGGL(pk, dim3((unsigned)((j->n_clips + kpw - 1) / kpw)), dim3(256), (size_t)lds_req,
                           (hipStream_t)stream, jj);
        return hipGetLastError() == hipSuccess ? 0 : -1001;
    }
    auto kern = j->channels == 2 ? (j->state ? k_biquad_pipe<2, true> : k_biquad_pipe<2, false>)
                                 : (j->state ? k_biquad_pipe<1, true> : k_biquad_pipe<1, false>);
    const int kpw = std::min(64 / j->n_sos, BQ_KPW);
    dim3 grid((unsigned)((j->n_clips + kpw - 1) / kpw));
    if (xmg_func_lds((const void *)kern, (int)BQ_LDS)) return -1001;   // once per (kernel, device)
    XmhFxJob jj = *j;
    hipLaunchKernelGGL(kern, grid, dim3(128), BQ_LDS, (hipStream_t)stream, jj);
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}

extern "C" int xmg_launch_fx_fir(const XmhFxJob *j, void *stream)
{
    const int K = j->fir_len;
    if (j->frames == 0 || j->n_clips == 0) return 0;
    if (j->hist_in && K > 1) {                        // streaming: next block's history first
        if (!j->hist_out || j->hist_out == j->hist_in) return -22;
        auto hk = j->channels == 1 ? k_fir_hist<1> : k_fir_hist<2>;
        hipLaunchKernelGGL(hk, dim3((unsigned)((K - 1) * j->channels + 255) / 256, (unsigned)j->n_clips), 256, 0,
                           (hipStream_t)stream, *j);
        if (hipGetLastError() != hipSuccess) return -1001;
    }
    const size_t rl = ((size_t)(FR_TILE + K - 1 + 14) * j->channels + 8) * sizeof(float);
    const size_t lds_rb = std::max(rl, (size_t)FR_TILE * j->channels * sizeof(float));
    if (lds_rb > 160 * 1024) return -1003;
    auto kr = j->channels == 1 ? k_fir_rb<1> : k_fir_rb<2>;
    if (lds_rb > 64 * 1024 && xmg_func_lds((const void *)kr, (int)lds_rb)) return -1001;
    hipLaunchKernelGGL(kr, dim3((unsigned)((j->frames + FR_TILE - 1) / FR_TILE), (unsigned)j->n_clips),
                       64 * FR_WAVES, lds_rb, (hipStream_t)stream, *j);
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}

extern "C" int xmg_synth(void *out, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips,
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
