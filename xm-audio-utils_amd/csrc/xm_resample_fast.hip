// xm_resample_fast.hip — the headline kernel: 48 kHz -> 44.1 kHz (L/M =
// 147/160) polyphase resample of stereo fp32 tracks + per-track gain ramp +
// in-order track sum, fused in one pass over HBM (SURVEY.md §8(a) a2+a4+a7).
//
// Arithmetic is scipy resample_poly's (include/xm_audio_common.h): per output
// acc = sum_t x[j0+t]*H[ph][t] in ascending t, each mul and add rounded
// separately (-ffp-contract=off), then mix = ((+0 + g0*r0) + g1*r1) + ...
// Two exact shortcuts, both argued in DESIGN.md §"Exactness of the fast path":
//  * tap 22 of every phase is an exact 0 for 147/160 (the 160-zero pre-pad),
//    so each output uses taps 0..21 (finite inputs);
//  * the +0 seeds of the dot product and of the mix are folded into one
//    final "+ 0.0f", which maps -0 to +0 and leaves every other value alone.
//
// Work decomposition (MI355X-first):
//  * super-period (SP) = 160 input frames -> 147 output frames; the filter
//    phase of output k of an SP does not depend on the SP, so a wave whose
//    64 lanes hold 64 consecutive SPs of ONE track runs a wave-uniform phase
//    sequence: the 22 coefficients of every output come from the scalar
//    cache as SGPR operands of v_pk_mul_f32 (stereo L/R packed), never from
//    VGPRs or LDS;
//  * the SP's 147 outputs are fully unrolled, so the sliding window over the
//    lane's 186 input frames is a static register window: every input frame
//    is loaded once (16-B buffer loads, 4 back-to-back per 64-B sector) and
//    used by up to 22 outputs from registers;
//  * buffer-resource range checking zero-fills frames outside [0, N): no
//    branches for clip edges (the lane holding SP 0 points its first 8
//    loads out of range);
//  * a workgroup = NT track waves x (8/NT) SP groups.  Each round of 8
//    outputs the waves exchange gain*r through a 32 KiB LDS buffer (double
//    buffered), one barrier, and every lane adds one output's NT tracks in
//    track order — the mix never touches HBM as partial sums.
#include <string.h>
#include "xm_device.h"

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
// Coefficients are read through the constant address space: wave-uniform
// addresses there always lower to s_load (scalar cache -> SGPR operands).
typedef const float __attribute__((address_space(4))) cfloat;

constexpr int L = 147, M = 160, RM = 11;   // reduced ratio, output offset rm
constexpr int TE = 22;                     // taps used (tap 22 is an exact zero)
constexpr int SPO = L;                     // outputs per super-period
constexpr int SPI = M;                     // input frames per super-period
constexpr int F0 = -16;                    // first loaded frame, relative to 160*sp
constexpr int G = 8;                       // outputs per exchange round
constexpr int ROUNDS = (SPO + G - 1) / G;  // 19
constexpr int WAVES = 8;                   // waves per workgroup
constexpr int HK_STRIDE = 24;              // floats per output row of the k-ordered table

// Input frame (relative to 160*sp + F0) of tap 0 for output k of an SP.
// (scipy: j0 = floor((m+rm)*M/L) - T + 1 with T = 23; relative to 160*sp + F0)
__host__ __device__ constexpr int rk(int k) { return ((k + RM) * M) / L - 22 - F0; }
// last pair (16 B = 2 frames) needed by outputs [0, k]
constexpr int last_pair(int k) { return (rk(k) + TE - 1) / 2; }
constexpr int first_pair() { return rk(0) / 2; }
constexpr int NPAIR = last_pair(SPO - 1) + 1;                   // 93 pairs = 186 frames
static_assert(rk(0) == 5, "window origin");
static_assert(NPAIR == 93, "pairs per SP");

struct FastArgs {
    const float *in;
    int64_t in_track_stride, in_mix_stride;     // floats
    const void *const *in_ptrs;
    float *out;
    int64_t out_mix_stride;                     // floats
    void *const *out_ptrs;
    const float *Hk;                            // [147][24] coefficients in output order
    int32_t n_mix, n_tracks;
    int32_t frames_in, frames_out;
    int32_t n_sp, groups_per_mix;
    int32_t unity;
    int32_t pad;
    XmhGain g[8];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes)
{
    // stride 0, num_records = bytes, default dword format flags for gfx950 raw buffers
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ float4 bload(__amdgpu_buffer_rsrc_t r, uint32_t voff, int imm)
{
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff + imm, 0, 0));
}

// exact per-output gain (xm_device.h::xm_gain_f32 with wave-uniform params)
__device__ __forceinline__ float gain_at(const XmhGain &g, int n)
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

template <int NT, bool UNITY>
__global__ __launch_bounds__(512) void k_rs147_mix(FastArgs a)
{
    extern __shared__ __attribute__((aligned(16))) f2 xbuf[];   // [2][G][NT][SPWG]
    constexpr int SPG = WAVES / NT;            // SP groups per workgroup
    constexpr int SPWG = 64 * SPG;             // SPs per workgroup
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tr = w % NT;                     // this wave's track
    const int grp = w / NT;                    // this wave's SP group within the WG
    const int mix = blockIdx.x / a.groups_per_mix;
    const int wg_sp0 = (blockIdx.x % a.groups_per_mix) * SPWG;
    const int sp_local = grp * 64 + lane;
    const int sp = wg_sp0 + sp_local;          // super-period of this lane

    const float *trk = a.in_ptrs ? (const float *)a.in_ptrs[(int64_t)mix * a.n_tracks + tr]
                                 : a.in + (int64_t)mix * a.in_mix_stride + (int64_t)tr * a.in_track_stride;
    // The resource starts 16 frames before the clip so every in-clip offset
    // is non-negative (no 32-bit wrap): frame f lives at byte (f + 16) * 8 and
    // num_records = (N + 16) * 8 makes every frame >= N read as 0.  The lane
    // holding SP 0 sends its first 8 loads (frames -16..-1) out of range, so
    // they read 0 too and the bytes before the clip are never touched.
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(trk + 2 * F0, (uint32_t)(a.frames_in - F0) * 8u);
    const uint32_t vbase = (uint32_t)sp * (SPI * 8u);
    const uint32_t vlo = sp == 0 ? 0x80000000u : vbase;

    XmhGain gp = a.g[0];
#pragma unroll
    for (int i = 1; i < NT; ++i)
        if (tr == i) gp = a.g[i];   // wave-uniform select: keeps the params in SGPRs
    cfloat *Hk = (cfloat *)a.Hk;

    f2 x[2 * NPAIR];
    auto load_pair = [&](int p) {
        const float4 v = p < 8 ? bload(rs, vlo, p * 16) : bload(rs, vbase, p * 16);
        x[2 * p] = f2{v.x, v.y};
        x[2 * p + 1] = f2{v.z, v.w};
    };

    // prologue: everything round 0 needs
#pragma unroll
    for (int p = first_pair(); p <= last_pair(G - 1); ++p) load_pair(p);

    float *ob = a.out_ptrs ? (float *)a.out_ptrs[mix] : a.out + (int64_t)mix * a.out_mix_stride;

#pragma unroll
    for (int q = 0; q < ROUNDS; ++q) {
        const int k0 = q * G;
        const int kend = k0 + G < SPO ? k0 + G : SPO;
        // prefetch the pairs the next round adds
        if (q + 1 < ROUNDS) {
            const int kn = (q + 2) * G - 1 < SPO ? (q + 2) * G - 1 : SPO - 1;
#pragma unroll
            for (int p = last_pair(kend - 1) + 1; p <= last_pair(kn); ++p) load_pair(p);
        }
        // gains of this round (per lane: its SP's output frames n0..n0+7)
        const int n0 = sp * SPO + k0;
        float gk[G];
        if (UNITY) {
#pragma unroll
            for (int i = 0; i < G; ++i) gk[i] = 1.0f;
        } else {
            const bool vary = gp.len == 0 ? (n0 < (int)gp.start && n0 + G - 1 >= (int)gp.start)
                                          : (n0 + G - 1 > (int)gp.start && n0 < (int)gp.start + gp.len);
            if (__builtin_amdgcn_ballot_w64(vary)) {
#pragma unroll
                for (int i = 0; i < G; ++i) gk[i] = gain_at(gp, n0 + i);
            } else {
                const float g = gain_at(gp, n0);
#pragma unroll
                for (int i = 0; i < G; ++i) gk[i] = g;
            }
        }
        f2 *buf = xbuf + (q & 1) * (G * NT * SPWG);
        // two outputs at a time: two independent add chains interleaved so the
        // dependent pk_add latency of one hides behind the other's work
#pragma unroll
        for (int k = k0; k < kend; k += 2) {
            const bool two = k + 1 < kend;
            cfloat *h0 = Hk + k * HK_STRIDE;
            cfloat *h1 = Hk + (two ? k + 1 : k) * HK_STRIDE;
            const int ra = rk(k), rb = rk(two ? k + 1 : k);
            f2 acc0 = x[ra] * h0[0];
            f2 acc1 = x[rb] * h1[0];
#pragma unroll
            for (int t = 1; t < TE; ++t) {
                acc0 = acc0 + x[ra + t] * h0[t];
                if (two) acc1 = acc1 + x[rb + t] * h1[t];
            }
            buf[((k - k0) * NT + tr) * SPWG + sp_local] = UNITY ? acc0 : acc0 * gk[k - k0];
            if (two) buf[((k + 1 - k0) * NT + tr) * SPWG + sp_local] = UNITY ? acc1 : acc1 * gk[k + 1 - k0];
        }
        // LDS writes visible to the other waves; global loads stay in flight
        // (a __syncthreads() fence would drain vmcnt, i.e. the prefetch).
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // exchange: lane handles output k0 + kk of SP spo, summing NT tracks in order
        constexpr int OUT_PER_LANE = (G * SPWG) / (64 * WAVES);   // = 8 / NT
#pragma unroll
        for (int o = 0; o < OUT_PER_LANE; ++o) {
            const int idx = (o * WAVES + w) * 64 + lane;          // 0 .. G*SPWG-1
            const int kk = idx / SPWG, spo = idx % SPWG;
            if (k0 + kk < kend) {
                f2 s = buf[(kk * NT + 0) * SPWG + spo];
#pragma unroll
                for (int t2 = 1; t2 < NT; ++t2) s = s + buf[(kk * NT + t2) * SPWG + spo];
                s = s + f2{0.0f, 0.0f};                           // -0 -> +0 (scipy seeds are +0)
                const int64_t n = (int64_t)(wg_sp0 + spo) * SPO + k0 + kk;
                if (n < a.frames_out) *(f2 *)(ob + n * 2) = s;
            }
        }
    }
}

}  // namespace

// Host-side k-ordered coefficient table for the fast path:
// Hk[k][t] = H[((k+rm)*M) % L][t], t < 22, rows padded to 24 floats.
extern "C" int xmh_fast_table_147_160(const float *H, int T, float *Hk /* 147*24 */)
{
    if (T != 23) return -1003;
    for (int ph = 0; ph < L; ++ph)
        if (H[ph * T + 22] != 0.0f) return -1003;   // tap 22 must be an exact zero
    for (int k = 0; k < SPO; ++k) {
        const int ph = ((k + RM) * M) % L;
        for (int t = 0; t < HK_STRIDE; ++t) Hk[k * HK_STRIDE + t] = t < TE ? H[ph * T + t] : 0.0f;
    }
    return 0;
}

extern "C" int xmh_launch_mix_fast(const XmhMixJob *j, void *stream, int *n_launches)
{
    const int NT = j->n_tracks;
    if (!(j->rs.L == L && j->rs.M == M && j->rs.rm == RM && j->rs.T == 23 && j->rs.Hrun) ||
        j->fmt != 2 || j->channels != 2 || !(NT == 1 || NT == 2 || NT == 4 || NT == 8) ||
        j->frames_in <= 0 || j->frames_in >= (1 << 27) || j->n_mix <= 0)
        return -1003;   // not this kernel's job: generic path
    FastArgs a;
    memset(&a, 0, sizeof a);
    a.in = (const float *)j->in;
    a.in_track_stride = j->in_track_stride;
    a.in_mix_stride = j->in_mix_stride;
    a.in_ptrs = j->in_ptrs;
    a.out = (float *)j->out;
    a.out_mix_stride = j->out_mix_stride;
    a.out_ptrs = j->out_ptrs;
    a.Hk = j->rs.Hrun;
    a.n_mix = j->n_mix;
    a.n_tracks = NT;
    a.frames_in = (int32_t)j->frames_in;
    a.frames_out = (int32_t)j->frames_out;
    a.n_sp = (int32_t)((j->frames_out + SPO - 1) / SPO);
    const int spwg = 64 * (WAVES / NT);
    a.groups_per_mix = (a.n_sp + spwg - 1) / spwg;
    a.unity = j->unity;
    if (!j->gains_host) return -1003;
    for (int i = 0; i < NT; ++i) {
        a.g[i] = j->gains_host[i];
        // outputs are < 2^27: clamping the ramp start to +-2^28 keeps
        // clamp(n - start, 0, len) unchanged and fits int32 arithmetic
        const int64_t lim = (int64_t)1 << 28;
        a.g[i].start = a.g[i].start < -lim ? -lim : (a.g[i].start > lim ? lim : a.g[i].start);
    }
    const size_t lds = 2 * G * 512 * sizeof(f2);   // 64 KiB
    const int64_t blocks = (int64_t)a.n_mix * a.groups_per_mix;
    if (blocks > 0x7fffffff) return -1003;
    const bool u = j->unity && NT == 1;
    auto kern = NT == 1 ? (u ? k_rs147_mix<1, true> : k_rs147_mix<1, false>)
              : NT == 2 ? k_rs147_mix<2, false> : NT == 4 ? k_rs147_mix<4, false> : k_rs147_mix<8, false>;
    static bool attr_done[5];
    const int ai = NT == 1 ? (u ? 4 : 0) : NT == 2 ? 1 : NT == 4 ? 2 : 3;
    if (!attr_done[ai]) {
        if (hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return -1001;
        attr_done[ai] = true;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(512), lds, (hipStream_t)stream, a);
    if (n_launches) *n_launches += 1;
    return hipGetLastError() == hipSuccess ? 0 : -1001;
}
