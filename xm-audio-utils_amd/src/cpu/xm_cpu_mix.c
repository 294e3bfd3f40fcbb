/*
 * xm_cpu_mix.c — the CPU backend's mix jobs: polyphase resample + gain ramp +
 * ordered track sum (include/xm_audio_common.h), the
 * timeline mix (§8(f) 2-3) and config 5's finish.  Every output is the same
 * separately rounded fp32 / Q15 arithmetic, in the same order, as the gfx950
 * kernels (csrc/xm_mix_generic.hip, csrc/xm_resample_fast.hip), so a CPU
 * handle and a GPU handle give the same bits.
 *
 * Resampling layout.  Output m = m0 + v*L + k (k < L) has the filter phase of
 * output m0 + k and reads the input M*v frames later: the L outputs of a
 * "block" repeat with period M in the input.  A chunk is VW = 16 consecutive
 * blocks; the input window of each block is staged channel by channel into
 * xt[f][v] (block v in vector lane v), so output k of all 16 blocks is one
 * vertical SIMD dot product over the taps, coefficient broadcast from the
 * phase table, taps in ascending order from +0: exactly the scalar
 * acc = acc + x*h chain per lane.  Frames outside [0, N) are staged as 0
 * (equal to scipy's skipped taps up to the sign of zero, which the +0-seeded
 * chain never produces: xm_audio_common.h).
 */
#include <stdlib.h>
#include <string.h>

#include "xm_cpu.h"

#define VW 16
typedef float v16f __attribute__((vector_size(64)));

/* the tap loops are compiled for AVX-512, AVX2 and baseline x86-64 and picked
 * at load time; -ffp-contract=off keeps every mul and add separate in each */
#if defined(__x86_64__) && !defined(__SANITIZE_ADDRESS__)
#define XMC_SIMD __attribute__((target_clones("avx512f", "avx2", "default")))
#else
#define XMC_SIMD
#endif

#define XM_EINVAL_ (-22)
#define XM_ENOMEM_ (-12)

typedef struct {
    const XmhMixJob *j;
    int C, s16, resample, in_conv, in_planar, out_planar, in_elem, out_elem;
    int L, M, T;
    int64_t rm, N, ob, ib, fo;
    int64_t per_item, items_per_mix;
    /* resampling: phase and window offset of output k of a chunk, relative to
     * the chunk's first input frame (the same for every chunk: chunks start
     * L*VW outputs apart, so m0 mod L is fixed); F = frames staged per block */
    int32_t *ph, *jb;
    int F;
    int rc;
} MixCtx;

static const void *track_ptr(const XmhMixJob *j, int64_t b, int tr, int elem)
{
    if (j->in_ptrs) return j->in_ptrs[b * j->n_tracks + tr];
    return (const char *)j->in + (b * j->in_mix_stride + (int64_t)tr * j->in_track_stride) * elem;
}

static void *out_ptr(const XmhMixJob *j, int64_t b, int elem)
{
    if (j->out_ptrs) return j->out_ptrs[b];
    return (char *)j->out + b * j->out_mix_stride * elem;
}

/* cnt frames of channel c from absolute frame a0 on, as the mix's resampler
 * sees them (f32 mix: the sample, or s16 x 2^-15; s16 mix: the integer value,
 * or sat16(rint(f32 x 32768))), to dst[i*ds]; 0 outside [0, N) */
static void load_run(const MixCtx *x, const void *trk, int64_t a0, int cnt, int c, float *dst, int ds)
{
    int i = 0;
    for (; i < cnt && a0 + i < 0; ++i) dst[(size_t)i * ds] = 0.0f;
    int64_t hi = x->N - a0;
    if (hi > cnt) hi = cnt;
    if (i < hi) {
        const int64_t st = x->in_planar ? 1 : x->C;
        const int64_t q0 = (x->in_planar ? (int64_t)c * x->N + a0 : (a0 - x->ib) * x->C + c) + i * st;
        const int n = (int)hi - i;
        float *d = dst + (size_t)i * ds;
        if (!x->s16 && !x->in_conv) {
            const float *s = (const float *)trk + q0;
            for (int k = 0; k < n; ++k) d[(size_t)k * ds] = s[k * st];
        } else if (!x->s16) {
            const int16_t *s = (const int16_t *)trk + q0;
            for (int k = 0; k < n; ++k) d[(size_t)k * ds] = (float)s[k * st] * 0x1p-15f;
        } else if (!x->in_conv) {
            const int16_t *s = (const int16_t *)trk + q0;
            for (int k = 0; k < n; ++k) d[(size_t)k * ds] = (float)s[k * st];
        } else {
            const float *s = (const float *)trk + q0;
            for (int k = 0; k < n; ++k) d[(size_t)k * ds] = (float)xmc_round_sat16(s[k * st] * 32768.0f);
        }
        i = (int)hi;
    }
    for (; i < cnt; ++i) dst[(size_t)i * ds] = 0.0f;
}

/* r[k][v] = sum over t (ascending, from +0) of xt[jb[k] + t][v] * H[ph[k]][t] */
XMC_SIMD static void rs_block(float *restrict r, const float *restrict xt, const float *restrict H,
                              const int32_t *restrict ph, const int32_t *restrict jb, int L, int T)
{
    v16f *ro = (v16f *)r;
    const v16f *xv = (const v16f *)xt;
    int k = 0;
    for (; k + 4 <= L; k += 4) {   /* four independent chains hide the add latency */
        const float *h0 = H + (size_t)ph[k] * T, *h1 = H + (size_t)ph[k + 1] * T;
        const float *h2 = H + (size_t)ph[k + 2] * T, *h3 = H + (size_t)ph[k + 3] * T;
        const v16f *x0 = xv + jb[k], *x1 = xv + jb[k + 1], *x2 = xv + jb[k + 2], *x3 = xv + jb[k + 3];
        v16f a0 = {0}, a1 = {0}, a2 = {0}, a3 = {0};
        for (int t = 0; t < T; ++t) {
            a0 = a0 + x0[t] * h0[t];
            a1 = a1 + x1[t] * h1[t];
            a2 = a2 + x2[t] * h2[t];
            a3 = a3 + x3[t] * h3[t];
        }
        ro[k] = a0;
        ro[k + 1] = a1;
        ro[k + 2] = a2;
        ro[k + 3] = a3;
    }
    for (; k < L; ++k) {
        const float *h0 = H + (size_t)ph[k] * T;
        const v16f *x0 = xv + jb[k];
        v16f a0 = {0};
        for (int t = 0; t < T; ++t) a0 = a0 + x0[t] * h0[t];
        ro[k] = a0;
    }
}

/* output sample i of mix b from its f32 or int32 sum (the kernels' store epilogues) */
static inline void store_f32(const MixCtx *x, void *o, int64_t i, float acc)
{
    if (x->j->out_conv == 1) ((int16_t *)o)[i] = (int16_t)xmc_round_sat16(acc * 32768.0f);
    else ((float *)o)[i] = acc + 0.0f;   /* -0 -> +0 (the contract's +0 seed) */
}

static inline void store_i32(const MixCtx *x, void *o, int64_t i, int32_t acc)
{
    if (x->j->partial) ((int32_t *)o)[i] = acc;
    else if (x->j->out_conv == 2) ((float *)o)[i] = (float)xmc_sat16(acc) * 0x1p-15f;
    else ((int16_t *)o)[i] = xmc_sat16(acc);
}

static inline int64_t out_idx(const MixCtx *x, int64_t m_rel, int c)
{
    return x->out_planar ? (int64_t)c * x->fo + m_rel : m_rel * x->C + c;
}

/* ---- resampling mixes: one item = mix b, outputs [o0, o1) (relative) ----- */
static void item_resample(void *vctx, int64_t item)
{
    MixCtx *x = vctx;
    const XmhMixJob *j = x->j;
    const int C = x->C, L = x->L, T = x->T, F = x->F, nt = j->n_tracks;
    const int64_t b = item / x->items_per_mix, q = item % x->items_per_mix;
    const int64_t o0 = q * x->per_item, o1 = o0 + x->per_item < x->fo ? o0 + x->per_item : x->fo;
    const size_t blk = (size_t)L * VW;   /* outputs per chunk */
    float *xt = aligned_alloc(64, sizeof(float) * (size_t)F * VW * C);
    float *r = aligned_alloc(64, sizeof(float) * blk);
    float *accf = aligned_alloc(64, sizeof(float) * blk * C);   /* f32 sums, or int32 (s16 mixes) */
    float *gb = aligned_alloc(64, sizeof(float) * blk);          /* per-output gains, or Q15 gains */
    if (!xt || !r || !accf || !gb) {
        x->rc = XM_ENOMEM_;
        goto out;
    }
    int32_t *acci = (int32_t *)accf, *gq = (int32_t *)gb;
    void *o = out_ptr(j, b, x->out_elem);
    for (int64_t c0 = o0; c0 < o1; c0 += (int64_t)blk) {
        const int64_t m0 = x->ob + c0;                            /* absolute output frame of (k, v) = (0, 0) */
        const int64_t mend = x->ob + (c0 + (int64_t)blk < o1 ? c0 + (int64_t)blk : o1);
        const int64_t J0 = ((m0 + x->rm) * x->M) / L - T + 1;      /* first input frame of block 0 */
        memset(accf, 0, sizeof(float) * blk * C);                 /* +0.0f / 0 */
        for (int tr = 0; tr < nt; ++tr) {
            const void *trk = track_ptr(j, b, tr, x->in_elem);
            for (int c = 0; c < C; ++c)
                for (int v = 0; v < VW; ++v) load_run(x, trk, J0 + (int64_t)v * x->M, F, c, xt + (size_t)c * F * VW + v, VW);
            const XmhGain *g = &j->gains[tr];
            const int konst = xmc_gain_const(g, m0, m0 + (int64_t)blk - 1);
            if (!konst)
                for (int k = 0; k < L; ++k)
                    for (int v = 0; v < VW; ++v) {
                        const int64_t m = m0 + (int64_t)v * L + k;
                        if (x->s16) gq[k * VW + v] = xmc_gain_q15(g, m);
                        else gb[k * VW + v] = xmc_gain_f32(g, m);
                    }
            for (int c = 0; c < C; ++c) {
                rs_block(r, xt + (size_t)c * F * VW, j->rs.H, x->ph, x->jb, L, T);
                if (x->s16) {
                    int32_t *a = acci + (size_t)c * blk;
                    const int32_t g1 = konst ? xmc_gain_q15(g, m0) : 0;
                    for (size_t i = 0; i < blk; ++i)
                        a[i] += xmc_q15_term(xmc_round_sat16(r[i]), konst ? g1 : gq[i]);
                } else {
                    float *a = accf + (size_t)c * blk;
                    if (konst) {
                        const float g1 = xmc_gain_f32(g, m0);
                        for (size_t i = 0; i < blk; ++i) a[i] = a[i] + g1 * r[i];
                    } else {
                        for (size_t i = 0; i < blk; ++i) a[i] = a[i] + gb[i] * r[i];
                    }
                }
            }
        }
        for (int k = 0; k < L; ++k)
            for (int v = 0; v < VW; ++v) {
                const int64_t m = m0 + (int64_t)v * L + k;
                if (m >= mend) continue;
                for (int c = 0; c < C; ++c) {
                    const size_t i = (size_t)c * blk + (size_t)k * VW + v;
                    if (x->s16) store_i32(x, o, out_idx(x, m - x->ob, c), acci[i]);
                    else store_f32(x, o, out_idx(x, m - x->ob, c), accf[i]);
                }
            }
    }
out:
    free(xt);
    free(r);
    free(accf);
    free(gb);
}

/* ---- mixes without resampling (L == M): one item = mix b, frames [o0, o1) */
static void item_direct(void *vctx, int64_t item)
{
    MixCtx *x = vctx;
    const XmhMixJob *j = x->j;
    const int C = x->C, nt = j->n_tracks;
    const int64_t b = item / x->items_per_mix, q = item % x->items_per_mix;
    const int64_t o0 = q * x->per_item, o1 = o0 + x->per_item < x->fo ? o0 + x->per_item : x->fo;
    const int64_t n = o1 - o0;
    float *accf = malloc(sizeof(float) * (size_t)(n * C));
    float *xs = malloc(sizeof(float) * (size_t)n);
    if (!accf || !xs) {
        x->rc = XM_ENOMEM_;
        free(accf);
        free(xs);
        return;
    }
    int32_t *acci = (int32_t *)accf;
    memset(accf, 0, sizeof(float) * (size_t)(n * C));
    for (int tr = 0; tr < nt; ++tr) {
        const void *trk = track_ptr(j, b, tr, x->in_elem);
        const XmhGain *g = &j->gains[tr];
        const int64_t m0 = x->ob + o0;   /* absolute frame: gains; input frame m reads row m - in_base */
        const int konst = xmc_gain_const(g, m0, m0 + n - 1);
        for (int c = 0; c < C; ++c) {
            load_run(x, trk, m0, (int)n, c, xs, 1);   /* the sample as the mix sees it (s16: its integer value) */
            if (x->s16) {
                const int32_t g1 = xmc_gain_q15(g, m0);
                for (int64_t i = 0; i < n; ++i)
                    acci[i * C + c] += xmc_q15_term((int32_t)xs[i], konst ? g1 : xmc_gain_q15(g, m0 + i));
            } else if (konst) {
                const float g1 = xmc_gain_f32(g, m0);
                for (int64_t i = 0; i < n; ++i) accf[i * C + c] = accf[i * C + c] + g1 * xs[i];
            } else {
                for (int64_t i = 0; i < n; ++i) accf[i * C + c] = accf[i * C + c] + xmc_gain_f32(g, m0 + i) * xs[i];
            }
        }
    }
    void *o = out_ptr(j, b, x->out_elem);
    for (int64_t i = 0; i < n; ++i)
        for (int c = 0; c < C; ++c) {
            if (x->s16) store_i32(x, o, out_idx(x, o0 + i, c), acci[i * C + c]);
            else store_f32(x, o, out_idx(x, o0 + i, c), accf[i * C + c]);
        }
    free(accf);
    free(xs);
}

int xmc_launch_mix(const XmhMixJob *j, void *stream, int *n_launches, int *n_fast)
{
    (void)stream;
    (void)n_fast;   /* no fused kernel on the CPU */
    if (j->frames_out == 0 || j->n_mix == 0) return 0;
    if (j->channels != 1 && j->channels != 2) return XM_EINVAL_;
    const int s16 = j->fmt == 1;
    if (j->partial && (!s16 || j->out_conv)) return XM_EINVAL_;   /* partials are the s16 (Q15) mix */
    if ((j->in_base || j->out_base) && j->io_flags) return XM_EINVAL_;   /* layouts / conversion: whole clips */
    MixCtx x;
    memset(&x, 0, sizeof x);
    x.j = j;
    x.C = j->channels;
    x.s16 = s16;
    x.in_conv = (j->io_flags & XMH_IO_IN_CONV) != 0;
    x.in_planar = (j->io_flags & XMH_IO_IN_PLANAR) != 0 && x.C == 2;
    x.out_planar = (j->io_flags & XMH_IO_OUT_PLANAR) != 0 && x.C == 2;
    x.in_elem = (x.in_conv != s16) ? 2 : 4;
    x.out_elem = j->partial ? 4 : s16 ? (j->out_conv == 2 ? 4 : 2) : (j->out_conv == 1 ? 2 : 4);
    x.N = j->frames_in;
    x.ob = j->out_base;
    x.ib = j->in_base;
    x.fo = j->frames_out;
    x.resample = j->rs.L != j->rs.M;
    int rc = 0;
    if (x.resample) {
        x.L = j->rs.L;
        x.M = j->rs.M;
        x.T = j->rs.T;
        x.rm = j->rs.rm;
        const int L = x.L;
        x.ph = malloc(sizeof(int32_t) * (size_t)L);
        x.jb = malloc(sizeof(int32_t) * (size_t)L);
        if (!x.ph || !x.jb) {
            free(x.ph);
            free(x.jb);
            return XM_ENOMEM_;
        }
        /* chunks start at ob + multiples of L*VW: output k of every chunk has
         * the phase and window offset of output ob + k of the first one */
        const int64_t J0 = ((x.ob + x.rm) * x.M) / L - x.T + 1;
        for (int k = 0; k < L; ++k) {
            const int64_t Mx = (x.ob + k + x.rm) * x.M;
            x.ph[k] = (int32_t)(Mx % L);
            x.jb[k] = (int32_t)(Mx / L - x.T + 1 - J0);
        }
        x.F = x.jb[L - 1] + x.T;
        const int64_t blk = (int64_t)L * VW;
        int64_t nblk = (32768 + blk - 1) / blk;   /* ~32k outputs per item */
        x.per_item = nblk * blk;
        x.items_per_mix = (x.fo + x.per_item - 1) / x.per_item;
        rc = xmc_parallel((int64_t)j->n_mix * x.items_per_mix, item_resample, &x);
        free(x.ph);
        free(x.jb);
    } else {
        x.per_item = 65536;
        x.items_per_mix = (x.fo + x.per_item - 1) / x.per_item;
        rc = xmc_parallel((int64_t)j->n_mix * x.items_per_mix, item_direct, &x);
    }
    if (n_launches) *n_launches += 1;
    return rc ? rc : x.rc;
}

/* ---- timeline mix: placed (already resampled) tracks ---------------------- */
typedef struct {
    const XmhMixJob *j;
    int64_t per_item, items_per_mix;
} PlaceCtx;

static void item_placed(void *vctx, int64_t item)
{
    const PlaceCtx *p = vctx;
    const XmhMixJob *j = p->j;
    const int C = j->channels, s16 = j->fmt == 1;
    const int64_t b = item / p->items_per_mix, q = item % p->items_per_mix;
    const int64_t m0 = q * p->per_item, m1 = m0 + p->per_item < j->frames_out ? m0 + p->per_item : j->frames_out;
    const int out_elem = s16 ? (j->out_conv == 2 ? 4 : 2) : (j->out_conv == 1 ? 2 : 4);
    void *o = out_ptr(j, b, out_elem);
    for (int64_t m = m0; m < m1; ++m)
        for (int c = 0; c < C; ++c) {
            int32_t acci = 0;
            float accf = 0.0f;
            for (int tr = 0; tr < j->n_tracks; ++tr) {
                const int64_t tf = m - j->place[2 * tr], len = j->place[2 * tr + 1];
                if (tf < 0 || tf >= len) continue;   /* a +-0 term: leaves the sum (up to the final +0) */
                const void *xp = j->in_ptrs[b * j->n_tracks + tr];
                if (s16) acci += xmc_q15_term(((const int16_t *)xp)[tf * C + c], xmc_gain_q15(&j->gains[tr], m));
                else accf = accf + xmc_gain_f32(&j->gains[tr], m) * ((const float *)xp)[tf * C + c];
            }
            const int64_t i = m * C + c;
            if (s16 && j->out_conv == 2) ((float *)o)[i] = (float)xmc_sat16(acci) * 0x1p-15f;
            else if (s16) ((int16_t *)o)[i] = xmc_sat16(acci);
            else if (j->out_conv == 1) ((int16_t *)o)[i] = (int16_t)xmc_round_sat16(accf * 32768.0f);
            else ((float *)o)[i] = accf + 0.0f;
        }
}

int xmc_launch_mix_placed(const XmhMixJob *j, void *stream, int *n_launches)
{
    (void)stream;
    if (j->frames_out == 0 || j->n_mix == 0) return 0;
    if (!j->place || !j->in_ptrs || (j->channels != 1 && j->channels != 2)) return XM_EINVAL_;
    PlaceCtx p = {j, 65536, (j->frames_out + 65535) / 65536};
    const int rc = xmc_parallel((int64_t)j->n_mix * p.items_per_mix, item_placed, &p);
    if (n_launches) *n_launches += 1;
    return rc;
}

/* ---- config 5 finish: saturate the summed int32 partials, parts in order - */
typedef struct {
    const int32_t *parts;
    int n_parts;
    int64_t part_stride, part_mix_stride, out_mix_stride, samples;
    int16_t *out;
} FinishCtx;

static void item_finish(void *vctx, int64_t b)
{
    const FinishCtx *f = vctx;
    const int32_t *p = f->parts + b * f->part_mix_stride;
    int16_t *y = f->out + b * f->out_mix_stride;
    for (int64_t i = 0; i < f->samples; ++i) {
        int32_t acc = 0;
        for (int q = 0; q < f->n_parts; ++q) acc += p[q * f->part_stride + i];
        y[i] = xmc_sat16(acc);
    }
}

int xmc_launch_finish_s16(const int32_t *parts, int n_parts, int64_t part_stride, int64_t part_mix_stride,
                          int16_t *out, int64_t out_mix_stride, int64_t batch, int64_t samples, void *stream)
{
    (void)stream;
    if (batch <= 0 || samples <= 0) return 0;
    FinishCtx f = {parts, n_parts, part_stride, part_mix_stride, out_mix_stride, samples, out};
    return xmc_parallel(batch, item_finish, &f);
}
