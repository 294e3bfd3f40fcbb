/*
 * xm_cpu_fx.c — the CPU backend's effects jobs (SURVEY.md §8(a) a8, a10;
 * include/xm_effects.h): the biquad cascade in scipy sosfilt's transposed
 * direct form II order and the FIR in upfirdn's order, both separately
 * rounded fp32, bit for bit the gfx950 kernels (csrc/xm_fx.hip).
 *
 *  - Biquad: the recurrence is serial in time, so the vector lanes are
 *    independent chains: up to 16 (clip, channel) streams of one job filtered
 *    together, each lane the scalar recurrence
 *        o = b0*x + z0;  z0 = (b1*x - a1*o) + z1;  z1 = b2*x - a2*o;  x = o
 *    for every section in order.  Streams are staged in 256-frame tiles.
 *  - FIR: lanes are 16 consecutive output samples of one clip (both channels
 *    of interleaved stereo ride along: tap t reads C*t samples back), each the
 *    chain acc = +0; acc = acc + x[n-K+1+t]*h[K-1-t] over t ascending.
 */
#include <stdlib.h>
#include <string.h>

#include "xm_cpu.h"

#define VW 16
typedef float v16f __attribute__((vector_size(64)));
typedef float v16fu __attribute__((vector_size(64), aligned(4)));   /* unaligned loads */

#if defined(__x86_64__) && !defined(__SANITIZE_ADDRESS__)
#define XMC_SIMD __attribute__((target_clones("avx512f", "avx2", "default")))
#else
#define XMC_SIMD
#endif

#define XM_EINVAL_ (-22)
#define XM_ENOMEM_ (-12)

/* ---- biquad cascade ------------------------------------------------------ */
#define BQ_TILE 256

typedef struct {
    const XmhFxJob *j;
    int lanes_per_group;   /* 16 mono clips or 8 stereo clips per group */
    int rc;
} BqCtx;

XMC_SIMD static void bq_tile(float *restrict xt, int n, const float *restrict sos, int ns, v16f *restrict z0,
                             v16f *restrict z1)
{
    v16f *x = (v16f *)xt;
    for (int i = 0; i < n; ++i) {
        v16f v = x[i];
        for (int s = 0; s < ns; ++s) {
            const float *q = sos + 6 * s;
            const v16f o = q[0] * v + z0[s];
            z0[s] = (q[1] * v - q[4] * o) + z1[s];
            z1[s] = q[2] * v - q[5] * o;
            v = o;
        }
        x[i] = v;
    }
}

static void item_biquad(void *vctx, int64_t grp)
{
    BqCtx *b = vctx;
    const XmhFxJob *j = b->j;
    const int C = j->channels, ns = j->n_sos, per = b->lanes_per_group / C;
    const int64_t k0 = grp * per;
    const int nk = (int)(j->n_clips - k0 < per ? j->n_clips - k0 : per);
    v16f *z0 = aligned_alloc(64, sizeof(v16f) * (size_t)ns), *z1 = aligned_alloc(64, sizeof(v16f) * (size_t)ns);
    float *xt = aligned_alloc(64, sizeof(float) * BQ_TILE * VW);
    if (!z0 || !z1 || !xt) {
        b->rc = XM_ENOMEM_;
        goto out;
    }
    memset(z0, 0, sizeof(v16f) * (size_t)ns);
    memset(z1, 0, sizeof(v16f) * (size_t)ns);
    memset(xt, 0, sizeof(float) * BQ_TILE * VW);   /* idle lanes filter zeros */
    if (j->state)   /* state[clip][section][z0, z1][channel] */
        for (int q = 0; q < nk; ++q)
            for (int s = 0; s < ns; ++s)
                for (int c = 0; c < C; ++c) {
                    const float *st = j->state + (((size_t)(k0 + q) * ns + s) * 2) * C;
                    z0[s][q * C + c] = st[c];
                    z1[s][q * C + c] = st[C + c];
                }
    for (int64_t f0 = 0; f0 < j->frames; f0 += BQ_TILE) {
        const int n = (int)(j->frames - f0 < BQ_TILE ? j->frames - f0 : BQ_TILE);
        for (int q = 0; q < nk; ++q) {
            const float *src = j->in_ptrs[k0 + q] + f0 * C;
            for (int i = 0; i < n; ++i)
                for (int c = 0; c < C; ++c) xt[i * VW + q * C + c] = src[i * C + c];
        }
        bq_tile(xt, n, j->sos, ns, z0, z1);
        for (int q = 0; q < nk; ++q) {
            float *dst = j->out_ptrs[k0 + q] + f0 * C;   /* in place allowed: the tile was read first */
            for (int i = 0; i < n; ++i)
                for (int c = 0; c < C; ++c) dst[i * C + c] = xt[i * VW + q * C + c];
        }
    }
    if (j->state)
        for (int q = 0; q < nk; ++q)
            for (int s = 0; s < ns; ++s)
                for (int c = 0; c < C; ++c) {
                    float *st = j->state + (((size_t)(k0 + q) * ns + s) * 2) * C;
                    st[c] = z0[s][q * C + c];
                    st[C + c] = z1[s][q * C + c];
                }
out:
    free(z0);
    free(z1);
    free(xt);
}

/* ---- FIR ----------------------------------------------------------------- */
#define FIR_TILE 8192   /* output frames per item */

typedef struct {
    const XmhFxJob *j;
    int64_t tiles;
    int rc;
} FirCtx;

/* y[i] = sum over t ascending (from +0) of e[i + C*t] * hr[t], i < n (a multiple of VW);
 * hr = the taps reversed (hr[t] = h[K-1-t]) */
XMC_SIMD static void fir_tile(float *restrict y, const float *restrict e, const float *restrict hr, int K, int C,
                              int n)
{
    int i = 0;
    for (; i + 4 * VW <= n; i += 4 * VW) {
        v16f a0 = {0}, a1 = {0}, a2 = {0}, a3 = {0};
        for (int t = 0; t < K; ++t) {
            const float *p = e + i + (size_t)t * C;
            a0 = a0 + *(const v16fu *)p * hr[t];
            a1 = a1 + *(const v16fu *)(p + VW) * hr[t];
            a2 = a2 + *(const v16fu *)(p + 2 * VW) * hr[t];
            a3 = a3 + *(const v16fu *)(p + 3 * VW) * hr[t];
        }
        *(v16fu *)(y + i) = a0;
        *(v16fu *)(y + i + VW) = a1;
        *(v16fu *)(y + i + 2 * VW) = a2;
        *(v16fu *)(y + i + 3 * VW) = a3;
    }
    for (; i < n; i += VW) {
        v16f a0 = {0};
        for (int t = 0; t < K; ++t) a0 = a0 + *(const v16fu *)(e + i + (size_t)t * C) * hr[t];
        *(v16fu *)(y + i) = a0;
    }
}

static void item_fir(void *vctx, int64_t item)
{
    FirCtx *fc = vctx;
    const XmhFxJob *j = fc->j;
    const int C = j->channels, K = j->fir_len;
    const int64_t k = item / fc->tiles, f0 = (item % fc->tiles) * FIR_TILE;
    const int64_t f1 = f0 + FIR_TILE < j->frames ? f0 + FIR_TILE : j->frames;
    const int n = (int)((f1 - f0) * C), npad = (n + VW - 1) / VW * VW;
    const int64_t h = (int64_t)(K - 1) * C;   /* history samples before the tile */
    float *e = malloc(sizeof(float) * (size_t)(h + npad + VW));
    float *y = malloc(sizeof(float) * (size_t)npad);
    float *hr = malloc(sizeof(float) * (size_t)K);
    if (!e || !y || !hr) {
        fc->rc = XM_ENOMEM_;
        goto out;
    }
    for (int t = 0; t < K; ++t) hr[t] = j->fir[K - 1 - t];
    const float *x = j->in_ptrs[k];
    /* e[s] = input sample f0*C - h + s; negative frames from the carried
     * history (streaming) or zero */
    for (int64_t s = 0; s < h; ++s) {
        const int64_t a = f0 * C - h + s;
        if (a >= 0) e[s] = x[a];
        else e[s] = j->hist_in ? j->hist_in[(int64_t)k * h + (h + a)] : 0.0f;
    }
    memcpy(e + h, x + f0 * C, sizeof(float) * (size_t)n);
    memset(e + h + n, 0, sizeof(float) * (size_t)(npad - n + VW));
    fir_tile(y, e, hr, K, C, npad);
    memcpy(j->out_ptrs[k] + f0 * C, y, sizeof(float) * (size_t)n);
out:
    free(e);
    free(y);
    free(hr);
}

typedef struct {
    const XmhFxJob *j;
} HistCtx;

/* the K-1 frames before the next block: the last K-1 of (history ++ block) */
static void item_fir_hist(void *vctx, int64_t k)
{
    const XmhFxJob *j = ((const HistCtx *)vctx)->j;
    const int64_t C = j->channels, h = (int64_t)(j->fir_len - 1) * C, n = j->frames * C;
    const float *x = j->in_ptrs[k];
    for (int64_t s = 0; s < h; ++s) {
        const int64_t a = n - h + s;   /* sample of (history ++ block), block-relative */
        j->hist_out[k * h + s] = a >= 0 ? x[a] : j->hist_in[k * h + (h + a)];
    }
}

int xmc_launch_fx(const XmhFxJob *j, void *stream, int *n_launches)
{
    (void)stream;
    if (j->n_clips <= 0 || j->frames <= 0) return 0;
    if (j->channels != 1 && j->channels != 2) return XM_EINVAL_;
    int rc;
    if (j->n_sos > 0) {
        BqCtx b = {j, VW, 0};
        const int per = VW / j->channels;
        rc = xmc_parallel((j->n_clips + per - 1) / per, item_biquad, &b);
        if (!rc) rc = b.rc;
    } else if (j->fir_len > 0) {
        const int K = j->fir_len;
        if (j->hist_in && K > 1 && (!j->hist_out || j->hist_out == j->hist_in)) return XM_EINVAL_;
        for (int k = 0; k < j->n_clips; ++k)
            if (j->in_ptrs[k] == j->out_ptrs[k]) return XM_EINVAL_;   /* the host never runs a FIR in place */
        FirCtx f = {j, (j->frames + FIR_TILE - 1) / FIR_TILE, 0};
        rc = xmc_parallel((int64_t)j->n_clips * f.tiles, item_fir, &f);
        if (!rc) rc = f.rc;
        if (!rc && j->hist_in && K > 1) {
            HistCtx hc = {j};
            rc = xmc_parallel(j->n_clips, item_fir_hist, &hc);
        }
    } else {
        return 0;
    }
    if (n_launches) *n_launches += 1;
    return rc;
}
