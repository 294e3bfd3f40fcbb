/*
 * xm_oracle.c — C restatement of the PCM hot path.  TEST INFRASTRUCTURE ONLY
 * (see xm_oracle.h).  Build: oracle/Makefile, -O2 -ffp-contract=off -fopenmp.
 *
 * Each routine restates the scipy 1.15.3 float32 algorithm named beside it;
 * the numpy twin is oracle/np_oracle.py and both are pinned to the committed
 * scipy golden vectors (tests/golden/, tools/gen_golden.py).
 */
#include "xm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif


/* ---- synthetic PCM (numpy twin np_oracle.gen_*) ---- */
static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static inline uint64_t gen_bits(uint64_t seed, uint64_t clip, uint64_t i)
{
    return mix64(seed + ((clip << 32) | i) * 0x9E3779B97F4A7C15ULL);
}

void xo_gen_f32(uint64_t seed, uint64_t clip, int channels, size_t frames, float *out)
{
    size_t n = frames * (size_t)channels;
    for (size_t i = 0; i < n; ++i) {
        int32_t v = (int32_t)(gen_bits(seed, clip, i) >> 40) - (1 << 23);
        out[i] = (float)v * 0x1p-23f;
    }
}

void xo_gen_s16(uint64_t seed, uint64_t clip, int channels, size_t frames, int16_t *out)
{
    size_t n = frames * (size_t)channels;
    for (size_t i = 0; i < n; ++i)
        out[i] = (int16_t)(uint16_t)(gen_bits(seed, clip, i) >> 48);
}

/* ---- resampler: scipy _signaltools.py:3686-3759 + _upfirdn.py ---------- */
size_t xo_resample_out_frames(size_t n, int L, int M)
{
    return (n * (size_t)L + (size_t)M - 1) / (size_t)M;
}

void xo_resample_f32(const float *H, int L, int M, int T, int rm,
                     const float *x, size_t N, int C, float *y)
{
    size_t nout = xo_resample_out_frames(N, L, M);
    for (size_t m = 0; m < nout; ++m) {
        int64_t Mx = ((int64_t)m + rm) * M;
        int64_t ph = Mx % L;
        int64_t j0 = Mx / L - T + 1;
        const float *h = H + ph * T;
        for (int c = 0; c < C; ++c) {
            float acc = 0.0f;
            for (int t = 0; t < T; ++t) {
                int64_t j = j0 + t;
                if (j >= 0 && j < (int64_t)N)
                    acc = acc + x[j * C + c] * h[t];
            }
            y[m * C + c] = acc;
        }
    }
}

static inline int16_t sat16(int64_t v)
{
    return (int16_t)(v < -32768 ? -32768 : v > 32767 ? 32767 : v);
}

void xo_resample_s16(const float *H, int L, int M, int T, int rm,
                     const int16_t *x, size_t N, int C, int16_t *y)
{
    size_t nout = xo_resample_out_frames(N, L, M);
    float *xf = malloc((N * C + 1) * sizeof(float));
    float *yf = malloc((nout * C + 1) * sizeof(float));
    for (size_t i = 0; i < N * (size_t)C; ++i) xf[i] = (float)x[i];
    xo_resample_f32(H, L, M, T, rm, xf, N, C, yf);
    for (size_t i = 0; i < nout * (size_t)C; ++i) y[i] = sat16(lrintf(yf[i]));
    free(xf);
    free(yf);
}

/* ---- gains (contract: include/xm_audio_common.h) ----------------------- */
float xo_gain_f32(const XmGainRamp *r, int64_t n)
{
    int xf = r->mode == XM_GAIN_XFADE_OUT;
    float g0 = xf ? 0.0f : r->gain0, g1 = xf ? 1.0f : r->gain1, g;
    if (r->ramp_len == 0) {
        g = n >= r->ramp_start ? g1 : g0;
    } else {
        int64_t k = n - r->ramp_start;
        k = k < 0 ? 0 : k > r->ramp_len ? r->ramp_len : k;
        float step = (g1 - g0) / (float)r->ramp_len;
        g = g0 + step * (float)k;
    }
    return xf ? 1.0f - g : g;
}

int32_t xo_gain_q15(const XmGainRamp *r, int64_t n)
{
    int xf = r->mode == XM_GAIN_XFADE_OUT;
    int64_t g0 = xf ? 0 : r->gain0_q15, g1 = xf ? 32768 : r->gain1_q15, g;
    if (r->ramp_len == 0) {
        g = n >= r->ramp_start ? g1 : g0;
    } else {
        int64_t k = n - r->ramp_start;
        k = k < 0 ? 0 : k > r->ramp_len ? r->ramp_len : k;
        g = g0 + ((g1 - g0) * k) / r->ramp_len;
    }
    return (int32_t)(xf ? 32768 - g : g);
}

/* ---- mix ------------------------------------------------------------- */
void xo_mix_f32(const float *const *r, const XmGainRamp *g, int ntr, size_t F, int C, float *out)
{
    for (size_t n = 0; n < F; ++n) {
        float gv[64];
        for (int tr = 0; tr < ntr; ++tr) gv[tr] = xo_gain_f32(&g[tr], (int64_t)n);
        for (int c = 0; c < C; ++c) {
            float acc = 0.0f;
            for (int tr = 0; tr < ntr; ++tr) acc = acc + gv[tr] * r[tr][n * C + c];
            out[n * C + c] = acc;
        }
    }
}

void xo_mix_s16(const int16_t *const *s, const XmGainRamp *g, int ntr, size_t F, int C, int16_t *out)
{
    for (size_t n = 0; n < F; ++n) {
        int32_t gv[64];
        for (int tr = 0; tr < ntr; ++tr) gv[tr] = xo_gain_q15(&g[tr], (int64_t)n);
        for (int c = 0; c < C; ++c) {
            int32_t acc = 0;
            for (int tr = 0; tr < ntr; ++tr)
                acc += ((int32_t)s[tr][n * C + c] * gv[tr] + 16384) >> 15;
            out[n * C + c] = sat16(acc);
        }
    }
}

void xo_resample_mix_f32(const float *H, int L, int M, int T, int rm,
                         const float *const *x, const XmGainRamp *g, int ntr,
                         size_t N, int C, float *out)
{
    size_t F = xo_resample_out_frames(N, L, M);
    float *buf = malloc((F * C * (size_t)ntr + 1) * sizeof(float));
    const float *r[64];
    for (int tr = 0; tr < ntr; ++tr) {
        xo_resample_f32(H, L, M, T, rm, x[tr], N, C, buf + (size_t)tr * F * C);
        r[tr] = buf + (size_t)tr * F * C;
    }
    xo_mix_f32(r, g, ntr, F, C, out);
    free(buf);
}

void xo_resample_mix_s16(const float *H, int L, int M, int T, int rm,
                         const int16_t *const *x, const XmGainRamp *g, int ntr,
                         size_t N, int C, int16_t *out)
{
    size_t F = xo_resample_out_frames(N, L, M);
    int16_t *buf = malloc((F * C * (size_t)ntr + 1) * sizeof(int16_t));
    const int16_t *r[64];
    for (int tr = 0; tr < ntr; ++tr) {
        xo_resample_s16(H, L, M, T, rm, x[tr], N, C, buf + (size_t)tr * F * C);
        r[tr] = buf + (size_t)tr * F * C;
    }
    xo_mix_s16(r, g, ntr, F, C, out);
    free(buf);
}

/* ---- effects: scipy sosfilt (TDF-II) and upfirdn order --------------- */
void xo_biquad_f32(const float *sos, int nsec, const float *x, size_t N, int C, float *y)
{
    float (*z)[2] = calloc((size_t)(nsec > 0 ? nsec : 1), sizeof *z);   /* any cascade length */
    if (!z) abort();
    for (int c = 0; c < C; ++c) {
        memset(z, 0, sizeof *z * (size_t)(nsec > 0 ? nsec : 1));
        for (size_t n = 0; n < N; ++n) {
            float v = x[n * C + c];
            for (int s = 0; s < nsec; ++s) {
                const float *q = sos + 6 * s;
                float o = q[0] * v + z[s][0];
                z[s][0] = (q[1] * v - q[4] * o) + z[s][1];
                z[s][1] = q[2] * v - q[5] * o;
                v = o;
            }
            y[n * C + c] = v;
        }
    }
    free(z);
}

void xo_fir_f32(const float *h, int K, const float *x, size_t N, int C, float *y)
{
    for (size_t n = 0; n < N; ++n)
        for (int c = 0; c < C; ++c) {
            float acc = 0.0f;
            for (int t = 0; t < K; ++t) {
                int64_t j = (int64_t)n - K + 1 + t;
                if (j >= 0) acc = acc + x[j * C + c] * h[K - 1 - t];
            }
            y[n * C + c] = acc;
        }
}

/* ---- CPU-baseline batch drivers (OpenMP over mixes) ------------------- */
int xo_batch_resample_mix_f32(const float *H, int L, int M, int T, int rm,
                              const float *in, const XmGainRamp *g, int ntr,
                              size_t nmix, size_t N, int C, float *out, int threads)
{
    size_t F = xo_resample_out_frames(N, L, M);
    int used = 1;
#ifdef _OPENMP
    if (threads < 1) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
    for (long b = 0; b < (long)nmix; ++b) {
        const float *x[64];
        for (int tr = 0; tr < ntr; ++tr) x[tr] = in + ((size_t)b * ntr + tr) * N * C;
        xo_resample_mix_f32(H, L, M, T, rm, x, g, ntr, N, C, out + (size_t)b * F * C);
#ifdef _OPENMP
        if (b == 0) used = omp_get_num_threads();
#endif
    }
    return used;
}

int xo_batch_mix_s16(const int16_t *in, const XmGainRamp *g, int ntr, size_t nmix,
                     size_t F, int C, int16_t *out, int threads)
{
    int used = 1;
#ifdef _OPENMP
    if (threads < 1) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
    for (long b = 0; b < (long)nmix; ++b) {
        const int16_t *s[64];
        for (int tr = 0; tr < ntr; ++tr) s[tr] = in + ((size_t)b * ntr + tr) * F * C;
        xo_mix_s16(s, g, ntr, F, C, out + (size_t)b * F * C);
#ifdef _OPENMP
        if (b == 0) used = omp_get_num_threads();
#endif
    }
    return used;
}
