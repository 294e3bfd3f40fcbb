/*
 * xm_design.c — xm_resample_design(): a C restatement of the float64 filter
 * design scipy 1.15.3 resample_poly performs before casting to float32
 * (scipy/signal/_signaltools.py:3697-3726 -> _fir_filter_design.py firwin ->
 * windows.kaiser -> special.i0 (Cephes) and numpy's pairwise np.sum), so any
 * rate pair gets a scipy-identical fp32 table at create time.  tests/
 * test_abi.py pins the result bit-for-bit against scipy's tables committed in
 * tests/golden/tables.npz for every rate pair there.
 *
 * Device-free on purpose: tools/gen_coefs.c links this file at build time to
 * bake the 48k->44.1k table into csrc/xm_resample_fast.hip as instruction
 * literals, and the library re-checks the two agree before using that kernel.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "xm_audio_common.h"

/* ---- Cephes i0 (scipy.special.i0 / numpy.i0): Chebyshev expansions ------- */
static const double I0_A[30] = {
    -4.4153416464793395e-18, 3.3307945188222384e-17, -2.431279846547955e-16, 1.715391285555133e-15,
    -1.1685332877993451e-14, 7.676185498604936e-14, -4.856446783111929e-13, 2.95505266312964e-12,
    -1.726826291441556e-11, 9.675809035373237e-11, -5.189795601635263e-10, 2.6598237246823866e-09,
    -1.300025009986248e-08, 6.046995022541919e-08, -2.670793853940612e-07, 1.1173875391201037e-06,
    -4.4167383584587505e-06, 1.6448448070728896e-05, -5.754195010082104e-05, 0.00018850288509584165,
    -0.0005763755745385824, 0.0016394756169413357, -0.004324309995050576, 0.010546460394594998,
    -0.02373741480589947, 0.04930528423967071, -0.09490109704804764, 0.17162090152220877,
    -0.3046826723431984, 0.6767952744094761};
static const double I0_B[25] = {
    -7.233180487874754e-18, -4.830504485944182e-18, 4.46562142029676e-17, 3.461222867697461e-17,
    -2.8276239805165836e-16, -3.425485619677219e-16, 1.7725601330565263e-15, 3.8116806693526224e-15,
    -9.554846698828307e-15, -4.150569347287222e-14, 1.54008621752141e-14, 3.8527783827421426e-13,
    7.180124451383666e-13, -1.7941785315068062e-12, -1.3215811840447713e-11, -3.1499165279632416e-11,
    1.1889147107846439e-11, 4.94060238822497e-10, 3.3962320257083865e-09, 2.266668990498178e-08,
    2.0489185894690638e-07, 2.8913705208347567e-06, 6.889758346916825e-05, 0.0033691164782556943,
    0.8044904110141088};

static double chbevl(double x, const double *a, int n)
{
    double b0 = a[0], b1 = 0.0, b2 = 0.0;
    for (int i = 1; i < n; ++i) {
        b2 = b1;
        b1 = b0;
        b0 = x * b1 - b2 + a[i];
    }
    return 0.5 * (b0 - b2);
}

static double bessel_i0(double x)
{
    if (x < 0) x = -x;
    if (x <= 8.0) return exp(x) * chbevl(x / 2.0 - 2.0, I0_A, 30);
    return exp(x) * chbevl(32.0 / x - 2.0, I0_B, 25) / sqrt(x);
}

/* numpy DOUBLE_pairwise_sum (blocks of 8, PW_BLOCKSIZE 128). */
static double pairwise_sum(const double *a, size_t n)
{
    if (n < 8) {
        double res = 0.0;
        for (size_t i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        size_t i;
        for (int k = 0; k < 8; ++k) r[k] = a[k];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    size_t n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

/* np.sum of a 1-D contiguous float64 array: a[0] + pairwise(a[1:]). */
static double np_sum(const double *a, size_t n)
{
    if (n == 0) return 0.0;
    return a[0] + pairwise_sum(a + 1, n - 1);
}

static long gcd_l(long a, long b)
{
    while (b) {
        long t = a % b;
        a = b;
        b = t;
    }
    return a;
}

size_t xm_resample_out_frames(int in_rate, int out_rate, size_t frames_in)
{
    if (in_rate <= 0 || out_rate <= 0) return 0;
    long g = gcd_l(in_rate, out_rate);
    size_t L = (size_t)(out_rate / g), M = (size_t)(in_rate / g);
    return (frames_in * L + M - 1) / M;
}

int xm_resample_design(int in_rate, int out_rate, XmResampleDesign *d, float *H)
{
    if (!d || in_rate <= 0 || out_rate <= 0) return XM_EINVAL;
    long g = gcd_l(in_rate, out_rate);
    long L = out_rate / g, M = in_rate / g;
    memset(d, 0, sizeof *d);
    d->L = (int32_t)L;
    d->M = (int32_t)M;
    if (L == 1 && M == 1) {           /* identity: no filter (scipy returns x.copy()) */
        d->T = 1;
        if (H) H[0] = 1.0f;
        return XM_OK;
    }
    long mx = L > M ? L : M;
    if (mx > 4096) return XM_ENOSYS;  /* keeps tables < 64 KiB-ish; see DESIGN.md */
    long half = 10 * mx;
    long ntaps = 2 * half + 1;
    long pre = M - half % M;
    long T = (pre + ntaps + L - 1) / L;
    d->T = (int32_t)T;
    d->rm = (int32_t)((half + pre) / M);
    d->half = (int32_t)half;
    d->pre = (int32_t)pre;
    if (!H) return XM_OK;

    double *h = malloc(sizeof(double) * (size_t)ntaps);
    float *hp = calloc((size_t)(L * T), sizeof(float));
    if (!h || !hp) {
        free(h);
        free(hp);
        return XM_ENOMEM;
    }
    /* firwin(ntaps, 1/mx, window=('kaiser', 5.0)) in float64 */
    const double cutoff = 1.0 / (double)mx;
    const double alpha = 0.5 * (double)(ntaps - 1);
    const double beta = 5.0;
    const double i0b = bessel_i0(beta);
    const double pi = 3.141592653589793;
    for (long n = 0; n < ntaps; ++n) {
        double m = (double)n - alpha;
        double x = cutoff * m;
        double y = pi * (x == 0.0 ? 1.0e-20 : x);
        double v = cutoff * (sin(y) / y);
        double r = ((double)n - alpha) / alpha;            /* kaiser: alpha == (M-1)/2 */
        double w = bessel_i0(beta * sqrt(1.0 - r * r)) / i0b;
        h[n] = v * w;
    }
    double s = np_sum(h, (size_t)ntaps);
    for (long n = 0; n < ntaps; ++n) h[n] = h[n] / s;
    /* astype(float32); h *= up  (float32 multiply) ; prepend `pre` zeros */
    for (long n = 0; n < ntaps; ++n) {
        float f = (float)h[n];
        f = f * (float)L;
        hp[pre + n] = f;   /* hp has length L*T >= pre + ntaps */
    }
    /* H[ph][t] = hp[ph + L*(T-1-t)] */
    for (long ph = 0; ph < L; ++ph)
        for (long t = 0; t < T; ++t) {
            long idx = ph + L * (T - 1 - t);
            H[ph * T + t] = idx < pre + ntaps ? hp[idx] : 0.0f;
        }
    free(h);
    free(hp);
    return XM_OK;
}
