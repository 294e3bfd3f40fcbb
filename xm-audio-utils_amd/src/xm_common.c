/*
 * xm_common.c — status strings, version, rate-pair design and gain
 * descriptors for the C host layer (SURVEY.md §1 layer L2).
 *
 * The filter design itself lives in xm_design.c (device-free, so the build
 * can also bake the 147/160 table into the fast kernel).
 */
#include <stdlib.h>
#include <string.h>

#include "xm_internal.h"

const char *xm_strerror(int status)
{
    switch (status) {
    case XM_OK: return "ok";
    case XM_EINVAL: return "invalid argument";
    case XM_ENOMEM: return "out of memory";
    case XM_EDEVICE: return "HIP device error (no usable MI355X / gfx950 device or runtime failure)";
    case XM_ECOMM: return "cross-device communication error";
    case XM_ENOSYS: return "not supported by this build";
    default: return "unknown error";
    }
}

const char *xm_version(void) { return "xm-audio-mi355x 0.1.0 (gfx950)"; }

int xm_device_count(void) { return xmh_device_count(); }

int xm_table_build(XmTable *t, int in_rate, int out_rate)
{
    memset(t, 0, sizeof *t);
    int rc = xm_resample_design(in_rate, out_rate, &t->d, NULL);
    if (rc) return rc;
    size_t n = (size_t)t->d.L * (size_t)t->d.T;
    float *H = malloc(n * sizeof(float));
    if (!H) return XM_ENOMEM;
    rc = xm_resample_design(in_rate, out_rate, &t->d, H);
    if (!rc) rc = xmh_malloc((void **)&t->H_dev, n * sizeof(float));
    if (!rc) rc = xmh_memcpy_h2d(t->H_dev, H, n * sizeof(float), NULL);
    /* specialised 48k->44.1k kernel (csrc/xm_resample_fast.hip): only if its
     * baked coefficients are this very table */
    t->fast = !rc && xmh_fast_table_check(H, t->d.L, t->d.M, t->d.T) == 0;
    if (!rc) rc = xmh_stream_sync(NULL);
    free(H);
    if (rc) xm_table_free(t);
    return rc;
}

void xm_table_free(XmTable *t)
{
    xmh_free(t->H_dev);
    t->H_dev = NULL;
    t->fast = 0;
}

int xm_gain_to_dev(const XmGainRamp *g, XmhGain *d)
{
    memset(d, 0, sizeof *d);
    if (g->ramp_len < 0 || g->ramp_len >= (1 << 24)) return XM_EINVAL;
    if (g->mode != XM_GAIN_RAMP && g->mode != XM_GAIN_XFADE_OUT) return XM_EINVAL;
    int xf = g->mode == XM_GAIN_XFADE_OUT;
    if (!xf && (g->gain0_q15 < 0 || g->gain0_q15 > 65535 || g->gain1_q15 < 0 || g->gain1_q15 > 65535))
        return XM_EINVAL;
    d->g0 = xf ? 0.0f : g->gain0;
    d->g1 = xf ? 1.0f : g->gain1;
    d->q0 = xf ? 0 : g->gain0_q15;
    d->q1 = xf ? 32768 : g->gain1_q15;
    d->len = (int32_t)g->ramp_len;
    d->start = g->ramp_start;
    d->flags = xf ? (int32_t)XMH_GAIN_XFADE_OUT : 0;
    /* fp32 step exactly as the contract: (g1 - g0) / (float)len, no contraction */
    d->step = d->len ? (d->g1 - d->g0) / (float)d->len : 0.0f;
    return XM_OK;
}

int xm_synth_pcm(void *dst, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips, int channels,
                 int64_t frames, int device, void *stream)
{
    if (!dst || (fmt != XM_FMT_S16 && fmt != XM_FMT_F32) || n_clips < 0 || frames < 0 ||
        (channels != 1 && channels != 2) || (device < 0 && device != XM_DEVICE_CPU))
        return XM_EINVAL;
    if (device != XM_DEVICE_CPU && device >= xmh_device_count()) return XM_EDEVICE;
    int rc = xmh_set_device(device);
    if (!rc) rc = xmh_synth(dst, fmt, seed, clip0, n_clips, channels, frames, stream);
    if (!rc && !stream) rc = xmh_stream_sync(NULL);
    return rc;
}
