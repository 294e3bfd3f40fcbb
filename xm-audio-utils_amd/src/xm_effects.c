/*
 * xm_effects.c — the xm_effects_* C API: chain construction (biquad sections,
 * RBJ EQ bands designed in fp64, FIR taps), staging and dispatch of the
 * gfx950 effects kernels (csrc/xm_fx.hip).  Build-owned API (reference has
 * none: /root/reference/README.md:1); contract in include/xm_effects.h.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "xm_internal.h"

struct XmEffects {
    XmEffectsConfig cfg;
    int n_effects;
    struct {
        int kind;          /* 1 biquad section, 2 FIR */
        int n;             /* taps for FIR */
        float sos[6];
        float *fir;        /* host copy */
    } fx[XM_MAX_EFFECTS];
    XmFxStage stages[XM_MAX_EFFECTS];
    int n_stages;
    int dirty;
    void *own_stream, *stream;
    int user_stream;
    void *d_buf[2];
    size_t d_cap[2];
    void **d_ptrs;
    void **h_ptrs;
    size_t ptr_cap;
    /* streaming state (xm_effects_stream_reset): per stage, biquad
     * [clip][section][z0,z1][ch] in st[s][0]; FIR [clip][K-1][ch] history
     * ping-ponging between st[s][0] and st[s][1] (st_cur[s] = current) */
    float *st[XM_MAX_EFFECTS][2];
    int st_cur[XM_MAX_EFFECTS];
    size_t st_clips;
    int st_ready;
    /* multi-device chain (xm_effects_create_multi / n_devices > 1): one
     * single-device chain per entry of devs, a worker thread per device
     * (src/xm_pool.c); a batch's clips are cut into contiguous blocks, block
     * d on devs[d].  Clips are independent, so the result is the one-device
     * result bit for bit.  The parent keeps the effect list (fx[]) and no
     * device resources of its own. */
    int n_sub;
    int devs[XM_MAX_DEVICES];
    XmEffects *sub[XM_MAX_DEVICES];
    XmPool *pool;
    size_t st_first[XM_MAX_DEVICES], st_cnt[XM_MAX_DEVICES];
};

XmEffects *xm_effects_create_ex(const XmEffectsConfig *cfg, int *status)
{
    int rc = XM_OK;
    XmEffects *e = NULL;
    if (!cfg || cfg->rate <= 0 || (cfg->channels != 1 && cfg->channels != 2) ||
        (cfg->mem_kind != XM_MEM_HOST && cfg->mem_kind != XM_MEM_DEVICE) ||
        (cfg->device < 0 && cfg->device != XM_DEVICE_CPU)) {
        rc = XM_EINVAL;
        goto out;
    }
    if (cfg->device != XM_DEVICE_CPU && cfg->device >= xmh_device_count()) {
        rc = XM_EDEVICE;
        goto out;
    }
    e = calloc(1, sizeof *e);
    if (!e) {
        rc = XM_ENOMEM;
        goto out;
    }
    e->cfg = *cfg;
    if (cfg->device == XM_DEVICE_CPU) e->cfg.mem_kind = XM_MEM_DEVICE;   /* host memory is the CPU's: no staging */
    if ((rc = xmh_set_device(cfg->device))) goto out;
    if ((rc = xmh_stream_create(&e->own_stream))) goto out;
    e->stream = e->own_stream;
out:
    if (rc) xm_effects_freep(&e);
    if (status) *status = rc;
    return e;
}

XmEffects *xm_effects_create_multi(const XmEffectsConfig *cfg, const int *devices, int n_devices, int *status)
{
    int rc = XM_OK;
    XmEffects *e = NULL;
    if (!cfg || !devices || n_devices < 1 || n_devices > XM_MAX_DEVICES || cfg->rate <= 0 ||
        (cfg->channels != 1 && cfg->channels != 2) || (cfg->mem_kind != XM_MEM_HOST && cfg->mem_kind != XM_MEM_DEVICE)) {
        rc = XM_EINVAL;
        goto out;
    }
    for (int d = 0; d < n_devices; ++d)
        if (devices[d] < 0 || devices[d] >= xmh_device_count()) {
            rc = XM_EDEVICE;
            goto out;
        }
    if (n_devices == 1) {   /* one device: the plain single-device chain (set_stream, single-device mixers) */
        XmEffectsConfig c = *cfg;
        c.device = devices[0];
        return xm_effects_create_ex(&c, status);
    }
    e = calloc(1, sizeof *e);
    if (!e) {
        rc = XM_ENOMEM;
        goto out;
    }
    e->cfg = *cfg;
    e->cfg.device = devices[0];
    e->n_sub = n_devices;
    for (int d = 0; d < n_devices && !rc; ++d) {
        XmEffectsConfig c = *cfg;
        c.device = e->devs[d] = devices[d];
        e->sub[d] = xm_effects_create_ex(&c, &rc);
    }
    if (!rc) e->pool = xm_pool_create(n_devices, e, &rc);
out:
    if (rc) xm_effects_freep(&e);
    if (status) *status = rc;
    return e;
}

XmEffects *xm_effects_create(int rate, int channels, int n_devices)
{
    XmEffectsConfig c = {rate, channels, XM_MEM_HOST, 0};
    if (n_devices < 0 || n_devices > XM_MAX_DEVICES) return NULL;
    if (n_devices == 0) c.device = XM_DEVICE_CPU;   /* 0 = the host CPU backend */
    if (n_devices <= 1) return xm_effects_create_ex(&c, NULL);
    int devs[XM_MAX_DEVICES];
    for (int d = 0; d < n_devices; ++d) devs[d] = d;
    return xm_effects_create_multi(&c, devs, n_devices, NULL);
}

int xm_effects_n_devices(const XmEffects *e)
{
    if (!e) return XM_EINVAL;
    return e->n_sub ? e->n_sub : 1;
}

int xm_effects_is_multi(const XmEffects *e) { return e && e->n_sub > 0; }

static void free_stream_state(XmEffects *e)
{
    for (int i = 0; i < XM_MAX_EFFECTS; ++i)
        for (int k = 0; k < 2; ++k) {
            xmh_free(e->st[i][k]);
            e->st[i][k] = NULL;
        }
    e->st_ready = 0;
    e->st_clips = 0;
}

static void free_stages(XmEffects *e)
{
    for (int i = 0; i < e->n_stages; ++i) xmh_free(e->stages[i].coef_dev);
    e->n_stages = 0;
    free_stream_state(e);   /* streams belong to the chain they were started on */
}

void xm_effects_freep(XmEffects **pe)
{
    if (!pe || !*pe) return;
    XmEffects *e = *pe;
    if (e->n_sub) {
        xm_pool_free(&e->pool);
        for (int d = 0; d < e->n_sub; ++d) xm_effects_freep(&e->sub[d]);
        for (int i = 0; i < e->n_effects; ++i) free(e->fx[i].fir);
        free(e);
        *pe = NULL;
        return;
    }
    xmh_set_device(e->cfg.device);
    if (e->own_stream) xmh_stream_sync(e->own_stream);
    free_stages(e);
    free_stream_state(e);
    for (int i = 0; i < e->n_effects; ++i) free(e->fx[i].fir);
    xmh_free(e->d_buf[0]);
    xmh_free(e->d_buf[1]);
    xmh_free(e->d_ptrs);
    xmh_host_free(e->h_ptrs);
    xmh_stream_destroy(e->own_stream);
    free(e);
    *pe = NULL;
}

/* undo the effect just added to sub-chains 0 .. n-1 of a multi-device chain */
static void drop_last(XmEffects *e, int n)
{
    for (int d = 0; d < n; ++d) {
        XmEffects *s = e->sub[d];
        if (s->n_effects == 0) continue;
        s->n_effects--;
        free(s->fx[s->n_effects].fir);
        s->fx[s->n_effects].fir = NULL;
        s->dirty = 1;
    }
}

int xm_effects_add_biquad(XmEffects *e, const float sos[6])
{
    if (!e || !sos) return XM_EINVAL;
    if (sos[3] != 1.0f) return XM_EINVAL;   /* scipy sosfilt requires a0 == 1 */
    for (int i = 0; i < 6; ++i)
        if (!isfinite(sos[i])) return XM_EINVAL;
    if (e->n_effects >= XM_MAX_EFFECTS) return XM_ENOMEM;
    /* a cascade longer than XM_MAX_SOS sections is split by the stager */
    for (int d = 0; d < e->n_sub; ++d) {   /* multi-device: every device's chain */
        const int rc = xm_effects_add_biquad(e->sub[d], sos);
        if (rc) {
            drop_last(e, d);   /* every device keeps the same chain */
            return rc;
        }
    }
    e->fx[e->n_effects].kind = 1;
    memcpy(e->fx[e->n_effects].sos, sos, sizeof(float) * 6);
    e->n_effects++;
    e->dirty = 1;
    return XM_OK;
}

/* RBJ audio-EQ-cookbook (R. Bristow-Johnson), fp64, normalised by a0, cast to
 * fp32.  Mirrored by oracle/np_oracle.py:rbj_section for the parity tests. */
int xm_effects_add_eq_band(XmEffects *e, int band, double f0, double gain_db, double q)
{
    if (!e || f0 <= 0.0 || f0 >= 0.5 * e->cfg.rate || q <= 0.0 || !isfinite(gain_db)) return XM_EINVAL;
    const double A = pow(10.0, gain_db / 40.0);
    const double w0 = 2.0 * 3.141592653589793 * f0 / (double)e->cfg.rate;
    const double cw = cos(w0), sw = sin(w0);
    double alpha, b[3], a[3];
    if (band == XM_EQ_LOWSHELF || band == XM_EQ_HIGHSHELF)
        alpha = sw / 2.0 * sqrt((A + 1.0 / A) * (1.0 / q - 1.0) + 2.0);
    else
        alpha = sw / (2.0 * q);
    switch (band) {
    case XM_EQ_PEAKING:
        b[0] = 1 + alpha * A; b[1] = -2 * cw; b[2] = 1 - alpha * A;
        a[0] = 1 + alpha / A; a[1] = -2 * cw; a[2] = 1 - alpha / A;
        break;
    case XM_EQ_LOWSHELF: {
        const double sa = 2 * sqrt(A) * alpha;
        b[0] = A * ((A + 1) - (A - 1) * cw + sa); b[1] = 2 * A * ((A - 1) - (A + 1) * cw);
        b[2] = A * ((A + 1) - (A - 1) * cw - sa);
        a[0] = (A + 1) + (A - 1) * cw + sa; a[1] = -2 * ((A - 1) + (A + 1) * cw);
        a[2] = (A + 1) + (A - 1) * cw - sa;
        break;
    }
    case XM_EQ_HIGHSHELF: {
        const double sa = 2 * sqrt(A) * alpha;
        b[0] = A * ((A + 1) + (A - 1) * cw + sa); b[1] = -2 * A * ((A - 1) + (A + 1) * cw);
        b[2] = A * ((A + 1) + (A - 1) * cw - sa);
        a[0] = (A + 1) - (A - 1) * cw + sa; a[1] = 2 * ((A - 1) - (A + 1) * cw);
        a[2] = (A + 1) - (A - 1) * cw - sa;
        break;
    }
    case XM_EQ_LOWPASS:
        b[0] = (1 - cw) / 2; b[1] = 1 - cw; b[2] = (1 - cw) / 2;
        a[0] = 1 + alpha; a[1] = -2 * cw; a[2] = 1 - alpha;
        break;
    case XM_EQ_HIGHPASS:
        b[0] = (1 + cw) / 2; b[1] = -(1 + cw); b[2] = (1 + cw) / 2;
        a[0] = 1 + alpha; a[1] = -2 * cw; a[2] = 1 - alpha;
        break;
    default:
        return XM_EINVAL;
    }
    const float sos[6] = {(float)(b[0] / a[0]), (float)(b[1] / a[0]), (float)(b[2] / a[0]), 1.0f,
                          (float)(a[1] / a[0]), (float)(a[2] / a[0])};
    return xm_effects_add_biquad(e, sos);
}

int xm_effects_add_fir(XmEffects *e, const float *h, int K)
{
    if (!e || !h || K < 1 || K > XM_MAX_FIR) return XM_EINVAL;
    if (e->n_effects >= XM_MAX_EFFECTS) return XM_ENOMEM;
    float *c = malloc(sizeof(float) * (size_t)K);   /* the parent's copy first: nothing to undo if it fails */
    if (!c) return XM_ENOMEM;
    for (int d = 0; d < e->n_sub; ++d) {   /* multi-device: every device's chain */
        const int rc = xm_effects_add_fir(e->sub[d], h, K);
        if (rc) {
            drop_last(e, d);   /* every device keeps the same chain */
            free(c);
            return rc;
        }
    }
    memcpy(c, h, sizeof(float) * (size_t)K);
    e->fx[e->n_effects].kind = 2;
    e->fx[e->n_effects].n = K;
    e->fx[e->n_effects].fir = c;
    e->n_effects++;
    e->dirty = 1;
    return XM_OK;
}

int xm_effects_count(const XmEffects *e) { return e ? e->n_effects : XM_EINVAL; }

int xm_effects_get_biquad(const XmEffects *e, int i, float sos[6])
{
    if (!e || !sos || i < 0 || i >= e->n_effects || e->fx[i].kind != 1) return XM_EINVAL;
    memcpy(sos, e->fx[i].sos, sizeof(float) * 6);
    return XM_OK;
}

int xm_effects_set_stream(XmEffects *e, void *s)
{
    if (!e) return XM_EINVAL;
    if (e->n_sub) return XM_ENOSYS;   /* one stream per device, owned by the sub-chains */
    if (e->cfg.device == XM_DEVICE_CPU) return XM_OK;   /* CPU calls are synchronous */
    e->stream = s ? s : e->own_stream;
    e->user_stream = s != NULL;
    return XM_OK;
}

/* the chain's device (XM_DEVICE_CPU for a CPU chain); a multi-device chain has none */
int xm_effects_device(const XmEffects *e) { return e && !e->n_sub ? e->cfg.device : XM_DEVICE_NONE_; }

XmEffects *xm_effects_clone_on(const XmEffects *src, int device, int *status)
{
    XmEffectsConfig c = src->cfg;
    c.device = device;
    int rc = XM_OK;
    XmEffects *e = xm_effects_create_ex(&c, &rc);
    for (int i = 0; e && !rc && i < src->n_effects; ++i)
        rc = src->fx[i].kind == 1 ? xm_effects_add_biquad(e, src->fx[i].sos)
                                  : xm_effects_add_fir(e, src->fx[i].fir, src->fx[i].n);
    if (rc) xm_effects_freep(&e);
    if (status) *status = rc;
    return e;
}

/* Group consecutive biquads into cascades (<= XM_MAX_SOS sections each) and
 * upload coefficients. */
static int build_stages(XmEffects *e)
{
    if (!e->dirty) return XM_OK;
    xmh_set_device(e->cfg.device);
    free_stages(e);
    int rc = XM_OK;
    for (int i = 0; !rc && i < e->n_effects;) {
        XmFxStage *s = &e->stages[e->n_stages];
        if (e->fx[i].kind == 1) {
            float buf[6 * XM_MAX_SOS];
            int n = 0;
            while (i < e->n_effects && e->fx[i].kind == 1 && n < XM_MAX_SOS) {
                memcpy(buf + 6 * n, e->fx[i].sos, sizeof(float) * 6);
                ++n;
                ++i;
            }
            s->kind = 1;
            s->n = n;
            rc = xmh_malloc((void **)&s->coef_dev, sizeof(float) * 6 * (size_t)n);
            if (!rc) rc = xmh_memcpy_h2d(s->coef_dev, buf, sizeof(float) * 6 * (size_t)n, e->stream);
        } else {
            s->kind = 2;
            s->n = e->fx[i].n;
            /* at least 16 floats, zero past the taps: the FIR kernel loads
             * coefficients in 14-tap blocks (csrc/xm_fx.hip k_fir_rb) */
            const size_t nc = s->n < 16 ? 16 : (size_t)s->n;
            float *hc = calloc(nc, sizeof(float));
            if (!hc) rc = XM_ENOMEM;
            if (!rc) {
                memcpy(hc, e->fx[i].fir, sizeof(float) * (size_t)s->n);
                rc = xmh_malloc((void **)&s->coef_dev, sizeof(float) * nc);
            }
            if (!rc) rc = xmh_memcpy_h2d(s->coef_dev, hc, sizeof(float) * nc, e->stream);
            if (!rc) rc = xmh_stream_sync(e->stream);   /* hc is pageable host memory */
            free(hc);
            ++i;
        }
        if (!rc) e->n_stages++;
    }
    if (!rc) rc = xmh_stream_sync(e->stream);
    if (!rc) e->dirty = 0;
    return rc;
}

int xm_effects_stages(const XmEffects *ce, const XmFxStage **stages, int *n)
{
    XmEffects *e = (XmEffects *)ce;   /* lazily built cache */
    if (e->n_sub) return XM_EINVAL;   /* a multi-device chain has no stages of its own */
    int rc = build_stages(e);
    if (rc) return rc;
    *stages = e->stages;
    *n = e->n_stages;
    return XM_OK;
}

static int grow(void **p, size_t *cap, size_t need)
{
    if (*cap >= need) return XM_OK;
    xmh_free(*p);
    *p = NULL;
    *cap = 0;
    int rc = xmh_malloc(p, need);
    if (!rc) *cap = need;
    return rc;
}

static int ensure_ptrs(XmEffects *e, size_t n)
{
    if (e->ptr_cap >= n) return XM_OK;
    xmh_free(e->d_ptrs);
    xmh_host_free(e->h_ptrs);
    e->d_ptrs = NULL;
    e->h_ptrs = NULL;
    e->ptr_cap = 0;
    int rc = xmh_malloc((void **)&e->d_ptrs, n * sizeof(void *));
    if (!rc) rc = xmh_host_alloc((void **)&e->h_ptrs, n * sizeof(void *));
    if (!rc) e->ptr_cap = n;
    return rc;
}

/* Runs every stage; ping-pong through two device buffers so FIR never reads
 * what it writes.  src/dst: device pointer tables (n clips each). */
static int run_chain(XmEffects *e, size_t batch, size_t frames, float **src, float **dst, int streaming,
                     size_t clip0)
{
    const int C = e->cfg.channels;
    const size_t per = frames * (size_t)C;
    int rc = grow(&e->d_buf[0], &e->d_cap[0], batch * per * sizeof(float) + 16);
    if (!rc) rc = grow(&e->d_buf[1], &e->d_cap[1], batch * per * sizeof(float) + 16);
    if (!rc) rc = ensure_ptrs(e, batch * 6);
    if (rc) return rc;
    rc = xmh_stream_sync(e->stream);
    if (rc) return rc;
    /* table layout: [0,b) src  [b,2b) dst  [2b,3b) buf0  [3b,4b) buf1 */
    for (size_t i = 0; i < batch; ++i) {
        e->h_ptrs[i] = src[i];
        e->h_ptrs[batch + i] = dst[i];
        e->h_ptrs[2 * batch + i] = (float *)e->d_buf[0] + i * per;
        e->h_ptrs[3 * batch + i] = (float *)e->d_buf[1] + i * per;
    }
    rc = xmh_memcpy_h2d(e->d_ptrs, e->h_ptrs, 4 * batch * sizeof(void *), e->stream);
    if (rc) return rc;
    void **T_src = e->d_ptrs, **T_dst = e->d_ptrs + batch;
    void **T_b[2] = {e->d_ptrs + 2 * batch, e->d_ptrs + 3 * batch};
    int launches = 0;
    if (e->n_stages == 0) {
        for (size_t i = 0; !rc && i < batch; ++i)
            if (src[i] != dst[i]) rc = xmh_memcpy_d2d(dst[i], src[i], per * sizeof(float), e->stream);
        return rc;
    }
    /* FIR reads neighbours of the samples it writes: never run it in place.
     * If any clip is processed in place and the chain has a FIR stage, first
     * copy the inputs to buf0.  A biquad cascade runs in place (each chunk is
     * read into LDS before its outputs are stored). */
    int inplace = 0, off = 0, has_fir = 0;
    for (int s = 0; s < e->n_stages; ++s) has_fir |= e->stages[s].kind == 2;
    for (size_t i = 0; has_fir && i < batch; ++i) inplace |= src[i] == dst[i];
    void **cur = T_src;
    if (inplace) {
        for (size_t i = 0; !rc && i < batch; ++i)
            rc = xmh_memcpy_d2d((float *)e->d_buf[0] + i * per, src[i], per * sizeof(float), e->stream);
        cur = T_b[0];
        off = 1;
    }
    for (int s = 0; !rc && s < e->n_stages; ++s) {
        const int last = s == e->n_stages - 1;
        void **nxt = last ? T_dst : T_b[(s + off) & 1];
        XmhFxJob j;
        memset(&j, 0, sizeof j);
        j.channels = C;
        j.n_clips = (int32_t)batch;
        j.frames = (int64_t)frames;
        j.in_ptrs = (const float *const *)cur;
        j.out_ptrs = (float *const *)nxt;
        const size_t C2 = (size_t)C;
        if (e->stages[s].kind == 1) {
            j.sos = e->stages[s].coef_dev;
            j.n_sos = e->stages[s].n;
            if (streaming) j.state = e->st[s][0] + clip0 * (size_t)j.n_sos * 2 * C2;
        } else {
            j.fir = e->stages[s].coef_dev;
            j.fir_len = e->stages[s].n;
            if (streaming && j.fir_len > 1) {
                const size_t off = clip0 * (size_t)(j.fir_len - 1) * C2;
                j.hist_in = e->st[s][e->st_cur[s]] + off;
                j.hist_out = e->st[s][e->st_cur[s] ^ 1] + off;
            }
        }
        rc = xmh_launch_fx(&j, e->stream, &launches);
        cur = nxt;
    }
    return rc;
}

static int process(XmEffects *e, const float *const *in, float *const *out, size_t batch, size_t frames,
                   int streaming)
{
    int rc = XM_OK;
    const size_t bytes = frames * (size_t)e->cfg.channels * sizeof(float);
    if (e->cfg.mem_kind == XM_MEM_DEVICE) {
        /* FIR stages must not run in place: route through scratch when in == out */
        float **src = malloc(sizeof(float *) * batch), **dst = malloc(sizeof(float *) * batch);
        if (!src || !dst) rc = XM_ENOMEM;
        for (size_t i = 0; !rc && i < batch; ++i) {
            src[i] = (float *)in[i];
            dst[i] = out[i];
        }
        if (!rc) rc = run_chain(e, batch, frames, src, dst, streaming, 0);
        free(src);
        free(dst);
    } else {
        /* host: stage through a device buffer (chunks of <= 1 GiB) */
        size_t chunk = bytes ? ((size_t)1 << 30) / bytes : batch;
        if (chunk < 1) chunk = 1;
        if (chunk > batch) chunk = batch;
        void *d_io = NULL;
        rc = xmh_malloc(&d_io, chunk * bytes * 2);
        float **src = malloc(sizeof(float *) * chunk), **dst = malloc(sizeof(float *) * chunk);
        if (!src || !dst) rc = XM_ENOMEM;
        for (size_t b0 = 0; !rc && b0 < batch; b0 += chunk) {
            size_t nb = batch - b0 < chunk ? batch - b0 : chunk;
            for (size_t i = 0; !rc && i < nb; ++i) {
                src[i] = (float *)d_io + i * (bytes / sizeof(float));
                dst[i] = (float *)d_io + (chunk + i) * (bytes / sizeof(float));
                rc = xmh_memcpy_h2d(src[i], in[b0 + i], bytes, e->stream);
            }
            if (!rc) rc = run_chain(e, nb, frames, src, dst, streaming, b0);
            for (size_t i = 0; !rc && i < nb; ++i) rc = xmh_memcpy_d2h(out[b0 + i], dst[i], bytes, e->stream);
            if (!rc) rc = xmh_stream_sync(e->stream);
        }
        free(src);
        free(dst);
        xmh_stream_sync(e->stream);
        xmh_free(d_io);
    }
    if (!rc && !e->user_stream) rc = xmh_stream_sync(e->stream);
    return rc;
}

/* ---- multi-device dispatch: block d of the clips on sub-chain d ---------- */
typedef struct {
    const float *const *in;
    float *const *out;
    size_t batch, frames;
    int stream;   /* 0 process_batch, 1 process_stream (blocks of stream_reset) */
} XmFxArg;

static int t_fx(void *ctx, int d, void *p)
{
    XmEffects *e = ctx;
    const XmFxArg *a = p;
    size_t f, c;
    if (a->stream) {
        f = e->st_first[d];
        c = e->st_cnt[d];
    } else {
        xm_block(a->batch, e->n_sub, d, &f, &c);
    }
    if (!c) return XM_OK;
    return a->stream ? xm_effects_process_stream(e->sub[d], a->in + f, a->out + f, c, a->frames)
                     : xm_effects_process_batch(e->sub[d], a->in + f, a->out + f, c, a->frames);
}

int xm_effects_process_batch(XmEffects *e, const float *const *in, float *const *out, size_t batch, size_t frames)
{
    if (!e || (batch && (!in || !out))) return XM_EINVAL;
    if (batch == 0 || frames == 0) return XM_OK;
    if (batch > (size_t)INT32_MAX / 2) return XM_EINVAL;
    if (e->n_sub) {
        XmFxArg a = {in, out, batch, frames, 0};
        return xm_pool_run(e->pool, t_fx, &a);
    }
    int rc = xmh_set_device(e->cfg.device);
    if (!rc) rc = build_stages(e);
    if (rc) return rc;
    return process(e, in, out, batch, frames, 0);
}

/* ---- streaming ---------------------------------- */
int xm_effects_stream_reset(XmEffects *e, size_t n_clips)
{
    if (!e || n_clips == 0 || n_clips > (size_t)INT32_MAX / 2) return XM_EINVAL;
    if (e->n_sub) {   /* device d streams block d of the clips */
        int rc = XM_OK;
        e->st_ready = 0;
        for (int d = 0; d < e->n_sub && !rc; ++d) {
            xm_block(n_clips, e->n_sub, d, &e->st_first[d], &e->st_cnt[d]);
            if (e->st_cnt[d]) rc = xm_effects_stream_reset(e->sub[d], e->st_cnt[d]);
        }
        if (rc) return rc;
        e->st_clips = n_clips;
        e->st_ready = 1;
        e->dirty = 0;
        return XM_OK;
    }
    int rc = xmh_set_device(e->cfg.device);
    if (!rc) rc = build_stages(e);
    if (rc) return rc;
    xmh_stream_sync(e->stream);   /* a previous block may still use the old state */
    free_stream_state(e);
    const size_t C = (size_t)e->cfg.channels;
    for (int s = 0; !rc && s < e->n_stages; ++s) {
        const size_t per = e->stages[s].kind == 1 ? (size_t)e->stages[s].n * 2 * C
                                                   : (size_t)(e->stages[s].n - 1) * C;
        if (per == 0) continue;   /* 1-tap FIR: no history */
        const size_t bytes = n_clips * per * sizeof(float);
        const int nbuf = e->stages[s].kind == 1 ? 1 : 2;
        for (int k = 0; !rc && k < nbuf; ++k) {
            rc = xmh_malloc((void **)&e->st[s][k], bytes);
            if (!rc) rc = xmh_memset(e->st[s][k], 0, bytes, e->stream);
        }
        e->st_cur[s] = 0;
    }
    if (!rc) rc = xmh_stream_sync(e->stream);
    if (rc) {
        free_stream_state(e);
        return rc;
    }
    e->st_clips = n_clips;
    e->st_ready = 1;
    return XM_OK;
}

int xm_effects_process_stream(XmEffects *e, const float *const *in, float *const *out, size_t n_clips,
                              size_t frames)
{
    if (!e || (n_clips && (!in || !out))) return XM_EINVAL;
    if (e->dirty || !e->st_ready || n_clips != e->st_clips) return XM_EINVAL;   /* reset first */
    if (frames == 0) return XM_OK;
    if (e->n_sub) {
        XmFxArg a = {in, out, n_clips, frames, 1};
        return xm_pool_run(e->pool, t_fx, &a);
    }
    int rc = xmh_set_device(e->cfg.device);
    if (rc) return rc;
    rc = process(e, in, out, n_clips, frames, 1);
    if (!rc)
        for (int s = 0; s < e->n_stages; ++s)
            if (e->stages[s].kind == 2) e->st_cur[s] ^= 1;   /* hist_out becomes the history */
    return rc;
}
