/*
 * xm_mixer_multi.c — multi-device mixer handles (SURVEY.md §8(b) n_devices:
 * "a handle spawns one host worker thread per GPU, joined before
 * process_batch returns"; §8(e) partitioning).
 *
 * A multi-device handle owns one single-device handle (the whole single-GPU
 * path: staging, kernels, streams) and one persistent host worker thread per
 * device.  Mixes are independent, so a batch is cut into contiguous blocks,
 * block d on device d, and no data crosses devices: the result is the
 * one-device result bit for bit.  Config 5 (BASELINE.json:11), where the
 * tracks of every mix live on different devices, is the one exchange: int32
 * Q15 partials per device, one RCCL reduce-scatter over xGMI (or device
 * copies + an ordered sum when a device appears twice in the list), and a
 * saturating finish on the device that owns each block of mixes.  int32 sums
 * of <= 64 Q15 terms are exact in any order, so the
 * collective's schedule cannot change a bit.
 */
#include <stdlib.h>
#include <string.h>

#include "xm_internal.h"

typedef int (*XmTask)(XmMulti *mu, int d, void *arg);

struct XmMulti {
    int n;
    int devs[XM_MAX_DEVICES];
    XmAudioMixer *sub[XM_MAX_DEVICES];
    XmEffects *fx[XM_MAX_DEVICES];     /* per-device clones of the track effects chain */
    XmMixerConfig cfg;
    int n_tracks;
    XmTrackDesc tracks[XM_MAX_TRACKS]; /* the handle's full track list */
    int span_mode;                     /* 0: every sub holds the full list; 1: sub d holds its
                                          config-5 subset; 2: unknown (a failed update) */
    XmPool *pool;                      /* worker d drives device d (src/xm_pool.c) */
    int ran[XM_MAX_DEVICES];           /* sub d ran a call in the last dispatch (its timing counts) */
    /* streaming: the block of mixes each device streams */
    size_t st_first[XM_MAX_DEVICES], st_cnt[XM_MAX_DEVICES];
    int st_on;
    /* config 5 exchange */
    int distinct;                      /* every device ordinal differs: RCCL */
    void *comm[XM_MAX_DEVICES];
    int comm_ready;
    void *part[XM_MAX_DEVICES], *recv[XM_MAX_DEVICES];
    size_t part_cap[XM_MAX_DEVICES], recv_cap[XM_MAX_DEVICES];
    void *cstream[XM_MAX_DEVICES];     /* the reduce-scatters' streams, beside the partials' */
};

/* run task on every device (device d on worker d) and join; the first failing
 * device's status (in device order) is returned */
typedef struct {
    XmTask t;
    void *arg;
} XmTramp;

static int tramp(void *ctx, int d, void *a)
{
    const XmTramp *tr = a;
    return tr->t((XmMulti *)ctx, d, tr->arg);
}

static int run_all(XmMulti *mu, XmTask t, void *arg)
{
    for (int d = 0; d < mu->n; ++d) mu->ran[d] = 0;   /* each task marks the subs it calls */
    XmTramp tr = {t, arg};
    return xm_pool_run(mu->pool, tramp, &tr);
}

static void block(size_t batch, int n, int d, size_t *first, size_t *cnt) { xm_block(batch, n, d, first, cnt); }

static int fmt_bytes(int fmt) { return fmt == XM_FMT_S16 ? 2 : 4; }

static int in_elem(const XmMixerConfig *c)
{
    const int conv = (c->flags & XM_MIXER_IN_CONVERT) != 0;
    return fmt_bytes(conv ? (c->sample_fmt == XM_FMT_S16 ? XM_FMT_F32 : XM_FMT_S16) : c->sample_fmt);
}

static int out_elem(const XmMixerConfig *c)
{
    const int conv = (c->flags & XM_MIXER_OUT_CONVERT) != 0;
    return fmt_bytes(conv ? (c->sample_fmt == XM_FMT_S16 ? XM_FMT_F32 : XM_FMT_S16) : c->sample_fmt);
}

/* ---- lifecycle ------------------------------------------------------------ */
XmMulti *xm_multi_create(const XmMixerConfig *cfg, const int *devs, int n, int *status)
{
    int rc = XM_OK;
    XmMulti *mu = calloc(1, sizeof *mu);
    if (!mu) {
        if (status) *status = XM_ENOMEM;
        return NULL;
    }
    mu->n = n;
    mu->cfg = *cfg;
    mu->cfg.n_devices = 1;   /* each sub-handle: one GPU */
    mu->distinct = 1;
    for (int d = 0; d < n; ++d) {
        mu->devs[d] = devs[d];
        for (int e = 0; e < d; ++e) mu->distinct &= devs[e] != devs[d];
    }
    for (int d = 0; d < n && !rc; ++d) {
        XmMixerConfig c = mu->cfg;
        c.device = devs[d];
        mu->sub[d] = xm_audio_mixer_create_ex(&c, &rc);
    }
    if (!rc) {   /* the handle's default track list: one unity track (as create_ex) */
        memset(&mu->tracks[0], 0, sizeof mu->tracks[0]);
        mu->tracks[0].gain.gain0 = mu->tracks[0].gain.gain1 = 1.0f;
        mu->tracks[0].gain.gain0_q15 = mu->tracks[0].gain.gain1_q15 = 32768;
        mu->n_tracks = 1;
    }
    if (!rc) mu->pool = xm_pool_create(n, mu, &rc);
    if (rc) {
        xm_multi_free(mu);
        mu = NULL;
    }
    if (status) *status = rc;
    return mu;
}

void xm_multi_free(XmMulti *mu)
{
    if (!mu) return;
    xm_pool_free(&mu->pool);
    for (int d = 0; d < mu->n; ++d) {
        if (mu->comm[d]) xmh_comm_destroy(mu->comm[d]);
        xmh_set_device(mu->devs[d]);
        if (mu->cstream[d]) {
            xmh_stream_sync(mu->cstream[d]);
            xmh_stream_destroy(mu->cstream[d]);
        }
        xmh_free(mu->part[d]);
        xmh_free(mu->recv[d]);
        xm_audio_mixer_freep(&mu->sub[d]);
        xm_effects_freep(&mu->fx[d]);
    }
    free(mu);
}

int xm_multi_n_devices(const XmMulti *mu) { return mu->n; }

/* ---- track list --------------------------------------------------------------
 * Every sub-handle holds the full list, except while config 5 runs: then sub
 * d holds its own tracks [d*T/n, (d+1)*T/n) (span_mode) until the next call
 * that needs the full list. */
static int set_full(XmMulti *mu)
{
    int rc = XM_OK;
    mu->span_mode = 2;
    for (int d = 0; d < mu->n && !rc; ++d) rc = xm_audio_mixer_set_tracks(mu->sub[d], mu->tracks, mu->n_tracks);
    if (!rc) mu->span_mode = 0;
    return rc;
}

static int ensure_full(XmMulti *mu) { return mu->span_mode != 0 ? set_full(mu) : XM_OK; }

/* install a new full list on every sub; on failure the handle keeps its
 * previous list (re-applied to the subs), as a single-device handle does */
static int replace_full(XmMulti *mu, const XmTrackDesc *tracks, int n_tracks)
{
    XmTrackDesc old[XM_MAX_TRACKS];
    const int old_n = mu->n_tracks;
    memcpy(old, mu->tracks, sizeof(XmTrackDesc) * (size_t)old_n);
    if (tracks != mu->tracks) memcpy(mu->tracks, tracks, sizeof(XmTrackDesc) * (size_t)n_tracks);
    mu->n_tracks = n_tracks;
    int rc = set_full(mu);
    if (rc) {
        memcpy(mu->tracks, old, sizeof(XmTrackDesc) * (size_t)old_n);
        mu->n_tracks = old_n;
        set_full(mu);    /* best effort; on failure span_mode stays 2 and the next call retries */
    }
    return rc;
}

int xm_multi_set_tracks(XmMulti *mu, const XmTrackDesc *tracks, int n_tracks)
{
    /* validate on the first sub-handle; the others see the same list */
    int rc = xm_audio_mixer_set_tracks(mu->sub[0], tracks, n_tracks);
    if (rc) return rc;   /* sub 0 kept its list (single-device rule) */
    return replace_full(mu, tracks, n_tracks);
}

int xm_multi_set_crossfade(XmMulti *mu, int from, int to, int64_t start, int64_t len)
{
    int rc = ensure_full(mu);
    if (rc) return rc;
    if ((rc = xm_audio_mixer_set_crossfade(mu->sub[0], from, to, start, len))) return rc;
    /* sub 0 now holds the new list: give it to the others */
    int n = 0;
    XmTrackDesc t[XM_MAX_TRACKS];
    const XmTrackDesc *t0 = xm_mixer_tracks(mu->sub[0], &n);
    memcpy(t, t0, sizeof(XmTrackDesc) * (size_t)n);
    return replace_full(mu, t, n);
}

int xm_multi_set_track_effects(XmMulti *mu, const XmEffects *fx)
{
    int rc = XM_OK;
    for (int d = 0; d < mu->n && !rc; ++d) rc = xm_audio_mixer_set_track_effects(mu->sub[d], NULL);
    for (int d = 0; d < mu->n; ++d) xm_effects_freep(&mu->fx[d]);
    if (rc || !fx) return rc;
    /* one copy of the chain per device (the coefficients live in its HBM) */
    for (int d = 0; d < mu->n && !rc; ++d) {
        mu->fx[d] = xm_effects_clone_on(fx, mu->devs[d], &rc);
        if (!rc) rc = xm_audio_mixer_set_track_effects(mu->sub[d], mu->fx[d]);
    }
    if (rc)
        for (int d = 0; d < mu->n; ++d) {
            xm_audio_mixer_set_track_effects(mu->sub[d], NULL);
            xm_effects_freep(&mu->fx[d]);
        }
    return rc;
}

int xm_multi_get_timing(const XmMulti *mu, XmMixerTiming *t)
{
    memset(t, 0, sizeof *t);
    for (int d = 0; d < mu->n; ++d) {   /* devices run concurrently: the slowest one's times */
        if (!mu->ran[d]) continue;      /* idle in the last call: its timing is an older call's */
        XmMixerTiming s;
        xm_audio_mixer_get_timing(mu->sub[d], &s);
        if (s.h2d_ms > t->h2d_ms) t->h2d_ms = s.h2d_ms;
        if (s.kernel_ms > t->kernel_ms) t->kernel_ms = s.kernel_ms;
        if (s.d2h_ms > t->d2h_ms) t->d2h_ms = s.d2h_ms;
        t->n_launches += s.n_launches;
        t->fast_launches += s.fast_launches;
    }
    return XM_OK;
}

/* ---- batch calls: block d on device d ------------------------------------ */
typedef struct {
    const void *const *in;
    void *const *out;
    const void *in1;
    void *out1;
    ptrdiff_t ts, ms, os;
    size_t batch, frames;
    const XmTrackPlacement *place;
} XmBatchArg;

static int t_batch(XmMulti *mu, int d, void *p)
{
    const XmBatchArg *a = p;
    size_t f, c;
    block(a->batch, mu->n, d, &f, &c);
    if (!c) return XM_OK;
    mu->ran[d] = 1;
    return xm_audio_mixer_process_batch(mu->sub[d], a->in + f * (size_t)mu->n_tracks, a->out + f, c, a->frames);
}

int xm_multi_process_batch(XmMulti *mu, const void *const *in, void *const *out, size_t batch, size_t frames_in)
{
    int rc = ensure_full(mu);
    if (rc) return rc;
    XmBatchArg a = {.in = in, .out = out, .batch = batch, .frames = frames_in};
    return run_all(mu, t_batch, &a);
}

static int t_strided(XmMulti *mu, int d, void *p)
{
    const XmBatchArg *a = p;
    size_t f, c;
    block(a->batch, mu->n, d, &f, &c);
    if (!c) return XM_OK;
    mu->ran[d] = 1;
    const char *in = (const char *)a->in1 + (ptrdiff_t)f * a->ms * in_elem(&mu->cfg);
    char *out = (char *)a->out1 + (ptrdiff_t)f * a->os * out_elem(&mu->cfg);
    return xm_audio_mixer_process_strided(mu->sub[d], in, a->ts, a->ms, out, a->os, c, a->frames);
}

int xm_multi_process_strided(XmMulti *mu, const void *in, ptrdiff_t ts, ptrdiff_t ms, void *out, ptrdiff_t os,
                             size_t batch, size_t frames_in)
{
    /* one base pointer cannot address HBM of several devices */
    if (mu->cfg.mem_kind == XM_MEM_DEVICE) return XM_EINVAL;
    int rc = ensure_full(mu);
    if (rc) return rc;
    XmBatchArg a = {.in1 = in, .out1 = out, .ts = ts, .ms = ms, .os = os, .batch = batch, .frames = frames_in};
    return run_all(mu, t_strided, &a);
}

typedef struct {
    const void *const *in;
    void *const *out;
    ptrdiff_t ts, ms, os;
    const size_t *batch;
    size_t frames;
} XmShardArg;

static int t_sharded(XmMulti *mu, int d, void *p)
{
    const XmShardArg *a = p;
    if (!a->batch[d]) return XM_OK;
    mu->ran[d] = 1;
    return xm_audio_mixer_process_strided(mu->sub[d], a->in[d], a->ts, a->ms, a->out[d], a->os, a->batch[d],
                                          a->frames);
}

int xm_multi_process_sharded(XmMulti *mu, const void *const *in, ptrdiff_t ts, ptrdiff_t ms, void *const *out,
                             ptrdiff_t os, const size_t *batch, size_t frames_in)
{
    int rc = ensure_full(mu);
    if (rc) return rc;
    XmShardArg a = {in, out, ts, ms, os, batch, frames_in};
    return run_all(mu, t_sharded, &a);
}

static int t_timeline(XmMulti *mu, int d, void *p)
{
    const XmBatchArg *a = p;
    size_t f, c;
    block(a->batch, mu->n, d, &f, &c);
    if (!c) return XM_OK;
    mu->ran[d] = 1;
    return xm_audio_mixer_process_timeline(mu->sub[d], a->in + f * (size_t)mu->n_tracks, a->place, a->out + f, c,
                                           a->frames);
}

int xm_multi_process_timeline(XmMulti *mu, const void *const *in, const XmTrackPlacement *place, void *const *out,
                              size_t batch, size_t out_frames)
{
    int rc = ensure_full(mu);
    if (rc) return rc;
    XmBatchArg a = {.in = in, .out = out, .batch = batch, .frames = out_frames, .place = place};
    return run_all(mu, t_timeline, &a);
}

/* ---- streaming (host memory): every device streams its block ------------ */
int xm_multi_stream_begin(XmMulti *mu, size_t batch)
{
    if (mu->cfg.mem_kind == XM_MEM_DEVICE) return XM_ENOSYS;
    int rc = ensure_full(mu);
    for (int d = 0; d < mu->n && !rc; ++d) {
        block(batch, mu->n, d, &mu->st_first[d], &mu->st_cnt[d]);
        if (mu->st_cnt[d]) rc = xm_audio_mixer_stream_begin(mu->sub[d], mu->st_cnt[d]);
    }
    mu->st_on = !rc;
    return rc;
}

size_t xm_multi_stream_out_frames(const XmMulti *mu, size_t frames_in, int flush)
{
    if (!mu->st_on) return 0;
    for (int d = 0; d < mu->n; ++d)   /* every active block releases the same frames */
        if (mu->st_cnt[d]) return xm_audio_mixer_stream_out_frames(mu->sub[d], frames_in, flush);
    return 0;
}

typedef struct {
    const void *in;
    void *out;
    ptrdiff_t ts, ms, os;
    size_t n, cap;
    int flush;
    size_t got[XM_MAX_DEVICES];
} XmStreamArg;

static int t_stream(XmMulti *mu, int d, void *p)
{
    XmStreamArg *a = p;
    a->got[d] = 0;
    if (!mu->st_cnt[d]) return XM_OK;
    mu->ran[d] = 1;
    const char *in = a->in ? (const char *)a->in + (ptrdiff_t)mu->st_first[d] * a->ms * in_elem(&mu->cfg)
                           : NULL;
    char *out = a->out ? (char *)a->out + (ptrdiff_t)mu->st_first[d] * a->os * out_elem(&mu->cfg) : NULL;
    if (a->flush) return xm_audio_mixer_stream_flush(mu->sub[d], out, a->os, a->cap, &a->got[d]);
    return xm_audio_mixer_stream_push(mu->sub[d], in, a->ts, a->ms, a->n, out, a->os, a->cap, &a->got[d]);
}

int xm_multi_stream_step(XmMulti *mu, const void *in, ptrdiff_t ts, ptrdiff_t ms, size_t n, void *out,
                         ptrdiff_t os, size_t out_cap, size_t *frames_out, int flush)
{
    if (frames_out) *frames_out = 0;
    if (!mu->st_on || !frames_out) return XM_EINVAL;
    if (mu->span_mode) return XM_EINVAL;   /* the track list changed mid-stream */
    XmStreamArg a = {in, out, ts, ms, os, n, out_cap, flush, {0}};
    int rc = run_all(mu, t_stream, &a);
    for (int d = 0; d < mu->n; ++d)
        if (mu->st_cnt[d]) {
            *frames_out = a.got[d];
            break;
        }
    if (flush || rc) mu->st_on = 0;
    return rc;
}

/* ---- config 5: tracks spanning devices -----------------------------------
 * The owned blocks (device q finishes mixes [q*nb, (q+1)*nb)) are cut into K
 * chunks of cb = nb/K mixes; chunk k is mixes q*nb + k*cb .. + cb of every
 * owner q.  Each device writes the int32 partial of chunk k as [n owners][cb
 * mixes][S] at part + k*n*cb*S, so one reduce-scatter of that region gives
 * device d the summed partials of its cb mixes of the chunk.  On distinct
 * devices chunk k's reduce-scatter runs on a stream of its own while chunk
 * k+1's partials compute: the xGMI exchange hides behind the HBM-bound
 * partials except for the last chunk's.  int32 sums are
 * exact in any order, so every K gives the same bits. */
typedef struct {
    const void *const *in;
    void *const *out;
    ptrdiff_t ts, ms, os;
    size_t batch, frames, fo, S, nb;
    size_t K, cb, k;   /* chunks, mixes per owner and chunk, the chunk of this dispatch */
    int phase;         /* 0 partials of chunk k; 1 its exchange by copies + finish; 2 finish after RCCL */
} XmSpanArg;

static int grow_on(int dev, void **p, size_t *cap, size_t need)
{
    if (*cap >= need) return XM_OK;
    int rc = xmh_set_device(dev);
    if (rc) return rc;
    xmh_free(*p);
    *p = NULL;
    *cap = 0;
    if ((rc = xmh_malloc(p, need))) return rc;
    *cap = need;
    return XM_OK;
}

static int t_span(XmMulti *mu, int d, void *p)
{
    const XmSpanArg *a = p;
    XmAudioMixer *s = mu->sub[d];
    const size_t cblk = a->cb * a->S;   /* int32 per owner in one chunk */
    mu->ran[d] = 1;
    int rc = xmh_set_device(mu->devs[d]);
    if (rc) return rc;
    if (a->phase == 0) {   /* chunk k's partial, owner by owner: [q][cb][S] */
        rc = grow_on(mu->devs[d], &mu->part[d], &mu->part_cap[d], a->batch * a->S * sizeof(int32_t));
        int32_t *dst = (int32_t *)mu->part[d] + a->k * (size_t)mu->n * cblk;
        for (int q = 0; q < mu->n && !rc; ++q) {
            const size_t m0 = (size_t)q * a->nb + a->k * a->cb;   /* first mix of owner q in chunk k */
            rc = xm_audio_mixer_process_partial_s16(s, (const int16_t *)a->in[d] + (ptrdiff_t)m0 * a->ms, a->ts, a->ms,
                                                    dst + (size_t)q * cblk, (ptrdiff_t)a->S, a->cb, a->frames);
        }
        return rc;
    }
    int16_t *out = (int16_t *)a->out[d];
    if (a->phase == 1) {   /* owner d's piece of every device's chunk k, then the ordered sum over parts */
        rc = grow_on(mu->devs[d], &mu->recv[d], &mu->recv_cap[d], (size_t)mu->n * cblk * sizeof(int32_t));
        void *st = xm_mixer_stream(s);
        for (int q = 0; q < mu->n && !rc; ++q)
            rc = xmh_memcpy_peer((int32_t *)mu->recv[d] + (size_t)q * cblk, mu->devs[d],
                                 (const int32_t *)mu->part[q] + (a->k * (size_t)mu->n + (size_t)d) * cblk, mu->devs[q],
                                 cblk * sizeof(int32_t), st);
        if (!rc)
            rc = xm_audio_mixer_finish_s16(s, (const int32_t *)mu->recv[d], mu->n, (ptrdiff_t)cblk, (ptrdiff_t)a->S,
                                           out + (ptrdiff_t)(a->k * a->cb) * a->os, a->os, a->cb, a->fo);
        return rc;
    }
    /* phase 2: the reduce-scatters summed every chunk of block d into recv[d] ([nb][S], mix order) */
    rc = xmh_stream_sync(mu->cstream[d]);
    if (!rc)
        rc = xm_audio_mixer_finish_s16(s, (const int32_t *)mu->recv[d], 1, 0, (ptrdiff_t)a->S, out, a->os, a->nb,
                                       a->fo);
    if (!rc) rc = xmh_comm_check(mu->comm[d]);
    return rc;
}

/* K: the largest count <= the asked one (0: 4) that divides the owned block */
static size_t span_chunks(int asked, size_t nb)
{
    size_t k = asked > 0 ? (size_t)asked : 4;
    if (k > nb) k = nb;
    while (k > 1 && nb % k) --k;
    return k ? k : 1;
}

int xm_multi_mix_spanning_s16(XmMulti *mu, const void *const *in, ptrdiff_t ts, ptrdiff_t ms, void *const *out,
                              ptrdiff_t os, size_t batch, size_t frames_in, int chunks)
{
    const int n = mu->n;
    if (mu->cfg.sample_fmt != XM_FMT_S16 || mu->cfg.mem_kind != XM_MEM_DEVICE ||
        (mu->cfg.flags & XM_MIXER_OUT_CONVERT))
        return XM_ENOSYS;
    if (!in || !out || mu->n_tracks % n || batch % (size_t)n) return XM_EINVAL;
    for (int d = 0; d < n; ++d)
        if (!in[d] || !out[d]) return XM_EINVAL;
    if (batch == 0) return XM_OK;
    const int per = mu->n_tracks / n;
    if (mu->span_mode != 1) {   /* sub d holds its own tracks */
        int rc = XM_OK;
        mu->span_mode = 2;
        for (int d = 0; d < n && !rc; ++d) rc = xm_audio_mixer_set_tracks(mu->sub[d], mu->tracks + d * per, per);
        if (rc) {
            set_full(mu);
            return rc;
        }
        mu->span_mode = 1;
    }
    XmSpanArg a;
    memset(&a, 0, sizeof a);
    a.in = in;
    a.out = out;
    a.ts = ts;
    a.ms = ms;
    a.os = os;
    a.batch = batch;
    a.frames = frames_in;
    a.fo = xm_resample_out_frames(mu->cfg.in_rate, mu->cfg.out_rate, frames_in);
    a.S = a.fo * (size_t)mu->cfg.channels;
    a.nb = batch / (size_t)n;
    a.K = span_chunks(chunks, a.nb);
    a.cb = a.nb / a.K;
    if (a.fo == 0) return XM_OK;
    int rc = XM_OK;
    if (!mu->distinct) {   /* a repeated device: per chunk, partials (joined), then copies + ordered finish */
        for (a.k = 0; a.k < a.K && !rc; ++a.k) {
            a.phase = 0;
            rc = run_all(mu, t_span, &a);
            a.phase = 1;
            if (!rc) rc = run_all(mu, t_span, &a);
        }
        return rc;
    }
    /* distinct devices: RCCL over xGMI, chunk k's reduce-scatter (one group
     * over the devices, on the exchange streams) beside chunk k+1's partials */
    if (!mu->comm_ready) {
        if ((rc = xmh_comm_init_all(mu->comm, n, mu->devs))) return rc;
        mu->comm_ready = 1;
    }
    for (int d = 0; d < n && !rc; ++d) {
        rc = grow_on(mu->devs[d], &mu->recv[d], &mu->recv_cap[d], a.nb * a.S * sizeof(int32_t));
        if (!rc && !mu->cstream[d] && !(rc = xmh_set_device(mu->devs[d]))) rc = xmh_stream_create(&mu->cstream[d]);
    }
    if (rc) return rc;
    const size_t cblk = a.cb * a.S;
    int queued = 0;
    for (a.k = 0; a.k < a.K && !rc; ++a.k) {
        a.phase = 0;
        rc = run_all(mu, t_span, &a);   /* chunk k's partials on every device, joined */
        if (rc) break;
        if ((rc = xmh_group_start())) break;
        for (int d = 0; d < n; ++d) {
            int r2 = xmh_set_device(mu->devs[d]);
            if (!r2)
                r2 = xmh_reduce_scatter_i32((const int32_t *)mu->part[d] + a.k * (size_t)n * cblk,
                                            (int32_t *)mu->recv[d] + a.k * cblk, cblk, mu->comm[d], mu->cstream[d]);
            if (!rc) rc = r2;
        }
        const int r3 = xmh_group_end();
        if (!rc) rc = r3;
        queued = 1;
    }
    if (rc) {   /* leave no exchange in flight */
        for (int d = 0; queued && d < n; ++d) {
            xmh_set_device(mu->devs[d]);
            xmh_stream_sync(mu->cstream[d]);
        }
        return rc;
    }
    a.phase = 2;   /* saturate the owned blocks once their exchanges landed */
    return run_all(mu, t_span, &a);
}
