/*
 * xm_audio_mixer.c — the xm_audio_mixer_* C API (SURVEY.md §1 layers L3/L2):
 * validation, handle state, host<->device staging, batch strides, and the
 * dispatch into the compute backend (csrc/xm_shim.h).  No arithmetic on
 * samples happens here: every sample is produced by a gfx950 kernel or, on a
 * handle created with n_devices == 0, by the host CPU backend (src/cpu/).
 * The backend is fixed at create time: a GPU handle without a usable GPU
 * fails with XM_EDEVICE, it never falls back to the CPU.
 *
 * Build-owned API (reference has none: /root/reference/README.md:1);
 * contract in include/xm_audio_mixer.h and include/xm_audio_common.h.
 */
#include <stdlib.h>
#include <string.h>

#include "xm_internal.h"

#define XM_FX_BLOCKS 8   /* time blocks of the config-4 pipeline */

struct XmAudioMixer {
    XmMixerConfig cfg;
    int n_tracks;
    XmTrackDesc tracks[XM_MAX_TRACKS];
    XmhGain gains[XM_MAX_TRACKS];
    XmhGain *gains_dev;
    int gains_dirty;
    int unity;                     /* single track, constant gain 1.0 */
    XmTable table;
    void *own_stream, *stream;
    int user_stream;
    void *ev[6];
    XmMixerTiming timing;
    int ev_done;                   /* this call recorded ev[2] then ev[3] (kernel window) */
    /* device scratch */
    void *d_in, *d_out, *d_fx;
    size_t d_in_cap, d_out_cap, d_fx_cap;
    void **d_ptrs;                 /* device pointer table (in ptrs then out ptrs) */
    size_t d_ptrs_cap;
    void **h_ptrs;                 /* pinned staging for the pointer table */
    const XmEffects *fx;
    /* streaming (xm_audio_mixer_stream_*): window rows [batch*n_tracks] of
     * st_cap frames, ping-pong st_win[st_cur]; row 0 holds absolute input
     * frame st_w0, rows hold st_recv - st_w0 valid frames */
    int st_on, st_ntr, st_cur;
    size_t st_batch, st_cap;
    int64_t st_recv, st_out, st_w0;
    void *st_win[2];
    /* per-track input rates (xm_audio_mixer_process_timeline): cached tables
     * for rates other than cfg.in_rate; trk_rt[tr] = index, -1 = m->table */
    XmTable rt[XM_MAX_TRACKS];
    int32_t rt_rate[XM_MAX_TRACKS];
    int n_rt, mixed_rates;
    int trk_rt[XM_MAX_TRACKS];
    int64_t *place_dev;            /* [XM_MAX_TRACKS][2] */
    XmhGain *unity_dev;            /* one unity-gain descriptor */
    XmMulti *multi;                /* multi-device handle: every call dispatches here */
    int span_chunks;               /* config 5: exchange chunks (0: automatic) */
    /* the time-block pipeline of resample -> biquad cascades -> mix (config 4,
     * run_fx_pipelined): the CU-masked biquad, resample and mix streams (split
     * fx_k of every 32 CUs), events per block, the biquad states and the
     * per-block pointer tables */
    void *fx_s[3];
    int fx_k;
    void *fx_ev[3][XM_FX_BLOCKS];
    float *fx_state;
    size_t fx_state_cap;
    void **fx_dtab, **fx_htab;
    size_t fx_tab_cap;
    /* the sequential effects path (run_with_effects): device pointer tables of
     * the track list and the two scratch sets, grown on demand and kept (a
     * hipFree per call would synchronise the whole device) */
    void *fx_seq_tab;
    size_t fx_seq_tab_cap;
};

void *xm_mixer_stream(const XmAudioMixer *m) { return m->stream; }

const XmTrackDesc *xm_mixer_tracks(const XmAudioMixer *m, int *n_tracks)
{
    *n_tracks = m->n_tracks;
    return m->tracks;
}

static int fmt_bytes(int fmt) { return fmt == XM_FMT_S16 ? 2 : 4; }

/* input element size (XM_MIXER_IN_CONVERT reads the other format) */
static int in_bytes(const XmAudioMixer *m)
{
    const int conv = (m->cfg.flags & XM_MIXER_IN_CONVERT) != 0;
    return fmt_bytes(conv ? (m->cfg.sample_fmt == XM_FMT_S16 ? XM_FMT_F32 : XM_FMT_S16) : m->cfg.sample_fmt);
}

/* the flags only whole-clip batch calls implement (stereo planar; mono is
 * planar and interleaved at once) */
static int io_flags(const XmAudioMixer *m)
{
    int f = 0;
    if (m->cfg.flags & XM_MIXER_IN_CONVERT) f |= XMH_IO_IN_CONV;
    if ((m->cfg.flags & XM_MIXER_PLANAR) && m->cfg.channels == 2) f |= XMH_IO_IN_PLANAR | XMH_IO_OUT_PLANAR;
    return f;
}

/* output element size (XM_MIXER_OUT_CONVERT writes the other format) */
static int out_bytes(const XmAudioMixer *m)
{
    const int conv = (m->cfg.flags & XM_MIXER_OUT_CONVERT) != 0;
    return fmt_bytes(conv ? (m->cfg.sample_fmt == XM_FMT_S16 ? XM_FMT_F32 : XM_FMT_S16) : m->cfg.sample_fmt);
}

static const XmhGain k_unity_desc = {1.0f, 1.0f, 0.0f, 32768, 32768, 0, 0, 0, 0};

/* the handle's device copy of one unity-gain descriptor, made on first use */
static int ensure_unity(XmAudioMixer *m)
{
    if (m->unity_dev) return XM_OK;
    int rc = xmh_malloc((void **)&m->unity_dev, sizeof k_unity_desc);
    if (!rc) rc = xmh_memcpy_h2d(m->unity_dev, &k_unity_desc, sizeof k_unity_desc, m->stream);
    return rc;
}

static int grow(void **p, size_t *cap, size_t need)
{
    if (*cap >= need) return XM_OK;
    xmh_free(*p);
    *p = NULL;
    *cap = 0;
    size_t n = need + need / 8 + 4096;
    int rc = xmh_malloc(p, n);
    if (rc) return rc;
    *cap = n;
    return XM_OK;
}

/* The host CPU backend (SURVEY.md §8(b) "n_devices (0 = CPU)"): n_devices ==
 * 0, or device == XM_DEVICE_CPU with n_devices <= 1. */
static int cfg_cpu(const XmMixerConfig *cfg) { return cfg->n_devices == 0 || (cfg->device == XM_DEVICE_CPU && cfg->n_devices <= 1); }

static int cfg_valid(const XmMixerConfig *cfg)
{
    return cfg && cfg->in_rate > 0 && cfg->out_rate > 0 && (cfg->channels == 1 || cfg->channels == 2) &&
           (cfg->sample_fmt == XM_FMT_S16 || cfg->sample_fmt == XM_FMT_F32) &&
           (cfg->mem_kind == XM_MEM_HOST || cfg->mem_kind == XM_MEM_DEVICE) &&
           (cfg->device >= 0 || (cfg->device == XM_DEVICE_CPU && cfg_cpu(cfg))) &&
           /* device memory on the CPU backend must be asked for explicitly
            * (device = XM_DEVICE_CPU: host memory, used in place); a config
            * with n_devices 0, a GPU ordinal and XM_MEM_DEVICE would hand HBM
            * pointers to the host, so it is refused */
           !(cfg_cpu(cfg) && cfg->mem_kind == XM_MEM_DEVICE && cfg->device != XM_DEVICE_CPU) &&
           !(cfg->flags & ~(int32_t)(XM_MIXER_OUT_CONVERT | XM_MIXER_IN_CONVERT | XM_MIXER_PLANAR)) &&
           cfg->n_devices >= 0 &&
           cfg->n_devices <= XM_MAX_DEVICES;
}

XmAudioMixer *xm_audio_mixer_create_multi(const XmMixerConfig *cfg, const int *devices, int n_devices, int *status)
{
    int rc = XM_OK;
    XmAudioMixer *m = NULL;
    XmMixerConfig c;
    if (!cfg || !devices || n_devices < 1 || n_devices > XM_MAX_DEVICES) {
        rc = XM_EINVAL;
        goto out;
    }
    c = *cfg;
    c.device = devices[0];
    c.n_devices = n_devices;
    if (!cfg_valid(&c)) {
        rc = XM_EINVAL;
        goto out;
    }
    for (int d = 0; d < n_devices; ++d)
        if (devices[d] < 0 || devices[d] >= xmh_device_count()) {
            rc = devices[d] < 0 ? XM_EINVAL : XM_EDEVICE;
            goto out;
        }
    m = calloc(1, sizeof *m);
    if (!m) {
        rc = XM_ENOMEM;
        goto out;
    }
    m->cfg = c;
    m->multi = xm_multi_create(&c, devices, n_devices, &rc);
    if (!rc) m->n_tracks = 1;
out:
    if (rc) xm_audio_mixer_freep(&m);
    if (status) *status = rc;
    return m;
}

XmAudioMixer *xm_audio_mixer_create_ex(const XmMixerConfig *cfg, int *status)
{
    int rc = XM_OK;
    XmAudioMixer *m = NULL;
    if (!cfg_valid(cfg)) {
        rc = XM_EINVAL;
        goto out;
    }
    if (cfg->n_devices > 1) {   /* devices device .. device+n-1 */
        int devs[XM_MAX_DEVICES];
        for (int d = 0; d < cfg->n_devices; ++d) devs[d] = cfg->device + d;
        return xm_audio_mixer_create_multi(cfg, devs, cfg->n_devices, status);
    }
    const int cpu = cfg_cpu(cfg);   /* n_devices 0 = the host CPU backend */
    if (!cpu && cfg->device >= xmh_device_count()) {
        rc = XM_EDEVICE;
        goto out;
    }
    m = calloc(1, sizeof *m);
    if (!m) {
        rc = XM_ENOMEM;
        goto out;
    }
    m->cfg = *cfg;
    if (cpu) {
        /* host memory is the CPU backend's device memory: HOST calls run in
         * place, with no staging copies */
        m->cfg.device = XMH_DEV_CPU;
        m->cfg.mem_kind = XM_MEM_DEVICE;
    }
    if ((rc = xmh_set_device(m->cfg.device))) goto out;
    if ((rc = xm_table_build(&m->table, cfg->in_rate, cfg->out_rate))) goto out;
    if ((rc = xmh_stream_create(&m->own_stream))) goto out;
    m->stream = m->own_stream;
    for (int i = 0; i < 6; ++i)
        if ((rc = xmh_event_create(&m->ev[i]))) goto out;
    if ((rc = xmh_malloc((void **)&m->gains_dev, sizeof(XmhGain) * XM_MAX_TRACKS))) goto out;
    /* default: one track at unity gain */
    XmTrackDesc t;
    memset(&t, 0, sizeof t);
    t.gain.gain0 = t.gain.gain1 = 1.0f;
    t.gain.gain0_q15 = t.gain.gain1_q15 = 32768;
    rc = xm_audio_mixer_set_tracks(m, &t, 1);
out:
    if (rc) xm_audio_mixer_freep(&m);
    if (status) *status = rc;
    return m;
}

XmAudioMixer *xm_audio_mixer_create(const XmMixerConfig *cfg) { return xm_audio_mixer_create_ex(cfg, NULL); }

void xm_audio_mixer_freep(XmAudioMixer **pm)
{
    if (!pm || !*pm) return;
    XmAudioMixer *m = *pm;
    if (m->multi || m->cfg.n_devices > 1) {   /* the sub-handles own every device resource */
        xm_multi_free(m->multi);
        free(m);
        *pm = NULL;
        return;
    }
    xmh_set_device(m->cfg.device);
    if (m->own_stream) xmh_stream_sync(m->own_stream);
    xm_table_free(&m->table);
    xmh_free(m->gains_dev);
    xmh_free(m->d_in);
    xmh_free(m->d_out);
    xmh_free(m->d_fx);
    xmh_free(m->st_win[0]);
    xmh_free(m->st_win[1]);
    for (int i = 0; i < m->n_rt; ++i) xm_table_free(&m->rt[i]);
    xmh_free(m->place_dev);
    xmh_free(m->unity_dev);
    xmh_free(m->d_ptrs);
    xmh_host_free(m->h_ptrs);
    for (int i = 0; i < 3; ++i)
        if (m->fx_s[i]) {
            xmh_stream_sync(m->fx_s[i]);
            xmh_stream_destroy(m->fx_s[i]);
        }
    for (int a = 0; a < 3; ++a)
        for (int k = 0; k < XM_FX_BLOCKS; ++k) xmh_event_destroy(m->fx_ev[a][k]);
    xmh_free(m->fx_state);
    xmh_free(m->fx_dtab);
    xmh_host_free(m->fx_htab);
    xmh_free(m->fx_seq_tab);
    for (int i = 0; i < 6; ++i) xmh_event_destroy(m->ev[i]);
    xmh_stream_destroy(m->own_stream);
    free(m);
    *pm = NULL;
}

int xm_audio_mixer_set_tracks(XmAudioMixer *m, const XmTrackDesc *tracks, int n_tracks)
{
    if (!m || !tracks || n_tracks < 1 || n_tracks > XM_MAX_TRACKS) return XM_EINVAL;
    if (m->multi) {
        int rc = xm_multi_set_tracks(m->multi, tracks, n_tracks);
        if (!rc) m->n_tracks = n_tracks;
        return rc;
    }
    XmhGain g[XM_MAX_TRACKS];
    int trk_rt[XM_MAX_TRACKS], mixed = 0, rc = XM_OK;
    for (int i = 0; i < n_tracks; ++i) {
        if (tracks[i].in_rate < 0) return XM_EINVAL;
        if ((rc = xm_gain_to_dev(&tracks[i].gain, &g[i]))) return rc;
    }
    /* per-track rate tables: the cache is rebuilt from this track list (kept
     * tables move over, new rates are designed, rates no track uses any more
     * are freed), so it never holds more than the distinct rates in use.  On
     * failure the handle keeps its previous tracks and tables. */
    XmTable nrt[XM_MAX_TRACKS];
    int32_t nrate[XM_MAX_TRACKS];
    int from_old[XM_MAX_TRACKS], nn = 0;
    for (int i = 0; i < n_tracks && !rc; ++i) {
        trk_rt[i] = -1;
        const int32_t r = tracks[i].in_rate;
        if (r == 0 || r == m->cfg.in_rate) continue;
        mixed = 1;
        int k = 0;
        while (k < nn && nrate[k] != r) ++k;
        if (k == nn) {
            int j = 0;
            while (j < m->n_rt && m->rt_rate[j] != r) ++j;
            if (j < m->n_rt) {
                nrt[nn] = m->rt[j];
                from_old[nn] = j;
            } else {
                if ((rc = xmh_set_device(m->cfg.device))) break;
                if ((rc = xm_table_build(&nrt[nn], r, m->cfg.out_rate))) break;
                from_old[nn] = -1;
            }
            nrate[nn++] = r;
        }
        trk_rt[i] = k;
    }
    if (rc) {
        for (int k = 0; k < nn; ++k)
            if (from_old[k] < 0) xm_table_free(&nrt[k]);
        return rc;
    }
    for (int j = 0; j < m->n_rt; ++j) {
        int kept = 0;
        for (int k = 0; k < nn; ++k) kept |= from_old[k] == j;
        if (!kept) {
            xmh_set_device(m->cfg.device);
            xm_table_free(&m->rt[j]);
        }
    }
    memcpy(m->rt, nrt, sizeof(XmTable) * (size_t)nn);
    memcpy(m->rt_rate, nrate, sizeof(int32_t) * (size_t)nn);
    m->n_rt = nn;
    memcpy(m->trk_rt, trk_rt, sizeof(int) * (size_t)n_tracks);
    m->mixed_rates = mixed;
    memcpy(m->tracks, tracks, sizeof(XmTrackDesc) * (size_t)n_tracks);
    memcpy(m->gains, g, sizeof(XmhGain) * (size_t)n_tracks);
    m->n_tracks = n_tracks;
    m->gains_dirty = 1;
    const XmhGain *g0 = &g[0];
    int const_one = (g0->flags == 0) &&
                    (m->cfg.sample_fmt == XM_FMT_F32 ? (g0->g0 == 1.0f && g0->g1 == 1.0f)
                                                     : (g0->q0 == 32768 && g0->q1 == 32768));
    m->unity = n_tracks == 1 && const_one;
    return XM_OK;
}

int xm_audio_mixer_set_crossfade(XmAudioMixer *m, int from, int to, int64_t start, int64_t len)
{
    if (!m || from < 0 || to < 0 || from >= m->n_tracks || to >= m->n_tracks || from == to || len < 0)
        return XM_EINVAL;
    if (m->multi) return xm_multi_set_crossfade(m->multi, from, to, start, len);
    XmTrackDesc t[XM_MAX_TRACKS];
    memcpy(t, m->tracks, sizeof(XmTrackDesc) * (size_t)m->n_tracks);
    t[from].gain.mode = XM_GAIN_XFADE_OUT;
    t[from].gain.ramp_start = start;
    t[from].gain.ramp_len = len;
    t[to].gain.mode = XM_GAIN_RAMP;
    t[to].gain.gain0 = 0.0f;
    t[to].gain.gain1 = 1.0f;
    t[to].gain.gain0_q15 = 0;
    t[to].gain.gain1_q15 = 32768;
    t[to].gain.ramp_start = start;
    t[to].gain.ramp_len = len;
    return xm_audio_mixer_set_tracks(m, t, m->n_tracks);
}

int xm_audio_mixer_set_track_effects(XmAudioMixer *m, const XmEffects *fx)
{
    if (!m) return XM_EINVAL;
    if (m->multi) {
        if (fx && m->cfg.sample_fmt != XM_FMT_F32) return XM_ENOSYS;
        return xm_multi_set_track_effects(m->multi, fx);
    }
    if (fx) {
        if (m->cfg.sample_fmt != XM_FMT_F32) return XM_ENOSYS;
        if (xm_effects_device(fx) != m->cfg.device) return XM_EINVAL;
    }
    m->fx = fx;
    return XM_OK;
}

size_t xm_audio_mixer_out_frames(const XmAudioMixer *m, size_t frames_in)
{
    if (!m) return 0;
    return xm_resample_out_frames(m->cfg.in_rate, m->cfg.out_rate, frames_in);
}

int xm_audio_mixer_set_stream(XmAudioMixer *m, void *s)
{
    if (!m) return XM_EINVAL;
    if (m->multi) return XM_ENOSYS;   /* a HIP stream belongs to one device */
    if (m->cfg.device == XMH_DEV_CPU) return XM_OK;   /* CPU calls are synchronous: nothing to order */
    m->stream = s ? s : m->own_stream;
    m->user_stream = s != NULL;
    return XM_OK;
}

int xm_audio_mixer_n_devices(const XmAudioMixer *m)
{
    if (!m) return XM_EINVAL;
    return m->multi ? xm_multi_n_devices(m->multi) : 1;
}

int xm_audio_mixer_get_timing(const XmAudioMixer *m, XmMixerTiming *t)
{
    if (!m || !t) return XM_EINVAL;
    if (m->multi) return xm_multi_get_timing(m->multi, t);
    *t = m->timing;
    return XM_OK;
}

/* every process-style call starts here: clears the timing of the last call */
static void begin_call(XmAudioMixer *m)
{
    memset(&m->timing, 0, sizeof m->timing);
    m->ev_done = 0;
}

/* ---- core: run one device-resident job ----------------------------------- */
static void job_init(XmAudioMixer *m, XmhMixJob *j, size_t batch, size_t frames_in)
{
    memset(j, 0, sizeof *j);
    j->fmt = m->cfg.sample_fmt;
    j->channels = m->cfg.channels;
    j->n_tracks = m->n_tracks;
    j->n_mix = (int32_t)batch;
    j->frames_in = (int64_t)frames_in;
    j->frames_out = (int64_t)xm_audio_mixer_out_frames(m, frames_in);
    j->gains = m->gains_dev;
    j->gains_host = m->gains;
    j->unity = m->unity;
    j->rs.L = m->table.d.L;
    j->rs.M = m->table.d.M;
    j->rs.T = m->table.d.T;
    j->rs.rm = m->table.d.rm;
    j->rs.H = m->table.H_dev;
    j->rs.fast = m->table.fast;
    if (m->cfg.flags & XM_MIXER_OUT_CONVERT) j->out_conv = m->cfg.sample_fmt == XM_FMT_F32 ? 1 : 2;
    j->io_flags = io_flags(m);
}

static int upload_gains(XmAudioMixer *m)
{
    if (!m->gains_dirty) return XM_OK;
    int rc = xmh_memcpy_h2d(m->gains_dev, m->gains, sizeof(XmhGain) * (size_t)m->n_tracks, m->stream);
    if (!rc) rc = xmh_stream_sync(m->stream);   /* m->gains is host pageable memory */
    if (!rc) m->gains_dirty = 0;
    return rc;
}

static int ptr_table(XmAudioMixer *m, const void *const *in, size_t n_in, void *const *out, size_t n_out,
                     const void *const **din, void *const **dout);

/* floats from one track's row of the effects scratch to the next: whole 64-B
 * lines, so every row (and every pipeline block, below) starts on a line */
static size_t fx_track_stride(int64_t frames, int C) { return ((size_t)frames * (size_t)C + 15) & ~(size_t)15; }

/* Effects path (config 4): resample every track into scratch at unity gain,
 * run the chain on each track in place, then the no-resample mix with the
 * track gains.  Order per track: resample -> effects -> gain -> ordered sum. */
/* Config 4 as a time-block pipeline.  The biquad stage is
 * serial in time (sosfilt's order, bit for bit) and its chain waves hold only
 * a fraction of the SIMDs (k_biquad_pc: 59 KB of LDS per workgroup, two per
 * CU, one latency-bound chain wave each), so the output is cut
 * into XM_FX_BLOCKS blocks of whole 147-output super-periods and the cheap
 * stages run beside the chain on the CUs it does not use:
 *   the biquad stream (fx_s[0]) is masked to the CUs i % 32 < k, enough for
 *   the whole biquad grid at once (k a multiple of 8: the same share of
 *   every XCD, whose workgroups are dealt round-robin);
 *   block 0's resample and the last block's mix run on the caller's stream
 *   over the whole GPU; the other blocks' resamples (fx_s[1]) and mixes
 *   (fx_s[2]) on the remaining CUs, i % 32 >= k.
 * Without the masks the resample grids, queued ahead, held every CU's LDS and
 * the biquad workgroups waited for whole CUs to drain: 10.86 ms against 9.84
 * for the three passes (profiles/r4_k_configs.jsonl).  Block k is filtered
 * once its resample has landed (section states carry from block to block, as
 * in xm_effects_process_stream) and mixed once filtered.  Every output is the
 * same kernel arithmetic as the three whole-clip passes (window jobs of the
 * same kernels, absolute gain indices), so the result is bit-identical.
 * XM_ENOSYS: not this path's shape, or no CU partition fits (the caller runs
 * the three passes). */
static int run_fx_pipelined(XmAudioMixer *m, const XmhMixJob *j0, const XmFxStage *st, int ns, float *scratch,
                            int *launches)
{
    const int C = j0->channels, ntr = j0->n_tracks;
    const int64_t F = j0->frames_out, N = j0->frames_in;
    const size_t ntot = (size_t)j0->n_mix * (size_t)ntr;
    const size_t per_track = fx_track_stride(F, C);
    if (m->cfg.device == XMH_DEV_CPU || ns < 1 || j0->in_ptrs || j0->out_ptrs || j0->io_flags || j0->in_base ||
        j0->out_base || j0->window || F < 32 * 16 * 147)   /* >= 16 super-periods in the smallest block */
        return XM_ENOSYS;
    if (j0->n_mix > 1 && j0->in_mix_stride != (int64_t)ntr * j0->in_track_stride) return XM_ENOSYS;
    int max_sos = 0;
    int64_t nwg = 0;   /* biquad workgroups of the largest stage (k_biquad_pc: 16 / n groups of 4 / C clips) */
    for (int s = 0; s < ns; ++s) {
        if (st[s].kind != 1 || st[s].n > 16) return XM_ENOSYS;   /* FIR stages: history handling, the three passes */
        max_sos = st[s].n > max_sos ? st[s].n : max_sos;
        int kpw = 16 / st[s].n * (4 / C);
        kpw = kpw < 12 ? kpw : 12;
        const int64_t w = ((int64_t)ntot + kpw - 1) / kpw;
        nwg = w > nwg ? w : nwg;
    }
    /* the CU split: the biquad grid resident at once (two k_biquad_pc
     * workgroups per CU: 59 KB of LDS each, csrc/xm_fx.hip PC_LDS), the other
     * CUs for the resample and the mix; k a multiple of 8 of every 32 CUs, so
     * every XCD gets the same share.  (Round 6 tried one workgroup of two
     * chain waves per CU, 93 KB: bq 7.58 against 7.38 ms and c4 8.22 against
     * 8.05 on one box, profiles/r6_g_ab.txt; reverted.) */
    int ksplit = 0;
    for (int k = 8; k < 32 && !ksplit; k += 8) {
        int nb = 0, nr = 0;
        xmh_stream_create_cus(NULL, 0, k, &nb);
        xmh_stream_create_cus(NULL, k, 32, &nr);
        if (2 * (int64_t)nb >= nwg && nr > 0) ksplit = k;
    }
    {   /* dev knob XM_FX_KSPLIT=k (8, 16, 24): the biquad's CUs per 32 */
        const char *e = getenv("XM_FX_KSPLIT");
        const int kf = e ? atoi(e) : 0;
        if (kf == 8 || kf == 16 || kf == 24) ksplit = kf;
    }
    if (!ksplit) return XM_ENOSYS;
    const int64_t L = m->table.d.L, M = m->table.d.M;
    const int fused = L == 147 && M == 160 && m->table.fast;   /* window jobs of the fused kernel */
    /* block starts in 32nds of the clip: 1, 2 and 4 at the head (block 0's
     * resample, on the whole GPU, is all the biquad waits for; each next
     * resample, on the other CUs, fits inside the block being filtered), 6 in
     * the body, 5 and 2 at the tail (the last mix runs after the last filter);
     * 8 blocks ran 0.7 % faster than 10 with a body of 4 (fewer block starts) */
    int cut[XM_FX_BLOCKS + 1] = {0, 2, 6, 14, 26, 38, 50, 60, 64};   /* 64ths of the clip */
    {   /* dev knob XM_FX_CUT="c1,...,c7": the inner block starts in 64ths */
        const char *e = getenv("XM_FX_CUT");
        int c[XM_FX_BLOCKS + 1] = {0}, n = 1, ok = e != NULL;
        for (const char *p = e; ok && *p && n < XM_FX_BLOCKS; ++n) {
            char *end;
            const long v = strtol(p, &end, 10);
            ok = end != p && v > c[n - 1] && v < 64;
            c[n] = (int)v;
            p = *end == ',' ? end + 1 : end;
        }
        if (ok && n == XM_FX_BLOCKS) {
            c[XM_FX_BLOCKS] = 64;
            memcpy(cut, c, sizeof cut);
        }
    }
    int64_t bs[XM_FX_BLOCKS + 1];
    int K = 0;
    bs[0] = 0;
    for (int k = 1; k <= XM_FX_BLOCKS; ++k) {
        /* whole groups of 8 super-periods (1176 outputs).  For stereo (C == 2)
         * every block then starts on a 64-B boundary of the f32 scratch rows
         * (1176 x 8 B = 147 x 64 B), so the window jobs' whole-segment stores
         * (k_rs147_mix SEG, sc1) write each 64-B line once and the biquad and
         * mix read whole lines.  Mono rows (1176 x 4 B = 4704 B) start odd
         * blocks 32 B off that grid: correct (stores are range-checked per
         * output), only the line-once property is stereo's */
        int64_t b = k == XM_FX_BLOCKS ? F : (F * cut[k] / 64 + 1175) / 1176 * 1176;
        b = b > F ? F : b;
        if (b > bs[K]) bs[++K] = b;
    }
    int rc = XM_OK;
    if (m->fx_k != ksplit)
        for (int i = 0; i < 3; ++i)
            if (m->fx_s[i]) {
                xmh_stream_sync(m->fx_s[i]);
                xmh_stream_destroy(m->fx_s[i]);
                m->fx_s[i] = NULL;
            }
    for (int i = 0; !rc && i < 3; ++i)
        if (!m->fx_s[i]) {
            int n = 0;
            rc = xmh_stream_create_cus(&m->fx_s[i], i ? ksplit : 0, i ? 32 : ksplit, &n);
        }
    if (rc) return rc;
    m->fx_k = ksplit;
    for (int a = 0; !rc && a < 3; ++a)
        for (int k = 0; !rc && k < XM_FX_BLOCKS; ++k)
            if (!m->fx_ev[a][k]) rc = xmh_event_create(&m->fx_ev[a][k]);
    if (!rc) rc = ensure_unity(m);
    /* biquad states [stage][clip][section][z0, z1][channel], zero at clip start */
    const size_t st_floats = (size_t)ns * ntot * (size_t)max_sos * 2u * (size_t)C;
    if (!rc && m->fx_state_cap < st_floats) {
        xmh_free(m->fx_state);
        m->fx_state = NULL;
        m->fx_state_cap = 0;
        rc = xmh_malloc((void **)&m->fx_state, st_floats * sizeof(float));
        if (!rc) m->fx_state_cap = st_floats;
    }
    /* block k's track pointers (scratch rows from the block's first frame) */
    const size_t ntab = (size_t)K * ntot;
    if (!rc && m->fx_tab_cap < ntab) {
        xmh_free(m->fx_dtab);
        xmh_host_free(m->fx_htab);
        m->fx_dtab = m->fx_htab = NULL;
        m->fx_tab_cap = 0;
        rc = xmh_malloc((void **)&m->fx_dtab, ntab * sizeof(void *));
        if (!rc) rc = xmh_host_alloc((void **)&m->fx_htab, ntab * sizeof(void *));
        if (!rc) m->fx_tab_cap = ntab;
    }
    if (rc) return rc;
    for (int k = 0; k < K; ++k)
        for (size_t i = 0; i < ntot; ++i) m->fx_htab[(size_t)k * ntot + i] = scratch + i * per_track + (size_t)bs[k] * C;
    void *sc = m->stream, *sb = m->fx_s[0], *sr = m->fx_s[1], *sm = m->fx_s[2];
    /* the internal streams start after everything earlier on the caller's stream */
    rc = xmh_event_record(m->fx_ev[2][0], sc);
    for (int i = 0; !rc && i < 3; ++i) rc = xmh_stream_wait(m->fx_s[i], m->fx_ev[2][0]);
    if (!rc) rc = xmh_memcpy_h2d(m->fx_dtab, m->fx_htab, ntab * sizeof(void *), sb);
    if (!rc) rc = xmh_memset(m->fx_state, 0, st_floats * sizeof(float), sb);
    const int64_t elem = (int64_t)in_bytes(m);
    for (int k = 0; !rc && k < K; ++k) {
        const int64_t o0 = bs[k], bl = bs[k + 1] - bs[k];
        void *rs = k == 0 ? sc : sr, *ms = k == K - 1 ? sc : sm;
        /* 1) resample block k of every track (1-track unity mixes) */
        XmhMixJob r = *j0;
        r.n_tracks = 1;
        r.n_mix = (int32_t)ntot;
        r.in_mix_stride = j0->in_track_stride;   /* track i of the flat list */
        r.in_track_stride = 0;
        r.gains = m->unity_dev;
        r.gains_host = &k_unity_desc;
        r.unity = 1;
        r.out_conv = 0;
        r.out = scratch + (size_t)o0 * C;
        r.out_mix_stride = (int64_t)per_track;
        r.frames_out = bl;
        rc = XM_ENOSYS;
        if (fused) {   /* window: input from the block's super-period origin, the 32 frames before it real */
            const int64_t a0 = o0 / 147 * 160;
            XmhMixJob w = r;
            w.in = (const char *)j0->in + a0 * C * elem;
            w.frames_in = N - a0;
            w.window = a0 > 0;
            rc = xmh_launch_mix_window(&w, rs, launches, &m->timing.fast_launches);
        }
        if (rc == XM_ENOSYS) {   /* any kernel: absolute output window */
            r.out_base = o0;
            rc = xmh_launch_mix(&r, rs, launches, &m->timing.fast_launches);
        }
        if (!rc) rc = xmh_event_record(m->fx_ev[0][k], rs);
        /* 2) the biquad cascades on block k, states carried */
        if (!rc) rc = xmh_stream_wait(sb, m->fx_ev[0][k]);
        for (int s = 0; !rc && s < ns; ++s) {
            XmhFxJob fj;
            memset(&fj, 0, sizeof fj);
            fj.channels = C;
            fj.n_clips = (int32_t)ntot;
            fj.frames = bl;
            fj.in_ptrs = (const float *const *)(m->fx_dtab + (size_t)k * ntot);
            fj.out_ptrs = (float *const *)(m->fx_dtab + (size_t)k * ntot);
            fj.sos = st[s].coef_dev;
            fj.n_sos = st[s].n;
            fj.state = m->fx_state + (size_t)s * ntot * (size_t)max_sos * 2u * (size_t)C;
            rc = xmh_launch_fx(&fj, sb, launches);
        }
        if (!rc) rc = xmh_event_record(m->fx_ev[1][k], sb);
        /* 3) the gained, ordered mix of block k */
        if (!rc) rc = xmh_stream_wait(ms, m->fx_ev[1][k]);
        if (!rc) {
            XmhMixJob x = *j0;
            x.in = scratch + (size_t)o0 * C;
            x.in_ptrs = NULL;
            x.in_ptrs_host = NULL;
            x.in_track_stride = (int64_t)per_track;
            x.in_mix_stride = (int64_t)(per_track * (size_t)ntr);
            x.frames_in = o0 + bl;   /* the absolute end: frames outside [0, frames_in) read as zero (xm_shim.h) */
            x.frames_out = bl;
            x.in_base = x.out_base = o0;   /* row 0 of the block is absolute frame o0 (gains at absolute frames) */
            x.out = (char *)j0->out + (size_t)o0 * C * (size_t)out_bytes(m);
            x.rs.L = x.rs.M = 1;
            x.rs.T = 1;
            x.rs.rm = 0;
            x.unity = 0;
            x.rs.fast = 0;
            rc = xmh_launch_mix(&x, ms, launches, &m->timing.fast_launches);
        }
    }
    /* the caller's stream continues after the other blocks' mixes (the last
     * block's biquad, which it waited for, follows every resample) */
    if (!rc) rc = xmh_event_record(m->fx_ev[2][1], sm);
    if (!rc) rc = xmh_stream_wait(sc, m->fx_ev[2][1]);
    if (rc) {   /* leave nothing in flight on the internal streams */
        for (int i = 0; i < 3; ++i) xmh_stream_sync(m->fx_s[i]);
    }
    return rc;
}

static int run_with_effects(XmAudioMixer *m, const XmhMixJob *j0, int *launches)
{
    const int C = j0->channels, ntr = j0->n_tracks;
    const size_t per_track = fx_track_stride(j0->frames_out, C);
    const size_t ntot = (size_t)j0->n_mix * (size_t)ntr;
    /* FIR stages read neighbours of what they write: they ping-pong between
     * two track buffers; biquad cascades run in place */
    const XmFxStage *st = NULL;
    int ns = 0, has_fir = 0;
    int rc = xm_effects_stages(m->fx, &st, &ns);
    if (rc) return rc;
    for (int s = 0; s < ns; ++s) has_fir |= st[s].kind == 2;
    const size_t buf_bytes = (ntot * per_track * sizeof(float) + 255) & ~(size_t)255;
    rc = grow(&m->d_fx, &m->d_fx_cap, buf_bytes * (has_fir ? 2 : 1) + 256);
    if (rc) return rc;
    float *scratch = (float *)m->d_fx;
    float *scratch2 = (float *)((char *)m->d_fx + buf_bytes);
    rc = run_fx_pipelined(m, j0, st, ns, scratch, launches);
    if (rc != XM_ENOSYS) {
        if (!rc) rc = xmh_stream_sync(m->stream);
        return rc;
    }
    /* 1) resample: treat every track as its own 1-track mix (unity gain) */
    rc = ensure_unity(m);
    if (rc) return rc;
    /* device pointer tables, one handle buffer: [0, ntot) the track list (when
     * the mixes are not ntr tracks apart), [ntot, 3 ntot) the two scratch sets */
    rc = grow(&m->fx_seq_tab, &m->fx_seq_tab_cap, sizeof(void *) * ntot * 3);
    if (rc) return rc;
    void **dtab = (void **)m->fx_seq_tab;
    XmhMixJob r = *j0;
    r.out_conv = 0;   /* tracks stay f32 in scratch; the final mix converts */
    r.io_flags = j0->io_flags & ~XMH_IO_OUT_PLANAR;   /* scratch is interleaved */
    r.n_tracks = 1;
    r.n_mix = (int32_t)ntot;
    r.gains = m->unity_dev;
    r.gains_host = &k_unity_desc;
    r.unity = 1;
    r.out = scratch;
    r.out_ptrs = NULL;
    r.out_mix_stride = (int64_t)per_track;
    const void **tp = NULL;   /* host table of the track pointers (irregular strides) */
    void **dtp = dtab;        /* its device copy: not m->d_ptrs, which may hold j0's output table */
    if (j0->in_ptrs) {
        r.in_ptrs = j0->in_ptrs;   /* same mix-major order */
    } else if (j0->n_mix == 1 || j0->in_mix_stride == (int64_t)ntr * j0->in_track_stride) {
        r.in_mix_stride = j0->in_track_stride;   /* track i of the flat list = mix i / ntr, track i % ntr */
        r.in_track_stride = 0;
    } else {
        /* mixes not ntr tracks apart: every track of the batch through a table */
        const int elem = in_bytes(m);
        tp = malloc(sizeof(void *) * ntot);
        if (!tp) rc = XM_ENOMEM;
        for (size_t i = 0; !rc && i < ntot; ++i)
            tp[i] = (const char *)j0->in +
                    ((int64_t)(i / (size_t)ntr) * j0->in_mix_stride + (int64_t)(i % (size_t)ntr) * j0->in_track_stride) *
                        elem;
        if (!rc) rc = xmh_memcpy_h2d(dtp, tp, sizeof(void *) * ntot, m->stream);
        r.in_ptrs = (const void *const *)dtp;
        r.in_ptrs_host = tp;
    }
    if (!rc) rc = xmh_launch_mix(&r, m->stream, launches, &m->timing.fast_launches);
    /* 2) effects chain on every track, in insertion order */
    void **tmp_ptrs = dtab + ntot;
    int cur = 0;   /* 0: tracks in scratch, 1: in scratch2 */
    if (!rc && ns > 0) {
        void **hp = malloc(sizeof(void *) * ntot * 2);
        if (!hp) rc = XM_ENOMEM;
        if (!rc) {
            for (size_t i = 0; i < ntot; ++i) {
                hp[i] = scratch + i * per_track;
                hp[ntot + i] = scratch2 + i * per_track;
            }
            rc = xmh_memcpy_h2d(tmp_ptrs, hp, sizeof(void *) * ntot * (has_fir ? 2 : 1), m->stream);
            if (!rc) rc = xmh_stream_sync(m->stream);
        }
        free(hp);
        for (int s = 0; !rc && s < ns; ++s) {
            XmhFxJob fj;
            memset(&fj, 0, sizeof fj);
            fj.channels = C;
            fj.n_clips = (int32_t)ntot;
            fj.frames = j0->frames_out;
            fj.in_ptrs = (const float *const *)(tmp_ptrs + (size_t)cur * ntot);
            if (st[s].kind == 1) {
                fj.out_ptrs = (float *const *)(tmp_ptrs + (size_t)cur * ntot);
                fj.sos = st[s].coef_dev;
                fj.n_sos = st[s].n;
            } else {
                fj.out_ptrs = (float *const *)(tmp_ptrs + (size_t)(cur ^ 1) * ntot);
                fj.fir = st[s].coef_dev;
                fj.fir_len = st[s].n;
            }
            rc = xmh_launch_fx(&fj, m->stream, launches);
            if (st[s].kind == 2) cur ^= 1;
        }
    }
    /* 3) mix, no resampling */
    if (!rc) {
        XmhMixJob x = *j0;
        x.in = cur ? scratch2 : scratch;
        x.in_ptrs = NULL;
        x.in_ptrs_host = NULL;
        x.in_track_stride = (int64_t)per_track;
        x.in_mix_stride = (int64_t)(per_track * (size_t)ntr);
        x.frames_in = j0->frames_out;
        x.rs.L = x.rs.M = 1;
        x.rs.T = 1;
        x.rs.rm = 0;
        x.unity = 0;
        x.rs.fast = 0;
        x.io_flags = j0->io_flags & XMH_IO_OUT_PLANAR;   /* reads the f32 interleaved scratch */
        rc = xmh_launch_mix(&x, m->stream, launches, &m->timing.fast_launches);
    }
    xmh_stream_sync(m->stream);   /* tp and the tables are read by the launches */
    free(tp);
    return rc;
}

static int run_job(XmAudioMixer *m, XmhMixJob *j)
{
    int launches = 0;
    int rc = xmh_event_record(m->ev[2], m->stream);
    if (rc) return rc;
    if (m->fx) rc = run_with_effects(m, j, &launches);
    else rc = xmh_launch_mix(j, m->stream, &launches, &m->timing.fast_launches);
    int rc2 = xmh_event_record(m->ev[3], m->stream);
    m->timing.n_launches += launches;
    if (!rc && !rc2) m->ev_done = 1;
    return rc ? rc : rc2;
}

/* Detects in[b*ntr + tr] == base + (b*ms + tr*ts)*elem.  Returns 1 if strided. */
static int as_strided(const void *const *p, size_t batch, int ntr, int elem, int64_t *ts, int64_t *ms)
{
    const char *base = (const char *)p[0];
    int64_t t = 0, mm = 0;
    if (ntr > 1) {
        int64_t d = (const char *)p[1] - base;
        if (d % elem) return 0;
        t = d / elem;
    }
    if (batch > 1) {
        int64_t d = (const char *)p[ntr] - base;
        if (d % elem) return 0;
        mm = d / elem;
    }
    for (size_t b = 0; b < batch; ++b)
        for (int tr = 0; tr < ntr; ++tr)
            if ((const char *)p[b * ntr + tr] != base + ((int64_t)b * mm + (int64_t)tr * t) * elem) return 0;
    *ts = t;
    *ms = mm;
    return 1;
}

static int ptr_table(XmAudioMixer *m, const void *const *in, size_t n_in, void *const *out, size_t n_out,
                     const void *const **din, void *const **dout)
{
    size_t n = n_in + n_out;
    int rc;
    if (m->d_ptrs_cap < n) {
        xmh_free(m->d_ptrs);
        xmh_host_free(m->h_ptrs);
        m->d_ptrs = NULL;
        m->h_ptrs = NULL;
        m->d_ptrs_cap = 0;
        if ((rc = xmh_malloc((void **)&m->d_ptrs, n * sizeof(void *)))) return rc;
        if ((rc = xmh_host_alloc((void **)&m->h_ptrs, n * sizeof(void *)))) return rc;
        m->d_ptrs_cap = n;
    }
    /* the previous call may still read the table on a user stream */
    if ((rc = xmh_stream_sync(m->stream))) return rc;
    if (in) memcpy(m->h_ptrs, in, n_in * sizeof(void *));
    if (out) memcpy(m->h_ptrs + n_in, out, n_out * sizeof(void *));
    if ((rc = xmh_memcpy_h2d(m->d_ptrs, m->h_ptrs, n * sizeof(void *), m->stream))) return rc;
    *din = in ? (const void *const *)m->d_ptrs : NULL;
    *dout = out ? (void *const *)(m->d_ptrs + n_in) : NULL;
    return XM_OK;
}

static int finish(XmAudioMixer *m, int rc)
{
    if (!rc && !m->user_stream) rc = xmh_stream_sync(m->stream);
    if (!rc && !m->user_stream && m->ev_done) {   /* only events this call recorded */
        float ms = 0.0f;
        if (!xmh_event_elapsed(&ms, m->ev[2], m->ev[3])) m->timing.kernel_ms = ms;
    }
    return rc;
}

static int process_device(XmAudioMixer *m, const void *const *in, void *const *out, size_t batch,
                          size_t frames_in)
{
    XmhMixJob j;
    job_init(m, &j, batch, frames_in);
    const int elem = in_bytes(m);
    int64_t ts = 0, ms = 0, os = 0, dummy = 0;
    const void *const *din = NULL;
    void *const *dout = NULL;
    int in_strided = as_strided(in, batch, m->n_tracks, elem, &ts, &ms);
    int out_strided = as_strided((const void *const *)out, batch, 1, out_bytes(m), &dummy, &os);
    int rc = XM_OK;
    if (!in_strided || !out_strided)
        rc = ptr_table(m, in_strided ? NULL : in, in_strided ? 0 : batch * (size_t)m->n_tracks,
                       out_strided ? NULL : out, out_strided ? 0 : batch, &din, &dout);
    if (rc) return rc;
    if (in_strided) {
        j.in = in[0];
        j.in_track_stride = ts;
        j.in_mix_stride = ms;
    } else {
        j.in_ptrs = din;
        j.in_ptrs_host = in;
    }
    if (out_strided) {
        j.out = out[0];
        j.out_mix_stride = os;
    } else {
        j.out_ptrs = dout;
    }
    return run_job(m, &j);
}

/* Host memory: stage mixes in chunks through device scratch, contiguous. */
static int process_host(XmAudioMixer *m, const void *const *in, void *const *out, size_t batch,
                        size_t frames_in)
{
    const int elem = in_bytes(m), C = m->cfg.channels, ntr = m->n_tracks;
    const size_t fout = xm_audio_mixer_out_frames(m, frames_in);
    const size_t in_track = frames_in * (size_t)C * (size_t)elem;
    const size_t out_mix = fout * (size_t)C * (size_t)out_bytes(m);
    const size_t per_mix = in_track * (size_t)ntr + out_mix;
    size_t chunk = per_mix ? ((size_t)2 << 30) / per_mix : batch;   /* <= 2 GiB per chunk */
    if (chunk < 1) chunk = 1;
    if (chunk > batch) chunk = batch;
    int rc = grow(&m->d_in, &m->d_in_cap, chunk * in_track * (size_t)ntr + 16);
    if (!rc) rc = grow(&m->d_out, &m->d_out_cap, chunk * out_mix + 16);
    float h2d = 0.0f, ker = 0.0f, d2h = 0.0f;
    for (size_t b0 = 0; !rc && b0 < batch; b0 += chunk) {
        size_t nb = batch - b0 < chunk ? batch - b0 : chunk;
        rc = xmh_event_record(m->ev[0], m->stream);
        for (size_t b = 0; !rc && b < nb; ++b)
            for (int tr = 0; !rc && tr < ntr; ++tr)
                rc = xmh_memcpy_h2d((char *)m->d_in + (b * (size_t)ntr + (size_t)tr) * in_track,
                                    in[(b0 + b) * (size_t)ntr + (size_t)tr], in_track, m->stream);
        if (rc) break;
        XmhMixJob j;
        job_init(m, &j, nb, frames_in);
        j.in = m->d_in;
        j.in_track_stride = (int64_t)(frames_in * (size_t)C);
        j.in_mix_stride = j.in_track_stride * ntr;
        j.out = m->d_out;
        j.out_mix_stride = (int64_t)(fout * (size_t)C);
        if ((rc = run_job(m, &j))) break;
        for (size_t b = 0; !rc && b < nb; ++b)
            rc = xmh_memcpy_d2h(out[b0 + b], (char *)m->d_out + b * out_mix, out_mix, m->stream);
        if (!rc) rc = xmh_event_record(m->ev[4], m->stream);
        if (!rc) rc = xmh_stream_sync(m->stream);
        float a = 0, k = 0, c = 0;
        if (!rc && !xmh_event_elapsed(&a, m->ev[0], m->ev[2])) h2d += a;
        if (!rc && !xmh_event_elapsed(&k, m->ev[2], m->ev[3])) ker += k;
        if (!rc && !xmh_event_elapsed(&c, m->ev[3], m->ev[4])) d2h += c;
    }
    m->timing.h2d_ms = h2d;
    m->timing.kernel_ms = ker;
    m->timing.d2h_ms = d2h;
    m->ev_done = 0;   /* kernel_ms is the sum over chunks, not the last chunk's window */
    return rc;
}

int xm_audio_mixer_process_batch(XmAudioMixer *m, const void *const *in, void *const *out, size_t batch,
                                 size_t frames_in)
{
    if (m && m->mixed_rates) return XM_ENOSYS;   /* tracks of other rates: process_timeline */
    if (!m || (batch && (!in || !out))) return XM_EINVAL;
    if (batch == 0) return XM_OK;
    if (batch > (size_t)INT32_MAX / XM_MAX_TRACKS) return XM_EINVAL;
    if (m->multi) return xm_multi_process_batch(m->multi, in, out, batch, frames_in);
    for (size_t i = 0; i < batch * (size_t)m->n_tracks; ++i)
        if (!in[i]) return XM_EINVAL;
    for (size_t i = 0; i < batch; ++i)
        if (!out[i]) return XM_EINVAL;
    int rc = xmh_set_device(m->cfg.device);
    if (rc) return rc;
    begin_call(m);
    if ((rc = upload_gains(m))) return rc;
    if (xm_audio_mixer_out_frames(m, frames_in) == 0) return XM_OK;
    if (m->cfg.mem_kind == XM_MEM_DEVICE) rc = process_device(m, in, out, batch, frames_in);
    else rc = process_host(m, in, out, batch, frames_in);
    return finish(m, rc);
}

int xm_audio_mixer_process_partial_s16(XmAudioMixer *m, const void *in, ptrdiff_t in_track_stride,
                                       ptrdiff_t in_mix_stride, int32_t *partial, ptrdiff_t partial_mix_stride,
                                       size_t batch, size_t frames_in)
{
    if (!m || (batch && (!in || !partial))) return XM_EINVAL;
    if (m->multi) return XM_ENOSYS;   /* config 5 on several devices: mix_spanning_s16 */
    if (m->cfg.sample_fmt != XM_FMT_S16 || m->cfg.mem_kind != XM_MEM_DEVICE || m->fx || m->mixed_rates ||
        (m->cfg.flags & XM_MIXER_OUT_CONVERT) || io_flags(m))
        return XM_ENOSYS;
    if (batch == 0) return XM_OK;
    if (batch > (size_t)INT32_MAX / XM_MAX_TRACKS) return XM_EINVAL;
    int rc = xmh_set_device(m->cfg.device);
    if (rc) return rc;
    begin_call(m);
    if ((rc = upload_gains(m))) return rc;
    if (xm_audio_mixer_out_frames(m, frames_in) == 0) return XM_OK;
    XmhMixJob j;
    job_init(m, &j, batch, frames_in);
    j.in = in;
    j.in_track_stride = in_track_stride;
    j.in_mix_stride = in_mix_stride;
    j.out = partial;
    j.out_mix_stride = partial_mix_stride;
    j.partial = 1;
    rc = run_job(m, &j);
    return finish(m, rc);
}

int xm_audio_mixer_finish_s16(XmAudioMixer *m, const int32_t *partials, int n_parts, ptrdiff_t part_stride,
                              ptrdiff_t partial_mix_stride, int16_t *out, ptrdiff_t out_mix_stride, size_t batch,
                              size_t out_frames)
{
    if (!m || n_parts < 1 || n_parts > XM_MAX_TRACKS) return XM_EINVAL;
    if (m->multi || m->cfg.sample_fmt != XM_FMT_S16 || m->cfg.mem_kind != XM_MEM_DEVICE || io_flags(m))
        return XM_ENOSYS;
    if (batch == 0 || out_frames == 0) return XM_OK;
    if (!partials || !out || batch > (size_t)INT32_MAX) return XM_EINVAL;
    int rc = xmh_set_device(m->cfg.device);
    if (rc) return rc;
    begin_call(m);
    rc = xmh_event_record(m->ev[2], m->stream);
    if (!rc)
        rc = xmh_launch_finish_s16(partials, n_parts, part_stride, partial_mix_stride, out, out_mix_stride,
                                   (int64_t)batch, (int64_t)out_frames * m->cfg.channels, m->stream);
    if (!rc) {
        m->timing.n_launches = 1;
        rc = xmh_event_record(m->ev[3], m->stream);
        if (!rc) m->ev_done = 1;
    }
    return finish(m, rc);
}

int xm_audio_mixer_process_strided(XmAudioMixer *m, const void *in, ptrdiff_t in_track_stride,
                                   ptrdiff_t in_mix_stride, void *out, ptrdiff_t out_mix_stride, size_t batch,
                                   size_t frames_in)
{
    if (m && m->mixed_rates) return XM_ENOSYS;   /* tracks of other rates: process_timeline */
    if (!m || (batch && (!in || !out))) return XM_EINVAL;
    if (batch == 0) return XM_OK;
    if (m->multi) return xm_multi_process_strided(m->multi, in, in_track_stride, in_mix_stride, out, out_mix_stride,
                                                  batch, frames_in);
    if (m->cfg.mem_kind != XM_MEM_DEVICE) {
        /* host memory: expand to pointer arrays */
        const int elem = in_bytes(m);
        size_t ntr = (size_t)m->n_tracks;
        const void **ip = malloc(sizeof(void *) * batch * ntr);
        void **op = malloc(sizeof(void *) * batch);
        int rc = (!ip || !op) ? XM_ENOMEM : XM_OK;
        for (size_t b = 0; !rc && b < batch; ++b) {
            for (size_t tr = 0; tr < ntr; ++tr)
                ip[b * ntr + tr] = (const char *)in + ((ptrdiff_t)b * in_mix_stride + (ptrdiff_t)tr * in_track_stride) * elem;
            op[b] = (char *)out + (ptrdiff_t)b * out_mix_stride * out_bytes(m);
        }
        if (!rc) rc = xm_audio_mixer_process_batch(m, (const void *const *)ip, (void *const *)op, batch, frames_in);
        free(ip);
        free(op);
        return rc;
    }
    if (batch > (size_t)INT32_MAX / XM_MAX_TRACKS) return XM_EINVAL;
    int rc = xmh_set_device(m->cfg.device);
    if (rc) return rc;
    begin_call(m);
    if ((rc = upload_gains(m))) return rc;
    if (xm_audio_mixer_out_frames(m, frames_in) == 0) return XM_OK;
    XmhMixJob j;
    job_init(m, &j, batch, frames_in);
    j.in = in;
    j.in_track_stride = in_track_stride;
    j.in_mix_stride = in_mix_stride;
    j.out = out;
    j.out_mix_stride = out_mix_stride;
    rc = run_job(m, &j);
    return finish(m, rc);
}

/* ---- streaming (build-owned) ----------------------
 * Output m of the whole-signal resample reads input frames up to
 * floor((m+rm)*M/L) and from floor((m+rm)*M/L) - T + 1 (xm_audio_common.h).
 * After R frames have arrived every m < ceil(L*R/M) - rm is final; the flush
 * (R = N) emits the rest up to ceil(N*L/M), frames >= N reading zero.  The
 * device window keeps the input frames the next output still needs; each
 * output is computed by the same kernel, taps and absolute gain index as in
 * one whole-signal call, so the concatenated blocks equal it bit for bit. */
static int64_t st_ready_out(const XmAudioMixer *m, int64_t R, int flush)
{
    const int64_t L = m->table.d.L, M = m->table.d.M, rm = m->table.d.rm;
    if (flush) return (int64_t)xm_audio_mixer_out_frames(m, (size_t)R);
    if (L == M) return R;
    int64_t e = (L * R + M - 1) / M - rm;
    return e > 0 ? e : 0;
}

static int64_t st_first_needed(const XmAudioMixer *m, int64_t mo)
{
    const int64_t L = m->table.d.L, M = m->table.d.M, rm = m->table.d.rm, T = m->table.d.T;
    if (L == M) return mo;
    return ((mo + rm) * M) / L - T + 1;
}

int xm_audio_mixer_stream_begin(XmAudioMixer *m, size_t batch)
{
    if (!m || batch == 0 || batch > (size_t)INT32_MAX / XM_MAX_TRACKS) return XM_EINVAL;
    if (m->multi) return xm_multi_stream_begin(m->multi, batch);
    if (m->fx || m->mixed_rates) return XM_ENOSYS;   /* effects: xm_effects_process_stream */
    if (io_flags(m)) return XM_ENOSYS;               /* XM_MIXER_IN_CONVERT / PLANAR: whole-clip calls */
    int rc = xmh_set_device(m->cfg.device);
    if (rc) return rc;
    if ((rc = xmh_stream_sync(m->stream))) return rc;   /* a previous stream's copies */
    m->st_on = 1;
    m->st_ntr = m->n_tracks;
    m->st_batch = batch;
    m->st_recv = m->st_out = m->st_w0 = 0;
    return XM_OK;
}

size_t xm_audio_mixer_stream_out_frames(const XmAudioMixer *m, size_t frames_in, int flush)
{
    if (m && m->multi) return xm_multi_stream_out_frames(m->multi, frames_in, flush);
    if (!m || !m->st_on) return 0;
    int64_t e = st_ready_out(m, m->st_recv + (int64_t)frames_in, flush);
    return e > m->st_out ? (size_t)(e - m->st_out) : 0;
}

/* Streaming through the fused 147/160 kernel: the outputs of this release
 * from the first super-period boundary ob_al = 147*ceil(out_base/147) on are
 * one window job -- input pointer at the window's frame a0 = 160*ob_al/147,
 * frames_in = R - a0 (frames past R read as zero, as the final flush needs;
 * a non-final release never reads them), output pointer and gain ramps
 * shifted by ob_al -- and the 32 frames before a0 are real samples
 * (job->window; the window keeps them, st_step step 3).  On success *j is cut
 * to the outputs before ob_al for the generic kernel; when the fused kernel
 * does not take the job, *j is left whole. */
/* The ratios whose fused kernel takes stream windows: 147/160 (48k -> 44.1k)
 * and 160/147 (44.1k -> 48k, round 5); a super-period is one period, L
 * outputs from M input frames, so window jobs start on multiples of L. */
static int st_fused_ratio(const XmAudioMixer *m)
{
    const int64_t L = m->table.d.L, M = m->table.d.M;
    return m->table.fast && ((L == 147 && M == 160) || (L == 160 && M == 147));
}

static int st_fast_part(XmAudioMixer *m, XmhMixJob *j, int64_t R, const char *win, size_t fb, int *launches)
{
    const int64_t L = m->table.d.L, M = m->table.d.M;
    if (!st_fused_ratio(m) || j->io_flags) return XM_OK;   /* out_conv 1: the kernel's s16 epilogue */
    const int64_t ob = j->out_base, oe = ob + j->frames_out;
    const int64_t ob_al = (ob + L - 1) / L * L, a0 = ob_al / L * M;
    if (oe - ob_al < 4 * L || a0 >= R || (a0 > 0 && a0 - 32 < m->st_w0)) return XM_OK;   /* too small to pay */
    XmhGain g[XM_MAX_TRACKS];
    for (int t = 0; t < m->n_tracks; ++t) {
        g[t] = m->gains[t];
        g[t].start -= ob_al;   /* the ramps are functions of n - start */
    }
    XmhMixJob w = *j;
    w.in = win + (size_t)(a0 - m->st_w0) * fb;
    w.frames_in = R - a0;
    w.frames_out = oe - ob_al;
    w.in_base = w.out_base = 0;
    w.out = (char *)j->out + (size_t)(ob_al - ob) * (size_t)m->cfg.channels * (size_t)out_bytes(m);
    w.gains_host = g;
    w.rs.fast = m->table.fast;
    w.window = a0 > 0;
    w.unity = m->unity;
    const int rc = xmh_launch_mix_window(&w, m->stream, launches, &m->timing.fast_launches);
    if (rc == XM_ENOSYS) return XM_OK;   /* not the fused kernel's shape: all generic */
    if (rc) return rc;
    j->frames_out = ob_al - ob;          /* the head before the first boundary */
    return XM_OK;
}

/* Device-memory pushes of the 147/160 stream: the super-period-aligned bulk
 * of the release reads the caller's block itself (no copy into the window).
 * The bulk starts at the first super-period boundary ob_al >= st_out whose
 * input frame a0 = 160*ob_al/147 has its 32-frame lead-in inside the block
 * (a0 - 32 >= B0, the block's first absolute frame); the outputs before ob_al
 * (the head) and everything of small blocks still run from the window.
 * Returns ob_al, or -1 when the bulk is too small to pay (the window path). */
static int64_t st_direct_cut(const XmAudioMixer *m, int64_t B0, int64_t R, int64_t mend, int flush)
{
    const int64_t L = m->table.d.L, M = m->table.d.M;
    if (flush || m->cfg.mem_kind != XM_MEM_DEVICE || !st_fused_ratio(m) || io_flags(m)) return -1;
    int64_t ob_al = (m->st_out + L - 1) / L * L;
    const int64_t q = (B0 + 32 + M - 1) / M;   /* first SP whose input frame a0 = q*M has its lead-in in the block */
    if (q * L > ob_al) ob_al = q * L;
    if (mend - ob_al < 4 * L || ob_al / L * M >= R) return -1;
    /* step 3 moves the frames the next release needs, [w0, R), from the
     * caller's block into the window, which holds at least the frames kept
     * plus the head's part of the block: decide here, before any launch,
     * that they fit (else the window path) */
    int64_t w0 = st_first_needed(m, mend) - 32;
    if (w0 > R) w0 = R;
    const int64_t held = (m->st_recv - m->st_w0) + (ob_al / L * M + 16 - B0);
    if (w0 >= B0 && R - w0 > held) return -1;
    return ob_al;
}

static int st_step(XmAudioMixer *m, const void *in, ptrdiff_t ts, ptrdiff_t ms, size_t n, void *out,
                   ptrdiff_t os, size_t out_cap, size_t *frames_out, int flush)
{
    if (frames_out) *frames_out = 0;
    if (m && m->multi) {
        if ((n && !in) || !frames_out) return XM_EINVAL;
        return xm_multi_stream_step(m->multi, in, ts, ms, n, out, os, out_cap, frames_out, flush);
    }
    if (!m || !m->st_on || (n && !in) || !frames_out) return XM_EINVAL;
    if (m->fx || m->mixed_rates || io_flags(m)) return XM_ENOSYS;   /* as stream_begin */
    if (m->n_tracks != m->st_ntr) return XM_EINVAL;   /* track list changed mid-stream */
    const int elem = fmt_bytes(m->cfg.sample_fmt), C = m->cfg.channels, ntr = m->st_ntr;
    const size_t batch = m->st_batch, rows = batch * (size_t)ntr, fb = (size_t)C * (size_t)elem;
    const size_t ofb = (size_t)C * (size_t)out_bytes(m);   /* output frame bytes */
    const int64_t R = m->st_recv + (int64_t)n;
    int64_t mend = st_ready_out(m, R, flush);
    if (mend < m->st_out) mend = m->st_out;
    const size_t nout = (size_t)(mend - m->st_out);
    if (nout && (!out || out_cap < nout)) return XM_EINVAL;
    int rc = xmh_set_device(m->cfg.device);
    if (rc) return rc;
    begin_call(m);
    if ((rc = upload_gains(m))) return rc;
    /* direct bulk (device memory): the window takes only the head's input,
     * frames [B0, a0 + 16) (the last head output reads up to a0 + 10) */
    const int64_t B0 = m->st_recv;
    const int64_t ob_dir = nout ? st_direct_cut(m, B0, R, mend, flush) : -1;
    const int64_t Ld = m->table.d.L, Md = m->table.d.M;
    const size_t n_app = ob_dir >= 0 ? (size_t)(ob_dir / Ld * Md + 16 - B0) : n;
    /* 1) append the block (or the head's part of it) to the window */
    const size_t keep = (size_t)(m->st_recv - m->st_w0);
    if (keep + n_app > m->st_cap) {
        size_t cap = keep + n_app + (keep + n_app) / 4 + 64;
        void *nw[2] = {NULL, NULL};
        rc = xmh_malloc(&nw[0], rows * cap * fb);
        if (!rc) rc = xmh_malloc(&nw[1], rows * cap * fb);
        if (!rc && keep)
            rc = xmh_memcpy2d(nw[0], cap * fb, m->st_win[m->st_cur], m->st_cap * fb, keep * fb, rows, m->stream);
        if (!rc) rc = xmh_stream_sync(m->stream);
        if (rc) {
            xmh_free(nw[0]);
            xmh_free(nw[1]);
            return rc;
        }
        xmh_free(m->st_win[0]);
        xmh_free(m->st_win[1]);
        m->st_win[0] = nw[0];
        m->st_win[1] = nw[1];
        m->st_cur = 0;
        m->st_cap = cap;
    }
    char *win = (char *)m->st_win[m->st_cur];
    const size_t pitch = m->st_cap * fb;
    if (n_app) {
        if (ms == (ptrdiff_t)ntr * ts || batch == 1)
            rc = xmh_memcpy2d(win + keep * fb, pitch, in, (size_t)ts * (size_t)elem, n_app * fb, rows, m->stream);
        else
            for (size_t b = 0; !rc && b < batch; ++b)
                rc = xmh_memcpy2d(win + (b * (size_t)ntr * pitch) + keep * fb, pitch,
                                  (const char *)in + (ptrdiff_t)b * ms * elem, (size_t)ts * (size_t)elem, n_app * fb,
                                  (size_t)ntr, m->stream);
        if (rc) return rc;
    }
    m->st_recv = R;
    /* 2) the outputs that are now final */
    if (nout) {
        int host = m->cfg.mem_kind != XM_MEM_DEVICE;
        if (host && (rc = grow(&m->d_out, &m->d_out_cap, batch * nout * ofb + 16))) return rc;
        XmhMixJob j;
        job_init(m, &j, batch, (size_t)R);
        j.frames_out = (int64_t)nout;
        j.in = win;
        j.in_track_stride = (int64_t)(m->st_cap * (size_t)C);
        j.in_mix_stride = j.in_track_stride * ntr;
        j.in_base = m->st_w0;
        j.out_base = m->st_out;
        j.rs.fast = 0;
        j.out = host ? m->d_out : out;
        j.out_mix_stride = host ? (int64_t)(nout * (size_t)C) : (int64_t)os;
        int launches = 0;
        rc = xmh_event_record(m->ev[2], m->stream);
        if (!rc && ob_dir >= 0) {
            /* the bulk [ob_dir, mend) on the fused kernel, straight from the
             * caller's block: window job at input frame a0, its 32 lead-in
             * frames real samples, ramps shifted by ob_dir */
            const int64_t a0 = ob_dir / Ld * Md;
            XmhGain g[XM_MAX_TRACKS];
            for (int t = 0; t < m->n_tracks; ++t) {
                g[t] = m->gains[t];
                g[t].start -= ob_dir;
            }
            XmhMixJob w = j;
            w.in = (const char *)in + (size_t)(a0 - B0) * fb;
            w.in_track_stride = ts;
            w.in_mix_stride = ms;
            w.frames_in = R - a0;
            w.frames_out = mend - ob_dir;
            w.in_base = w.out_base = 0;
            w.out = (char *)j.out + (size_t)(ob_dir - m->st_out) * ofb;
            w.gains_host = g;
            w.rs.fast = m->table.fast;
            w.window = 1;
            w.unity = m->unity;
            rc = xmh_launch_mix_window(&w, m->stream, &launches, &m->timing.fast_launches);
            if (rc == XM_ENOSYS) {   /* not the fused kernel's shape: the bulk on the generic kernel, same block */
                XmhMixJob gj = j;
                gj.in = in;
                gj.in_track_stride = ts;
                gj.in_mix_stride = ms;
                gj.in_base = B0;
                gj.out_base = ob_dir;
                gj.frames_out = mend - ob_dir;
                gj.out = w.out;
                rc = xmh_launch_mix(&gj, m->stream, &launches, &m->timing.fast_launches);
            }
            j.frames_out = ob_dir - m->st_out;                     /* the head: from the window */
        } else if (!rc) {
            rc = st_fast_part(m, &j, R, win, fb, &launches);       /* the super-period-aligned bulk */
        }
        if (!rc && j.frames_out)                                   /* the rest: generic kernel */
            rc = xmh_launch_mix(&j, m->stream, &launches, &m->timing.fast_launches);
        m->timing.n_launches += launches;
        if (!rc) rc = xmh_event_record(m->ev[3], m->stream);
        if (!rc) m->ev_done = 1;
        if (!rc && host)
            rc = xmh_memcpy2d(out, (size_t)os * (size_t)out_bytes(m), m->d_out, nout * ofb, nout * ofb, batch,
                              m->stream);
        if (rc) return rc;
    }
    if (m->cfg.mem_kind != XM_MEM_DEVICE) {   /* host buffers are the caller's again on return */
        if ((rc = xmh_stream_sync(m->stream))) return rc;
    }
    m->st_out = mend;
    /* 3) drop the frames no later output reads (move the rest to the other buffer) */
    /* + the fused kernel's 32-frame lead-in (its window ratios only: the
     * other kernels read the window from its first frame) */
    int64_t w0 = st_first_needed(m, mend) - (st_fused_ratio(m) ? 32 : 0);
    if (w0 > R) w0 = R;
    if (w0 < m->st_w0) w0 = m->st_w0;
    if (ob_dir >= 0 && w0 >= B0) {
        /* the window kept only the head's input: the frames the next release
         * needs, [w0, R), come from the caller's block */
        const size_t left = (size_t)(R - w0);
        char *nwin = (char *)m->st_win[m->st_cur ^ 1];
        if (left > m->st_cap) return XM_EINVAL;   /* excluded by st_direct_cut before any launch */
        if (ms == (ptrdiff_t)ntr * ts || batch == 1)
            rc = xmh_memcpy2d(nwin, pitch, (const char *)in + (size_t)(w0 - B0) * fb, (size_t)ts * (size_t)elem,
                              left * fb, rows, m->stream);
        else
            for (size_t b = 0; !rc && b < batch; ++b)
                rc = xmh_memcpy2d(nwin + b * (size_t)ntr * pitch, pitch,
                                  (const char *)in + (ptrdiff_t)b * ms * elem + (size_t)(w0 - B0) * fb,
                                  (size_t)ts * (size_t)elem, left * fb, (size_t)ntr, m->stream);
        if (rc) return rc;
        m->st_cur ^= 1;
        m->st_w0 = w0;
    } else if (w0 > m->st_w0 && !flush) {
        const size_t left = (size_t)(R - w0);
        if (left)
            rc = xmh_memcpy2d(m->st_win[m->st_cur ^ 1], pitch, win + (size_t)(w0 - m->st_w0) * fb, pitch,
                              left * fb, rows, m->stream);
        if (rc) return rc;
        m->st_cur ^= 1;
        m->st_w0 = w0;
    }
    *frames_out = nout;
    if (flush) m->st_on = 0;
    /* synchronous unless the caller installed a stream, whatever the block
     * size: the window copies above read the caller's `in` asynchronously */
    if (!nout) return m->user_stream ? XM_OK : xmh_stream_sync(m->stream);
    return finish(m, rc);
}

int xm_audio_mixer_stream_push(XmAudioMixer *m, const void *in, ptrdiff_t in_track_stride, ptrdiff_t in_mix_stride,
                               size_t frames_in, void *out, ptrdiff_t out_mix_stride, size_t out_cap,
                               size_t *frames_out)
{
    return st_step(m, in, in_track_stride, in_mix_stride, frames_in, out, out_mix_stride, out_cap, frames_out, 0);
}

int xm_audio_mixer_stream_flush(XmAudioMixer *m, void *out, ptrdiff_t out_mix_stride, size_t out_cap,
                                size_t *frames_out)
{
    return st_step(m, NULL, 0, 0, 0, out, out_mix_stride, out_cap, frames_out, 1);
}

/* ---- timeline mixes (build-owned) ---------
 * Each track is first resampled on its own (its XmTrackDesc.in_rate, same
 * kernels and order as a 1-track unity-gain mix, which equals the fused
 * per-track resample bit for bit: 0 + 1*r == r, and a Q15 unity term is the
 * sample itself), then placed at its output-frame offset and mixed with the
 * gains evaluated at the mix's output frame. */

static int timeline_device(XmAudioMixer *m, const void *const *in, const XmTrackPlacement *place,
                           void *const *out, size_t batch, size_t out_frames)
{
    const int ntr = m->n_tracks, C = m->cfg.channels, elem = fmt_bytes(m->cfg.sample_fmt);
    int rc = XM_OK, launches = 0;
    if (!m->place_dev && (rc = xmh_malloc((void **)&m->place_dev, sizeof(int64_t) * 2 * XM_MAX_TRACKS))) return rc;
    if ((rc = ensure_unity(m))) return rc;
    /* resampled lengths and scratch offsets */
    int64_t pl[2 * XM_MAX_TRACKS];
    size_t off[XM_MAX_TRACKS], scratch = 0;
    for (int tr = 0; tr < ntr; ++tr) {
        const XmTable *t = m->trk_rt[tr] < 0 ? &m->table : &m->rt[m->trk_rt[tr]];
        const int64_t n = place[tr].frames_in;
        pl[2 * tr] = place[tr].offset;
        pl[2 * tr + 1] = t->d.L == t->d.M ? n : (n * t->d.L + t->d.M - 1) / t->d.M;
        off[tr] = scratch;
        if (t->d.L != t->d.M) scratch += batch * (size_t)pl[2 * tr + 1] * (size_t)C * (size_t)elem + 256;
    }
    if ((rc = grow(&m->d_fx, &m->d_fx_cap, scratch + 16))) return rc;
    /* pointer table: [track-major inputs ntr*batch][mix-major placed tracks batch*ntr] + [batch outputs] */
    const size_t nb = batch * (size_t)ntr;
    const void **hp = malloc(sizeof(void *) * 2 * nb);
    if (!hp) return XM_ENOMEM;
    for (int tr = 0; tr < ntr; ++tr)
        for (size_t b = 0; b < batch; ++b) {
            const XmTable *t = m->trk_rt[tr] < 0 ? &m->table : &m->rt[m->trk_rt[tr]];
            hp[(size_t)tr * batch + b] = in[b * (size_t)ntr + (size_t)tr];
            hp[nb + b * (size_t)ntr + (size_t)tr] =
                t->d.L == t->d.M ? in[b * (size_t)ntr + (size_t)tr]
                                 : (const char *)m->d_fx + off[tr] + b * (size_t)pl[2 * tr + 1] * (size_t)C * (size_t)elem;
        }
    const void *const *din = NULL;
    void *const *dout = NULL;
    rc = ptr_table(m, hp, 2 * nb, out, batch, &din, &dout);
    if (!rc) rc = xmh_memcpy_h2d(m->place_dev, pl, sizeof(int64_t) * 2 * (size_t)ntr, m->stream);
    if (!rc) rc = xmh_event_record(m->ev[2], m->stream);
    for (int tr = 0; !rc && tr < ntr; ++tr) {
        const XmTable *t = m->trk_rt[tr] < 0 ? &m->table : &m->rt[m->trk_rt[tr]];
        if (t->d.L == t->d.M || place[tr].frames_in == 0) continue;
        XmhMixJob j;
        memset(&j, 0, sizeof j);
        j.fmt = m->cfg.sample_fmt;
        j.channels = C;
        j.n_tracks = 1;
        j.n_mix = (int32_t)batch;
        j.frames_in = place[tr].frames_in;
        j.frames_out = pl[2 * tr + 1];
        j.in_ptrs = din + (size_t)tr * batch;
        j.in_ptrs_host = (const void *const *)hp + (size_t)tr * batch;   /* the fused kernel's admission checks */
        j.out = (char *)m->d_fx + off[tr];
        j.out_mix_stride = pl[2 * tr + 1] * C;
        j.gains = m->unity_dev;
        j.gains_host = &k_unity_desc;
        j.unity = 1;
        j.rs.L = t->d.L;
        j.rs.M = t->d.M;
        j.rs.T = t->d.T;
        j.rs.rm = t->d.rm;
        j.rs.H = t->H_dev;
        j.rs.fast = t->fast;   /* 48k <-> 44.1k stereo f32 tracks: the fused kernel's 1-track rows */
        rc = xmh_launch_mix(&j, m->stream, &launches, &m->timing.fast_launches);
    }
    free(hp);
    if (!rc) {
        XmhMixJob j;
        memset(&j, 0, sizeof j);
        j.fmt = m->cfg.sample_fmt;
        j.channels = C;
        j.n_tracks = ntr;
        j.n_mix = (int32_t)batch;
        j.frames_out = (int64_t)out_frames;
        j.in_ptrs = din + nb;
        j.out_ptrs = dout;
        j.gains = m->gains_dev;
        j.place = m->place_dev;
        if (m->cfg.flags & XM_MIXER_OUT_CONVERT) j.out_conv = m->cfg.sample_fmt == XM_FMT_F32 ? 1 : 2;
        rc = xmh_launch_mix_placed(&j, m->stream, &launches);
    }
    if (!rc) rc = xmh_event_record(m->ev[3], m->stream);
    if (!rc) m->ev_done = 1;
    m->timing.n_launches += launches;
    return rc;
}

int xm_audio_mixer_process_timeline(XmAudioMixer *m, const void *const *in, const XmTrackPlacement *place,
                                    void *const *out, size_t batch, size_t out_frames)
{
    if (!m || !place || (batch && (!in || !out))) return XM_EINVAL;
    if (m->fx || io_flags(m)) return XM_ENOSYS;
    if (batch == 0 || out_frames == 0) return XM_OK;
    if (m->multi) return xm_multi_process_timeline(m->multi, in, place, out, batch, out_frames);
    if (batch > (size_t)INT32_MAX / XM_MAX_TRACKS) return XM_EINVAL;
    const int ntr = m->n_tracks;
    for (int tr = 0; tr < ntr; ++tr)
        if (place[tr].frames_in < 0 || place[tr].frames_in > ((int64_t)1 << 40)) return XM_EINVAL;
    for (size_t i = 0; i < batch * (size_t)ntr; ++i)
        if (!in[i]) return XM_EINVAL;
    for (size_t i = 0; i < batch; ++i)
        if (!out[i]) return XM_EINVAL;
    int rc = xmh_set_device(m->cfg.device);
    if (rc) return rc;
    begin_call(m);
    if ((rc = upload_gains(m))) return rc;
    if (m->cfg.mem_kind == XM_MEM_DEVICE) return finish(m, timeline_device(m, in, place, out, batch, out_frames));
    /* host memory: stage one mix at a time */
    const int C = m->cfg.channels, elem = fmt_bytes(m->cfg.sample_fmt);
    size_t in_bytes = 0, toff[XM_MAX_TRACKS];
    for (int tr = 0; tr < ntr; ++tr) {
        toff[tr] = in_bytes;
        in_bytes += (size_t)place[tr].frames_in * (size_t)C * (size_t)elem + 256;
    }
    const size_t out_mix_bytes = out_frames * (size_t)C * (size_t)out_bytes(m);
    rc = grow(&m->d_in, &m->d_in_cap, in_bytes + 16);
    if (!rc) rc = grow(&m->d_out, &m->d_out_cap, out_mix_bytes + 16);
    const void *dp[XM_MAX_TRACKS];
    void *dop[1];
    for (size_t b = 0; !rc && b < batch; ++b) {
        for (int tr = 0; !rc && tr < ntr; ++tr) {
            dp[tr] = (char *)m->d_in + toff[tr];
            rc = xmh_memcpy_h2d((void *)dp[tr], in[b * (size_t)ntr + (size_t)tr],
                                (size_t)place[tr].frames_in * (size_t)C * (size_t)elem, m->stream);
        }
        dop[0] = m->d_out;
        if (!rc) rc = timeline_device(m, dp, place, dop, 1, out_frames);
        if (!rc) rc = xmh_memcpy_d2h(out[b], m->d_out, out_mix_bytes, m->stream);
        if (!rc) rc = xmh_stream_sync(m->stream);
    }
    return finish(m, rc);
}

/* ---- multi-device entry points (src/xm_mixer_multi.c) -------------------- */
int xm_audio_mixer_process_sharded(XmAudioMixer *m, const void *const *in, ptrdiff_t in_track_stride,
                                   ptrdiff_t in_mix_stride, void *const *out, ptrdiff_t out_mix_stride,
                                   const size_t *batch, size_t frames_in)
{
    if (!m || !in || !out || !batch) return XM_EINVAL;
    if (m->multi)
        return xm_multi_process_sharded(m->multi, in, in_track_stride, in_mix_stride, out, out_mix_stride, batch,
                                        frames_in);
    if (m->cfg.mem_kind != XM_MEM_DEVICE) return XM_EINVAL;
    return xm_audio_mixer_process_strided(m, in[0], in_track_stride, in_mix_stride, out[0], out_mix_stride, batch[0],
                                          frames_in);
}

int xm_audio_mixer_set_span_chunks(XmAudioMixer *m, int chunks)
{
    if (!m || chunks < 0 || chunks > 64) return XM_EINVAL;
    m->span_chunks = chunks;
    return XM_OK;
}

int xm_audio_mixer_mix_spanning_s16(XmAudioMixer *m, const void *const *in, ptrdiff_t in_track_stride,
                                    ptrdiff_t in_mix_stride, void *const *out, ptrdiff_t out_mix_stride, size_t batch,
                                    size_t frames_in)
{
    if (!m || !in || !out) return XM_EINVAL;
    if (m->fx || m->mixed_rates) return XM_ENOSYS;
    if (m->multi)
        return xm_multi_mix_spanning_s16(m->multi, in, in_track_stride, in_mix_stride, out, out_mix_stride, batch,
                                         frames_in, m->span_chunks);
    /* one device holds every track: no exchange, the plain mix */
    if (m->cfg.sample_fmt != XM_FMT_S16 || m->cfg.mem_kind != XM_MEM_DEVICE || (m->cfg.flags & XM_MIXER_OUT_CONVERT) ||
        io_flags(m))
        return XM_ENOSYS;
    return xm_audio_mixer_process_strided(m, in[0], in_track_stride, in_mix_stride, out[0], out_mix_stride, batch,
                                          frames_in);
}
