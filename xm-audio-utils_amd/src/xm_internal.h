/*
 * xm_internal.h — host-side (C) internals shared by the API translation units.
 */
#ifndef XM_INTERNAL_H
#define XM_INTERNAL_H

#include "xm_audio_common.h"
#include "xm_audio_mixer.h"
#include "xm_effects.h"
#include "../csrc/xm_shim.h"

#define XM_MAX_TRACKS 64
#define XM_MAX_SOS 64   /* one lane per (clip, section) in one wave (csrc/xm_fx.hip k_biquad_pipe) */
#define XM_MAX_FIR 4096
#define XM_MAX_EFFECTS 128   /* biquad sections + FIR stages per chain */

/* Cached device resample table for one reduced ratio. */
typedef struct XmTable {
    XmResampleDesign d;
    float *H_dev;          /* L*T floats on the handle's device */
    int fast;              /* 1: the baked 147/160 kernel computes exactly this table */
} XmTable;

int  xm_table_build(XmTable *t, int in_rate, int out_rate);
void xm_table_free(XmTable *t);

/* Convert a public XmGainRamp to the device descriptor (validates ranges). */
int xm_gain_to_dev(const XmGainRamp *g, XmhGain *d);

/* Effects chain internals (used by the mixer for per-track chains). */
typedef struct XmFxStage {
    int kind;              /* 1 = biquad cascade, 2 = FIR */
    int n;                 /* sections or taps */
    float *coef_dev;       /* n*6 (biquad) or n (FIR) floats on device */
} XmFxStage;

int xm_effects_stages(const XmEffects *e, const XmFxStage **stages, int *n_stages);
#define XM_DEVICE_NONE_ (-2)   /* xm_effects_device of a multi-device chain */
int xm_effects_device(const XmEffects *e);
/* the same chain (host coefficient copies replayed) on another device */
XmEffects *xm_effects_clone_on(const XmEffects *src, int device, int *status);

/* ---- host worker pool of the multi-device handles (src/xm_pool.c) ------- */
#define XM_MAX_DEVICES 16
typedef struct XmPool XmPool;
/* worker d runs task(ctx, d, arg); status of the first failing worker (in d order) */
typedef int (*XmPoolTask)(void *ctx, int d, void *arg);
XmPool *xm_pool_create(int n, void *ctx, int *status);   /* n == 1: runs on the caller's thread */
void xm_pool_free(XmPool **p);
int  xm_pool_run(XmPool *p, XmPoolTask t, void *arg);
/* contiguous block d of n over `batch` items (the first batch % n blocks one longer) */
void xm_block(size_t batch, int n, int d, size_t *first, size_t *cnt);

/* ---- multi-device effects chains (src/xm_effects.c) ---------------------- */
/* 1 if e is a multi-device chain (sub-chains per device) */
int xm_effects_is_multi(const XmEffects *e);

/* ---- multi-device mixer handles (src/xm_mixer_multi.c) ----------------- */
typedef struct XmMulti XmMulti;
/* one single-device sub-handle per entry of devs (duplicates allowed) */
XmMulti *xm_multi_create(const XmMixerConfig *cfg, const int *devs, int n, int *status);
void xm_multi_free(XmMulti *mu);
int  xm_multi_n_devices(const XmMulti *mu);
int  xm_multi_set_tracks(XmMulti *mu, const XmTrackDesc *tracks, int n_tracks);
int  xm_multi_set_crossfade(XmMulti *mu, int from, int to, int64_t start, int64_t len);
int  xm_multi_set_track_effects(XmMulti *mu, const XmEffects *fx);
int  xm_multi_get_timing(const XmMulti *mu, XmMixerTiming *t);
int  xm_multi_process_batch(XmMulti *mu, const void *const *in, void *const *out, size_t batch, size_t frames_in);
int  xm_multi_process_strided(XmMulti *mu, const void *in, ptrdiff_t ts, ptrdiff_t ms, void *out, ptrdiff_t os,
                              size_t batch, size_t frames_in);
int  xm_multi_process_sharded(XmMulti *mu, const void *const *in, ptrdiff_t ts, ptrdiff_t ms, void *const *out,
                              ptrdiff_t os, const size_t *batch, size_t frames_in);
int  xm_multi_process_timeline(XmMulti *mu, const void *const *in, const XmTrackPlacement *place,
                               void *const *out, size_t batch, size_t out_frames);
int  xm_multi_stream_begin(XmMulti *mu, size_t batch);
size_t xm_multi_stream_out_frames(const XmMulti *mu, size_t frames_in, int flush);
int  xm_multi_stream_step(XmMulti *mu, const void *in, ptrdiff_t ts, ptrdiff_t ms, size_t n, void *out,
                          ptrdiff_t os, size_t out_cap, size_t *frames_out, int flush);
int  xm_multi_mix_spanning_s16(XmMulti *mu, const void *const *in, ptrdiff_t ts, ptrdiff_t ms, void *const *out,
                               ptrdiff_t os, size_t batch, size_t frames_in, int chunks);
/* the stream a single-device handle launches on (its own or the caller's) */
void *xm_mixer_stream(const XmAudioMixer *m);
/* a single-device handle's current track list */
const XmTrackDesc *xm_mixer_tracks(const XmAudioMixer *m, int *n_tracks);

#endif
