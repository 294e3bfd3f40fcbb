/*
 * xm_effects.h — biquad / FIR effects chain over batches of clips (C ABI).
 *
 * BUILD-OWNED ABI (reference has no headers: /root/reference/README.md:1;
 * prefix xm_effects_* from BASELINE.json:5, signatures from SURVEY.md §8(b)).
 *
 * Arithmetic (pinned to scipy 1.15.3 float32):
 *  biquad section (b0,b1,b2,1,a1,a2), transposed direct form II, state zero at
 *  clip start, per channel, sections applied in insertion order:
 *      y  = b0*x + z0;  z0 = (b1*x - a1*y) + z1;  z1 = b2*x - a2*y;  x = y
 *  (scipy sosfilt, _signaltools.py:4601 / _sosfilt.pyx)
 *  FIR of K taps, causal, output length = input length:
 *      acc=+0; for t=0..K-1: acc = acc + x[n-K+1+t]*h[K-1-t]   (x<0 := 0)
 *  (scipy upfirdn(h, x)[:N], _upfirdn.py:107)
 *  Effects run in insertion order; consecutive biquads form one cascade.
 */
#ifndef XM_EFFECTS_H
#define XM_EFFECTS_H

#include "xm_audio_common.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct XmEffects XmEffects;

typedef enum XmEqBand {
    XM_EQ_PEAKING   = 0,
    XM_EQ_LOWSHELF  = 1,
    XM_EQ_HIGHSHELF = 2,
    XM_EQ_LOWPASS   = 3,
    XM_EQ_HIGHPASS  = 4
} XmEqBand;

typedef struct XmEffectsConfig {
    int32_t rate;        /* Hz */
    int32_t channels;    /* 1 or 2 */
    int32_t mem_kind;    /* XmMemKind of in/out pointers */
    int32_t device;      /* HIP device ordinal, or XM_DEVICE_CPU (the host CPU backend) */
} XmEffectsConfig;

XM_API XmEffects *xm_effects_create_ex(const XmEffectsConfig *cfg, int *status);
/* Host-memory chain (SURVEY.md §8(b) form): n_devices == 0 on the host CPU
 * backend (XM_DEVICE_CPU), n_devices == 1 on GPU 0, n_devices > 1 over GPUs
 * 0 .. n_devices-1 (xm_effects_create_multi); NULL if n_devices is out of
 * [0, 16] or names a device that is not there. */
XM_API XmEffects *xm_effects_create(int rate, int channels, int n_devices);

/* Multi-device chain over an explicit device list (n_devices in [1, 16]; a
 * device may repeat).  One single-device chain and one host worker thread per
 * entry ("one host worker thread per GPU, joined before
 * process_batch returns").  Effects added to the handle reach every device.
 * process_batch / process_stream cut the clips into contiguous blocks, block
 * d (the first batch % n blocks one clip longer) on device d, and return when
 * every device is done; clips are independent, so the result equals the
 * one-device result bit for bit.  With XM_MEM_DEVICE, block d's pointers must
 * be on device d.  cfg->device is ignored; set_stream returns XM_ENOSYS.
 * Such a chain attaches to multi-device mixers (copied per device), not to a
 * single-device mixer (XM_EINVAL there).  A list of one device returns the
 * plain single-device chain on it.  An effect that cannot be added to every
 * device's chain is added to none. */
XM_API XmEffects *xm_effects_create_multi(const XmEffectsConfig *cfg, const int *devices, int n_devices,
                                          int *status);

/* Devices a chain runs on (1 for a single-device chain). */
XM_API int xm_effects_n_devices(const XmEffects *e);

/* sos = {b0, b1, b2, a0, a1, a2}; a0 must be 1 (as scipy sosfilt requires).
 * A chain holds up to 128 effects (XM_ENOMEM beyond); consecutive biquads run
 * as one cascade of up to 64 sections per pass over the clip. */
XM_API int xm_effects_add_biquad(XmEffects *e, const float sos[6]);

/* RBJ audio-EQ-cookbook section designed in fp64 and cast to fp32.
 * q is Q (peaking / pass filters) or shelf slope S (shelves). */
XM_API int xm_effects_add_eq_band(XmEffects *e, int band, double f0_hz, double gain_db, double q);

/* FIR with K taps (1 <= K <= 4096), copied. */
XM_API int xm_effects_add_fir(XmEffects *e, const float *h, int K);

/* Number of effects and the coefficients of biquad i (for inspection). */
XM_API int xm_effects_count(const XmEffects *e);
XM_API int xm_effects_get_biquad(const XmEffects *e, int index, float sos[6]);

/* Install a caller-owned hipStream_t (NULL: the chain's own stream, which is
 * created blocking: ordered after the legacy default stream's work, as a
 * synchronous caller expects).  A CPU chain accepts and ignores it. */
XM_API int xm_effects_set_stream(XmEffects *e, void *hip_stream);

/* in/out: batch pointers of frames*channels float32 samples (in == out allowed). */
XM_API int xm_effects_process_batch(XmEffects *e, const float *const *in, float *const *out,
                             size_t batch, size_t frames);

/* ---- streaming (build-owned) ----------------------
 * n_clips long signals fed in blocks.  xm_effects_stream_reset() (re)starts
 * n_clips streams at zero state for the chain as it is now; every
 * xm_effects_process_stream() call filters the next `frames` frames of each
 * stream (in[i] / out[i] as process_batch, in == out allowed), carrying on
 * the device the biquad state (z0, z1 per section and channel) and the last
 * K-1 input frames of every FIR stage.  Any split of a signal into blocks
 * (ragged, 1-frame or empty blocks) gives, bit for bit, the output of one
 * process_batch() over the whole signal.  Adding an effect ends the streams:
 * process_stream then fails with XM_EINVAL until the next reset, as it does
 * for an n_clips other than the reset's. */
XM_API int xm_effects_stream_reset(XmEffects *e, size_t n_clips);
XM_API int xm_effects_process_stream(XmEffects *e, const float *const *in, float *const *out,
                              size_t n_clips, size_t frames);

XM_API void xm_effects_freep(XmEffects **e);

#ifdef __cplusplus
}
#endif
#endif /* XM_EFFECTS_H */
