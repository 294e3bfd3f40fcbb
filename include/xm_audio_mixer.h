/*
 * xm_audio_mixer.h — multi-track resample + gain-ramp + mixdown (C ABI).
 *
 * BUILD-OWNED ABI.  The reference snapshot has no headers
 * (/root/reference/README.md:1 is the whole tree); BASELINE.json:5 names the
 * prefix xm_audio_mixer_* and requires "host code stays in C and calls
 * hand-written HIP kernels through a thin C-ABI shim".  These entry points
 * are the ones SURVEY.md §8(b) proposes (create / set_tracks / process_batch /
 * freep / strerror), plus a strided form and a stream hook for callers whose
 * buffers already live in HBM.  Arithmetic: xm_audio_common.h.
 *
 * Data layout: each track / mix is interleaved PCM, frames x channels
 * (channel planes with XM_MIXER_PLANAR).
 * One "mix" = n_tracks input tracks -> one output of out_frames frames.
 *
 * Threading: a handle is not re-entrant (one caller thread per handle);
 * distinct handles may be used concurrently.  Calls are synchronous unless
 * the caller installed a stream with xm_audio_mixer_set_stream(), in which
 * case DEVICE-memory calls are stream-ordered and return without waiting
 * (the cuBLAS/hipBLAS convention).
 *
 * Multi-device handles (SURVEY.md §8(b) n_devices, §8(e)): a handle created
 * with XmMixerConfig.n_devices > 1 (devices device .. device+n-1) or by
 * xm_audio_mixer_create_multi() (any device list) owns one single-device
 * handle and one host worker thread per device.  A batch call splits its
 * mixes into contiguous blocks, block d (the first batch % n blocks one mix
 * longer) running on device d, and joins every worker before it returns;
 * independent mixes need no exchange, so the result is the one-device result
 * bit for bit.  Tracks that span devices (config 5) meet in one exchange
 * inside xm_audio_mixer_mix_spanning_s16 (RCCL reduce-scatter over xGMI).
 * On such a handle set_stream, process_partial_s16 and finish_s16 return
 * XM_ENOSYS; DEVICE-memory batches go through process_batch (each block's
 * pointers on its device) or process_sharded.
 */
#ifndef XM_AUDIO_MIXER_H
#define XM_AUDIO_MIXER_H

#include "xm_audio_common.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct XmAudioMixer XmAudioMixer;
struct XmEffects;

/* XmMixerConfig.flags: write the output in the other sample format, converted
 * in the kernels' store epilogue.  F32 mixers write
 * s16 = saturate16(rint(y * 32768)) (ties to even); S16 mixers write
 * f32 = y * 2^-15 (exact) of the saturated Q15 mix.  Output buffers and
 * output strides are then in elements of the output format. */
#define XM_MIXER_OUT_CONVERT 1u
/* XmMixerConfig.flags: the inputs are in the other sample format, converted in
 * the kernels' load path.  F32 mixers read s16
 * tracks as x * 2^-15 (exact); S16 mixers read f32 tracks as
 * saturate16(rint(x * 32768)) (ties to even).  Input buffers and input
 * strides are then in elements of the input format. */
#define XM_MIXER_IN_CONVERT 2u
/* XmMixerConfig.flags: planar PCM (stereo; mono is the same either way).  A
 * track of frames_in frames is `channels` planes of frames_in samples (plane c
 * = samples [c*frames_in, (c+1)*frames_in) from the track's start), a mix
 * output `channels` planes of out_frames samples; track and mix strides keep
 * their meaning (elements from one track / mix to the next).  The layout is
 * read and written by the kernels' load and store paths, no transposes.
 * IN_CONVERT and PLANAR apply to process_batch and process_strided, with or
 * without per-track effects; the streaming, timeline and config-5 calls
 * return XM_ENOSYS on such a handle. */
#define XM_MIXER_PLANAR 4u

typedef struct XmMixerConfig {
    int32_t in_rate;      /* Hz, every track (per-track rates: XmTrackDesc.in_rate) */
    int32_t out_rate;     /* Hz of the mix */
    int32_t channels;     /* 1 or 2 */
    int32_t sample_fmt;   /* XmSampleFmt, input and output */
    int32_t mem_kind;     /* XmMemKind of the in/out pointers */
    int32_t device;       /* HIP device ordinal the handle runs on, or XM_DEVICE_CPU */
    int32_t flags;        /* 0 or XM_MIXER_OUT_CONVERT | XM_MIXER_IN_CONVERT | XM_MIXER_PLANAR */
    int32_t n_devices;    /* 0: the host CPU backend (SURVEY.md §8(b) "n_devices (0 = CPU)");
                             1: one GPU, `device` (XM_DEVICE_CPU: the CPU backend);
                             n > 1: GPUs device .. device+n-1.
                             ABI note (round 4 -> 5): before round 4, 0 meant one GPU.  A
                             CPU handle takes host pointers; with XM_MEM_DEVICE it must be
                             asked for explicitly (device = XM_DEVICE_CPU): n_devices 0 with
                             a GPU ordinal and XM_MEM_DEVICE is refused (XM_EINVAL), so a
                             zero-initialised config can never hand HBM pointers to the host */
} XmMixerConfig;

typedef struct XmTrackDesc {
    XmGainRamp gain;      /* per-track gain ramp / crossfade side */
    int32_t    in_rate;   /* 0 = XmMixerConfig.in_rate; another rate is resampled on its own
                             to out_rate (process_timeline only; the uniform-length calls
                             return XM_ENOSYS while such a track is set) */
    int32_t    reserved;
} XmTrackDesc;

/* Per-call timing of the last process call, from HIP events on the handle's
 * stream (milliseconds; 0 where a stage did not run). */
typedef struct XmMixerTiming {
    float h2d_ms;         /* host->device staging (XM_MEM_HOST only) */
    float kernel_ms;      /* all device compute of the call */
    float d2h_ms;         /* device->host copy-back (XM_MEM_HOST only) */
    int32_t n_launches;   /* kernels launched by the call */
    int32_t fast_launches; /* of those, launches of the fused super-period kernel
                             (k_rs147_mix: every ratio, layout and format it is
                             instantiated for); the others ran a
                             generic kernel */
} XmMixerTiming;

/* Create a mixer.  Returns NULL on failure; *status (if non-NULL) gets the
 * reason.  n_devices == 0 (or device == XM_DEVICE_CPU with n_devices <= 1)
 * creates it on the host CPU backend (XM_DEVICE_CPU:
 * every call runs on the host cores, in place on host pointers, with the
 * GPU's results bit for bit; no GPU needed).  n_devices >= 1 creates it on
 * GPUs and fails with XM_EDEVICE when they are not usable: a GPU handle never
 * falls back to the CPU.  On a CPU handle set_stream is accepted and
 * ignored (calls are synchronous), mix_spanning_s16 runs as one device, and
 * the timing reports host wall time in kernel_ms. */
XM_API XmAudioMixer *xm_audio_mixer_create_ex(const XmMixerConfig *cfg, int *status);
XM_API XmAudioMixer *xm_audio_mixer_create(const XmMixerConfig *cfg);

/* Multi-device handle over an explicit device list (n_devices in [1, 16];
 * a device may appear more than once: two blocks on one GPU).  cfg->device
 * and cfg->n_devices are ignored. */
XM_API XmAudioMixer *xm_audio_mixer_create_multi(const XmMixerConfig *cfg, const int *devices, int n_devices,
                                                 int *status);

/* Devices a handle runs on (1 for a single-device handle). */
XM_API int xm_audio_mixer_n_devices(const XmAudioMixer *m);

/* Replace the track list (n_tracks in [1, 64]). */
XM_API int xm_audio_mixer_set_tracks(XmAudioMixer *m, const XmTrackDesc *tracks, int n_tracks);

/* Convenience: make track_from fade out and track_to fade in over
 * [start, start+len) output frames (linear, g_from = 1 - g_to). */
XM_API int xm_audio_mixer_set_crossfade(XmAudioMixer *m, int track_from, int track_to,
                                 int64_t start, int64_t len);

/* Attach an effects chain applied to every track after resampling and before
 * the gain (NULL detaches).  The chain's rate/channels must match the mix.
 * A single-device handle keeps the pointer and reads the chain at each call
 * (the chain must live on the handle's device).  A multi-device handle copies
 * the chain onto each of its devices here, so effects added to `fx` later do
 * not reach it until set_track_effects is called again. */
XM_API int xm_audio_mixer_set_track_effects(XmAudioMixer *m, const struct XmEffects *fx);

/* Output frames per mix for a given input length. */
XM_API size_t xm_audio_mixer_out_frames(const XmAudioMixer *m, size_t frames_in);

/* Install a caller-owned hipStream_t (NULL restores the handle's own stream).
 * The handle's own stream is a blocking stream (hipStreamDefault): its work is
 * ordered after what the caller queued on the legacy default stream (a
 * memset or fill of the buffers) and the other way round, on that device. */
XM_API int xm_audio_mixer_set_stream(XmAudioMixer *m, void *hip_stream);

/* in  : batch*n_tracks pointers, mix-major: in[b*n_tracks + tr]
 * out : batch pointers, each out_frames*channels samples
 * All tracks hold frames_in frames.  Pointers of one call must all be of the
 * configured XmMemKind. */
XM_API int xm_audio_mixer_process_batch(XmAudioMixer *m, const void *const *in,
                                 void *const *out, size_t batch, size_t frames_in);

/* Same, for buffers laid out with constant strides (in SAMPLES, not bytes):
 * track tr of mix b starts at in + b*in_mix_stride + tr*in_track_stride,
 * mix b's output at out + b*out_mix_stride. */
XM_API int xm_audio_mixer_process_strided(XmAudioMixer *m, const void *in,
                                   ptrdiff_t in_track_stride, ptrdiff_t in_mix_stride,
                                   void *out, ptrdiff_t out_mix_stride,
                                   size_t batch, size_t frames_in);

/* Multi-device handles, DEVICE memory already resident per device (the bench
 * shape): in[d] / out[d] are device d's tracks and outputs, strided as
 * process_strided, batch[d] its mixes (0 = idle).  A single-device handle
 * takes n = 1 arrays. */
XM_API int xm_audio_mixer_process_sharded(XmAudioMixer *m, const void *const *in, ptrdiff_t in_track_stride,
                                          ptrdiff_t in_mix_stride, void *const *out, ptrdiff_t out_mix_stride,
                                          const size_t *batch, size_t frames_in);

/* ---- cross-device mixdown (BASELINE.json:11, config 5: the tracks of one mix
 * live on different devices).  Each device runs the tracks it holds through
 * process_partial_s16, which writes the Q15 track sum of every output sample
 * as int32 WITHOUT the final saturation.  The caller adds the partials of all
 * devices (any order and grouping: <= 64 tracks of |term| <= 65535 cannot
 * overflow int32, so the sum is exact, e.g. an RCCL reduce-scatter over
 * xGMI), and finish_s16 saturates.  partial + exchange + finish equals
 * process_* over all the tracks, bit for bit.  Gains are evaluated at the
 * mix's output frame index, so a device holding tracks [t0, t1) simply sets
 * those tracks' ramps.  S16 mixers with XM_MEM_DEVICE only (else XM_ENOSYS);
 * no per-track effects.  Layouts as process_strided (strides in elements);
 * partial + b*partial_mix_stride holds out_frames*channels int32. */
XM_API int xm_audio_mixer_process_partial_s16(XmAudioMixer *m, const void *in,
                                       ptrdiff_t in_track_stride, ptrdiff_t in_mix_stride,
                                       int32_t *partial, ptrdiff_t partial_mix_stride,
                                       size_t batch, size_t frames_in);

/* out + b*out_mix_stride gets saturate16(sum over p < n_parts, in p order, of
 * partials[p*part_stride + b*partial_mix_stride + i]) for every sample
 * i < out_frames*channels.  n_parts in [1, 64]; strides in elements. */
XM_API int xm_audio_mixer_finish_s16(XmAudioMixer *m, const int32_t *partials, int n_parts,
                              ptrdiff_t part_stride, ptrdiff_t partial_mix_stride,
                              int16_t *out, ptrdiff_t out_mix_stride,
                              size_t batch, size_t out_frames);

/* Config 5 inside the library, on a multi-device S16 / DEVICE-memory handle
 * of n devices: the handle's n_tracks tracks are split evenly over the
 * devices (n_tracks % n == 0), device d holding tracks [d*T/n, (d+1)*T/n) of
 * every mix at in[d] (layout as process_strided over those T/n tracks).
 * Every device forms the int32 partial of its tracks; the partials meet in
 * one exchange -- an RCCL reduce-scatter over xGMI when the devices are
 * distinct (communicator created on first use, ncclCommInitAll), device
 * copies when a device repeats -- and device d saturates the mixes it owns,
 * [d*batch/n, (d+1)*batch/n) (batch % n == 0), into out[d] (out_mix_stride
 * apart).  Equal bit for bit to one 64-track process_* call.  XM_ECOMM if
 * the exchange fails (RCCL absent or a communicator error). */
XM_API int xm_audio_mixer_mix_spanning_s16(XmAudioMixer *m, const void *const *in, ptrdiff_t in_track_stride,
                                           ptrdiff_t in_mix_stride, void *const *out, ptrdiff_t out_mix_stride,
                                           size_t batch, size_t frames_in);

/* Config 5's exchange in chunks (build-owned, round 6): the mixes each device
 * owns are cut into `chunks` groups; the partials of group k+1 compute while
 * group k's reduce-scatter crosses xGMI on a stream of its own, so only the
 * last group's exchange is exposed.  chunks = 0 (the default): up to 4; the
 * count used is the largest one not above the asked count that divides
 * batch/n.  Every count gives the same bits (int32 sums are exact in any
 * order).  XM_EINVAL outside [0, 64]. */
XM_API int xm_audio_mixer_set_span_chunks(XmAudioMixer *m, int chunks);

/* ---- streaming (build-owned) ----------------------
 * `batch` mixes whose tracks arrive in blocks.  stream_begin() starts them at
 * input frame 0; every stream_push() appends the next frames_in frames of
 * every track (layout as process_strided, strides in elements) and writes the
 * output frames that no later input can change, *frames_out of them, to
 * out + b*out_mix_stride (out_cap: the room per mix, in frames);
 * stream_flush() ends the signal (N = all frames pushed) and writes the
 * rest.  The concatenated outputs equal one process_* call over the whole
 * signal, bit for bit, for any split into blocks (ragged, 1-frame, empty):
 * each output is computed by the same taps, in the same order, with the gain
 * ramp at the same absolute output frame.  The handle keeps the input frames
 * the next output still needs (about T + M/L frames per track) on the device.
 * stream_out_frames(frames_in, flush) is the exact count the next push of
 * frames_in frames (flush = 0) or the flush (flush = 1, frames_in = 0) writes.
 * Not with per-track effects (XM_ENOSYS: stream those with
 * xm_effects_process_stream); set_tracks with another track count ends the
 * stream (XM_EINVAL until stream_begin). */
XM_API int xm_audio_mixer_stream_begin(XmAudioMixer *m, size_t batch);
XM_API size_t xm_audio_mixer_stream_out_frames(const XmAudioMixer *m, size_t frames_in, int flush);
XM_API int xm_audio_mixer_stream_push(XmAudioMixer *m, const void *in, ptrdiff_t in_track_stride,
                               ptrdiff_t in_mix_stride, size_t frames_in, void *out,
                               ptrdiff_t out_mix_stride, size_t out_cap, size_t *frames_out);
XM_API int xm_audio_mixer_stream_flush(XmAudioMixer *m, void *out, ptrdiff_t out_mix_stride,
                                size_t out_cap, size_t *frames_out);

/* ---- timeline mixes (build-owned; SURVEY.md §8(f) items 2-3: BGM/voice
 * layouts, BASELINE.json:11).  Every track has its own length and may have
 * its own input rate (XmTrackDesc.in_rate); it is resampled on its own to
 * out_rate (exactly as a 1-track process_* call would) and placed so that its
 * first resampled frame lands on output frame `offset` (negative: the head
 * is cut).  out[b] gets out_frames frames: out[m] = ordered track sum of
 * gain_tr(m) * r_tr[m - offset_tr], r_tr = 0 outside its resampled length;
 * frames no track covers are silence.  The same placement applies to every
 * mix of the batch.  in: batch*n_tracks pointers (mix-major), out: batch
 * pointers, of the configured XmMemKind (host memory is staged one mix at a
 * time).  Not with per-track effects (XM_ENOSYS). */
typedef struct XmTrackPlacement {
    int64_t offset;       /* output frame of the track's first resampled frame */
    int64_t frames_in;    /* input frames of this track, at its own rate */
} XmTrackPlacement;

XM_API int xm_audio_mixer_process_timeline(XmAudioMixer *m, const void *const *in,
                                    const XmTrackPlacement *place, void *const *out,
                                    size_t batch, size_t out_frames);

XM_API int xm_audio_mixer_get_timing(const XmAudioMixer *m, XmMixerTiming *t);

/* Destroy and NULL the handle (no-op on NULL). */
XM_API void xm_audio_mixer_freep(XmAudioMixer **m);

/* Diagnostics (tests): the super-period split of the calling thread's last
 * launch of the fused kernel k_rs147_mix.  *sp_per_lane = R,
 * the consecutive super-periods each lane walks (mono kernels: both halves of
 * the run, 2 x the SPs a lane iterates); *tasks_per_mix = waves per mix (per
 * group of mixes for the several-mixes-per-wave layouts).  XM_ENOSYS when
 * this thread has launched no fused kernel (CPU handles never do).  The
 * environment variable XM_FAST_SPLIT_R=R forces R (rounded up to what the
 * layout needs) so that small batches exercise the cross-SP paths. */
XM_API int xm_audio_mixer_last_fast_split(int *sp_per_lane, int *tasks_per_mix);

#ifdef __cplusplus
}
#endif
#endif /* XM_AUDIO_MIXER_H */
